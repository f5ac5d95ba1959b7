#!/bin/bash
# Round-3 PMC summaries: c2 Flat filter, then c5 coarse + PQ filter (one shard).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
SETS="FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS;SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
PMC_KERNEL="ivf_bf2_stream" PMC_SETS="$SETS" bash scripts/pmc_passes.sh || exit $?
mkdir -p gpurun_out/r03_c2_pmc && mv gpurun_out/pmc[0-9]* gpurun_out/pmc_summary.* gpurun_out/r03_c2_pmc/
PMC_KERNEL="coarse_stream|ivfpq_filter" PMC_BENCH_ARGS="--config c5 --shard-of 8" T_PMC=300 PMC_SETS="$SETS" bash scripts/pmc_passes.sh || exit $?
mkdir -p gpurun_out/r03_c5_pmc && mv gpurun_out/pmc[0-9]* gpurun_out/pmc_summary.* gpurun_out/r03_c5_pmc/
