#!/bin/bash
# PMC passes of the wide HNSW kernel on c4's quantizer (scripts/c4_wide_diag.py, DIAG_PMC).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
SETS=${SETS:-"SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS;SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"}
rm -rf gpurun_out/pmc[0-9]*
i=0
IFS=';' read -ra ARR <<< "$SETS"
for ctrs in "${ARR[@]}"; do
  i=$((i+1))
  DIAG_PMC=1 POINTS=${POINTS:-256:768} timeout -s KILL ${T_PMC:-240} rocprofv3 --pmc $ctrs --kernel-include-regex "${PMC_KERNEL:-k_hnsw_wide|k_hnsw_exact}" --output-format csv -d gpurun_out/pmc$i -o pmc -- python scripts/c4_wide_diag.py > gpurun_out/pmc$i.log 2>&1
  rc=$?; echo "pmc$i ($ctrs) rc=$rc"; tail -1 gpurun_out/pmc$i.log; [ "$rc" -eq 0 ] || exit $rc
done
python scripts/pmc_summary.py gpurun_out gpurun_out/pmc_summary.json > gpurun_out/pmc_summary.txt 2>&1; cat gpurun_out/pmc_summary.txt
