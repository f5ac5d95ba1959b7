#!/bin/bash
# HBM traffic (FETCH_SIZE / WRITE_SIZE, separate passes) + SQ activity of the
# dominant kernel of each config -> gpurun_out/pmc_<cfg>/pmc_summary.{txt,json}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for spec in ${PMC_SPECS:-c2:k_ivf_bf3_filter c3:k_ivfpq_filter c5:k_ivfpq_filter}; do
  c=${spec%%:*}; k=${spec#*:}
  rm -rf gpurun_out/pmc_$c; mkdir -p gpurun_out/pmc_$c
  i=0
  for ctrs in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    timeout -s KILL ${T_PMC:-240} rocprofv3 --pmc $ctrs --kernel-include-regex "$k" --output-format csv -d gpurun_out/pmc_$c/pmc$i -o pmc -- python bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline --recall-queries 0 > gpurun_out/pmc_$c/pmc$i.log 2>&1
    rc=$?; echo "pmc $c $i rc=$rc"; [ "$rc" -eq 0 ] || exit $rc
  done
  python scripts/pmc_summary.py gpurun_out/pmc_$c gpurun_out/pmc_$c/pmc_summary.json > gpurun_out/pmc_$c/pmc_summary.txt 2>&1; cat gpurun_out/pmc_$c/pmc_summary.txt
done
