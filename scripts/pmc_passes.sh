#!/bin/bash
# PMC passes (one rocprofv3 run per counter set) for one kernel of a bench run.
#   PMC_KERNEL=<regex> PMC_BENCH_ARGS="--config c3" PMC_SETS="A B C;D E" bash scripts/pmc_passes.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
BA="--steps 2 --warmup 1 --no-cpu-baseline --recall-queries 0 ${PMC_BENCH_ARGS:-}"
SETS=${PMC_SETS:-"FETCH_SIZE;WRITE_SIZE"}
i=0
IFS=';' read -ra ARR <<< "$SETS"
for ctrs in "${ARR[@]}"; do
  i=$((i+1))
  timeout -s KILL ${T_PMC:-120} rocprofv3 --pmc $ctrs --kernel-include-regex "${PMC_KERNEL:-ivf}" --output-format csv -d gpurun_out/pmc$i -o pmc -- python bench.py $BA > gpurun_out/pmc$i.log 2>&1
  rc=$?; echo "pmc$i ($ctrs) rc=$rc"; [ "$rc" -eq 0 ] || exit $rc
done
python scripts/pmc_summary.py gpurun_out gpurun_out/pmc_summary.json > gpurun_out/pmc_summary.txt 2>&1; cat gpurun_out/pmc_summary.txt
