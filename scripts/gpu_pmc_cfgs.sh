#!/bin/bash
# PMC passes (scripts/gpu_round.sh PMC=1) for the PQ configs; summaries kept
# per config as gpurun_out/pmc_<cfg>_summary.{txt,json}.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for c in ${CONFIGS:-c3 c5}; do
  extra=""; [ "$c" = c5 ] && extra="--shard-of 8"
  rm -rf gpurun_out/pmc1 gpurun_out/pmc2 gpurun_out/pmc3 gpurun_out/pmc4
  SKIP_TEST=1 SKIP_BENCH=1 PMC=1 PMC_KERNEL="ivfpq|coarse|rerank|query" PMC_BENCH_ARGS="--config $c $extra" bash scripts/gpu_round.sh > gpurun_out/pmc_$c.log 2>&1
  rc=$?; echo "pmc $c rc=$rc"; [ "$rc" -eq 0 ] || exit $rc
  cp gpurun_out/pmc_summary.txt gpurun_out/pmc_${c}_summary.txt
  cp gpurun_out/pmc_summary.json gpurun_out/pmc_${c}_summary.json
done
