#!/bin/bash
# Bench lines for the other BASELINE.json configs (c1, c3, c4) on one GPU.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for c in ${CONFIGS:-c1 c3 c4}; do
  timeout -k 10 ${T_CFG:-900} python -u bench.py --config $c --steps 10 --warmup 2 ${CFG_ARGS:-} > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err
  rc=$?; echo "bench $c rc=$rc"; cat gpurun_out/bench_$c.json; tail -2 gpurun_out/bench_$c.err
  [ "$rc" -eq 0 ] || exit $rc
done
