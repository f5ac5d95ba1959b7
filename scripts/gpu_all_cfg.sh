#!/bin/bash
# Bench lines + rocprof kernel stats / per-step kernel lists for c1 c3 c4 c5
# (c5 as one rank's share of an 8-GPU run) on one GPU.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in ${CONFIGS:-c1 c3 c4 c5}; do
  extra=""; [ "$c" = c5 ] && extra="--shard-of 8"
  timeout -k 10 ${T_CFG:-600} python -u bench.py --config $c --steps ${BSTEPS:-20} --warmup 2 $extra > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err
  rc=$?; echo "bench $c rc=$rc"; cat gpurun_out/bench_$c.json; tail -2 gpurun_out/bench_$c.err
  [ "$rc" -eq 0 ] || exit $rc
  if [ -n "$PROF" ]; then
    rm -rf gpurun_out/prof_$c
    timeout -k 10 ${T_PROF:-600} rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$c -o run --output-format csv -- python bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline --recall-queries 0 $extra > gpurun_out/prof_$c.json 2> gpurun_out/prof_$c.err
    rc=$?; echo "rocprof $c rc=$rc"; [ "$rc" -eq 0 ] || exit $rc
    python scripts/step_kernels.py gpurun_out/prof_$c > gpurun_out/prof_${c}_step.txt 2>&1; cat gpurun_out/prof_${c}_step.txt
  fi
done
