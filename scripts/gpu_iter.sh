#!/bin/bash
# Iteration loop on the GPU box: (optional) GPU tests, a short bench, and a
# rocprofv3 kernel-trace summary of a short bench.  Stops at the first
# failure that is not a plain test failure (rc 1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
CFG=${CFG:-c2}
if [ -n "$TESTS" ]; then
  timeout -k 10 ${T_TEST:-900} python -u -m pytest $TESTS -m gpu -q --timeout 600 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log; ok $rc || exit $rc
fi
timeout -k 10 600 python bench.py --config $CFG --steps ${STEPS:-50} --warmup 3 ${BENCH_ARGS:---no-cpu-baseline --recall-queries 0} > gpurun_out/bench_$CFG.json 2> gpurun_out/bench_$CFG.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_$CFG.json; tail -3 gpurun_out/bench_$CFG.err; ok $rc || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$CFG -o run --output-format csv -- python bench.py --config $CFG --steps 5 --warmup 1 --no-cpu-baseline --recall-queries 0 > gpurun_out/prof_$CFG.log 2>&1
rc=$?; echo "rocprof rc=$rc"; ok $rc || exit $rc
python scripts/step_kernels.py gpurun_out/prof_$CFG > gpurun_out/step_$CFG.txt 2>&1; cat gpurun_out/step_$CFG.txt
exit 0
