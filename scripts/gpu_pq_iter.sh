#!/bin/bash
# IVF-PQ iteration: PQ parity tests, then c3 bench + per-step kernel list
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T="tests/test_gpu_ref_fixtures.py tests/test_gpu_golden.py tests/test_gpu_pq_hnsw_io.py tests/test_gpu_configs.py tests/test_gpu_max_codes.py tests/test_gpu_idselector.py"
timeout -k 10 500 python -u -m pytest $T -k "${TK:-pq or c3 or c5}" -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pq_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -15 gpurun_out/pq_tests.log; [ "$rc" -eq 0 ] || exit $rc
CFG=${CFG:-c3}
timeout -k 10 300 python bench.py --config $CFG --steps 50 --warmup 3 --no-cpu-baseline --recall-queries 200 > gpurun_out/bench_$CFG.json 2> gpurun_out/bench_$CFG.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_$CFG.json; tail -2 gpurun_out/bench_$CFG.err; [ "$rc" -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$CFG -o run --output-format csv -- python bench.py --config $CFG --steps 5 --warmup 1 --no-cpu-baseline --recall-queries 0 > gpurun_out/prof_$CFG.log 2>&1
rc=$?; echo "rocprof rc=$rc"; [ "$rc" -eq 0 ] || exit $rc
python scripts/step_kernels.py gpurun_out/prof_$CFG 2>&1 | tail -14
