#!/bin/bash
# Round 6 validation: the arenas past 2^32 work-items, the C drop-in example,
# then the whole GPU parity suite and a short c2 bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_large_arena.py tests/test_ref_harness.py -v -m gpu -x --timeout 900 --timeout-method thread > gpurun_out/r6_large.log 2>&1
rc=$?; echo "large/harness rc=$rc"; grep -E "passed|failed|error" gpurun_out/r6_large.log | tail -3
[ "$rc" -eq 0 ] || exit $rc
if [ -n "$FULL" ]; then
timeout -k 10 600 python -u -m pytest tests -v -m gpu -x --timeout 300 --timeout-method thread --deselect tests/test_gpu_large_arena.py > gpurun_out/r6_suite.log 2>&1
rc=$?; echo "suite rc=$rc"; grep -E "passed|failed|error" gpurun_out/r6_suite.log | tail -3
[ "$rc" -eq 0 ] || exit $rc
fi
timeout -k 10 300 python -u bench.py --steps 100 --warmup 5 --no-cpu-baseline > gpurun_out/r6_c2.json 2> gpurun_out/r6_c2.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/r6_c2.json | head -c 3000
[ "$rc" -eq 0 ] || exit $rc
if [ -n "$C4GRID" ]; then
timeout -k 10 600 python -u bench.py --config c4 --nprobe 256 --efsearch 768 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r6_c4_np256_ef768.json 2> gpurun_out/r6_c4_np256_ef768.err
rc=$?; echo "bench c4 grid rc=$rc"; head -c 2500 gpurun_out/r6_c4_np256_ef768.json
fi
exit $rc
