#!/bin/bash
# HNSW GPU parity tests, then the c4 quantizer diagnostics (tie flags,
# sequential-kernel hop phases)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T="tests/test_gpu_ref_fixtures.py tests/test_gpu_pq_hnsw_io.py tests/test_gpu_golden.py tests/test_gpu_stats.py tests/test_gpu_configs.py"
timeout -k 10 400 python -u -m pytest $T -k "hnsw or c4" -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/hnsw_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/hnsw_tests.log; [ "$rc" -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/c4_hnsw_diag.py > gpurun_out/c4diag.log 2>&1
rc=$?; echo "diag rc=$rc"; grep -v "^\[faiss_amd\] hnsw: 0 of" gpurun_out/c4diag.log | tail -30; exit $rc
