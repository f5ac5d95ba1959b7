#!/bin/bash
# Round 6: arrival-log re-runs gated at k <= 512 — HNSW parity, then the c4 grid evidence.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_pq_hnsw_io.py tests/test_gpu_ref_fixtures.py tests/test_gpu_configs.py -k "hnsw or c4 or ref" -x -q -m gpu --timeout 600 --timeout-method thread > gpurun_out/r6i_suite.log 2>&1
rc=$?; tail -3 gpurun_out/r6i_suite.log; [ $rc -eq 0 ] || exit $rc
CFGS="c4g256 c4g1024" bash scripts/gpu_r6_evidence.sh
