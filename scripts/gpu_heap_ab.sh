#!/bin/bash
# HNSW exact-kernel experiment: HNSW GPU tests on the in-tree library and on
# the -DHNSW_WAVE_HEAP build (ab_libs/libpar.so), then a c4 A/B of the two.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T="tests/test_gpu_ref_fixtures.py tests/test_gpu_pq_hnsw_io.py tests/test_gpu_golden.py tests/test_gpu_stats.py tests/test_gpu_configs.py"
timeout -k 10 400 python -u -m pytest $T -k hnsw -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/heap_default.log 2>&1
rc=$?; echo "default rc=$rc"; tail -3 gpurun_out/heap_default.log; [ "$rc" -eq 0 ] || exit $rc
FAISS_AMD_LIB=$PWD/ab_libs/libpar.so timeout -k 10 400 python -u -m pytest $T -k hnsw -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/heap_par.log 2>&1
rc=$?; echo "par rc=$rc"; tail -3 gpurun_out/heap_par.log; [ "$rc" -eq 0 ] || exit $rc
CFG=c4 STEPS=10 VARIANTS="par:ab_libs/libpar.so: default::" bash scripts/ab_variants.sh
