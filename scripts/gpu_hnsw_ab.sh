#!/bin/bash
# c4 quantizer diagnostics for the in-tree library and each ab_libs/*.so
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
export EFS=${EFS:-64}
rm -f gpurun_out/c4_centroids.npy
timeout -k 10 200 python -u scripts/c4_hnsw_diag.py > gpurun_out/diag_default.log 2>&1
rc=$?; echo "== default rc=$rc"; grep -v "^\[faiss_amd\]" gpurun_out/diag_default.log | tail -6; [ "$rc" -eq 0 ] || exit $rc
if [ -n "$ENVAB" ]; then
  env $ENVAB timeout -k 10 200 python -u scripts/c4_hnsw_diag.py > gpurun_out/diag_env.log 2>&1
  rc=$?; echo "== $ENVAB rc=$rc"; grep -v "^\[faiss_amd\]" gpurun_out/diag_env.log | tail -6; [ "$rc" -eq 0 ] || exit $rc
fi
for L in ab_libs/*.so; do
  n=$(basename $L .so)
  FAISS_AMD_LIB=$PWD/$L timeout -k 10 200 python -u scripts/c4_hnsw_diag.py > gpurun_out/diag_$n.log 2>&1
  rc=$?; echo "== $n rc=$rc"; grep -v "^\[faiss_amd\]" gpurun_out/diag_$n.log | tail -6; [ "$rc" -eq 0 ] || exit $rc
done
