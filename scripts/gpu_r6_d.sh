#!/bin/bash
# Round 6: HNSW parity (sequential-kernel paths), the c4 wide diag per library variant, PMC passes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${TESTS:-x}" != none ]; then
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_configs.py::test_c4_wide_hnsw_grid tests/test_gpu_ref_fixtures.py tests/test_gpu_golden.py} -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r6d_suite.log 2>&1
rc=$?; tail -2 gpurun_out/r6d_suite.log; [ $rc -eq 0 ] || exit $rc
fi
for v in ${LIBS:-default}; do
  if [ "$v" = default ]; then L=""; else L="hnsw-ivf_amd/lib/ab/libfaiss_amd_$v.so"; fi
  FAISS_AMD_LIB=$L timeout -k 10 400 python -u scripts/c4_wide_diag.py > gpurun_out/wdiag_$v.log 2>&1
  rc=$?; echo "== $v rc=$rc"; grep -v "flagged for the" gpurun_out/wdiag_$v.log; [ $rc -eq 0 ] || exit $rc
done
if [ -n "$PMC" ]; then bash scripts/gpu_wide_pmc.sh; fi
