#!/bin/bash
# Round 6: HNSW parity tests, then c4 grid points with the flag statistics.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TESTS=${TESTS:-"tests/test_gpu_configs.py::test_c4_wide_hnsw_grid tests/test_gpu_hnsw.py tests/test_ref_fixtures.py"}
if [ "$TESTS" != none ]; then
timeout -k 10 700 python -u -m pytest $TESTS -v -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/r6c_suite.log 2>&1
rc=$?; echo "suite rc=$rc"; grep -E "passed|failed|error" gpurun_out/r6c_suite.log | tail -3
[ "$rc" -eq 0 ] || exit $rc
fi
for pt in ${POINTS:-256:768 1024:1024}; do
  np=${pt%%:*}; ef=${pt##*:}
  FAISS_AMD_HNSW_STATS=${STATS:-1} timeout -k 10 300 python -u bench.py --config c4 --nprobe $np --efsearch $ef --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline > gpurun_out/r6_c4_np${np}_ef${ef}.json 2> gpurun_out/r6_c4_np${np}_ef${ef}.err
  rc=$?; echo "c4 np$np ef$ef rc=$rc"
  [ "$rc" -eq 0 ] || exit $rc
  python - <<PY
import json
d=json.load(open('gpurun_out/r6_c4_np${np}_ef${ef}.json'))
print(d['value'], d['ms_per_step'], d.get('recall'), [(k['name'], round(k['ms_per_step'],3)) for k in d['kernels']])
PY
  grep -m3 "flagged" gpurun_out/r6_c4_np${np}_ef${ef}.err
done
exit 0
