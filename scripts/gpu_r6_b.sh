#!/bin/bash
# Round 6: the rest of the GPU suite, c2 bench lines (default and A/B libs), the c4 grid point.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "$TESTS" ]; then
timeout -k 10 700 python -u -m pytest $TESTS -v -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/r6b_suite.log 2>&1
rc=$?; echo "suite rc=$rc"; grep -E "passed|failed|error" gpurun_out/r6b_suite.log | tail -3
[ "$rc" -eq 0 ] || exit $rc
fi
for v in $LIBS; do
  if [ "$v" = default ]; then L=""; else L="hnsw-ivf_amd/lib/ab/libfaiss_amd_$v.so"; fi
  FAISS_AMD_LIB=$L timeout -k 10 300 python -u bench.py --steps 200 --warmup 5 --no-cpu-baseline > gpurun_out/r6_c2_$v.json 2> gpurun_out/r6_c2_$v.err
  rc=$?; echo "bench $v rc=$rc"; python -c "import json;d=json.load(open('gpurun_out/r6_c2_$v.json'));print(d['value'],d['ms_per_step'],[(k['name'],round(k['ms_per_step']*1e3,1)) for k in d['kernels']])"
  [ "$rc" -eq 0 ] || exit $rc
done
if [ -n "$C4GRID" ]; then
timeout -k 10 600 python -u bench.py --config c4 --nprobe 256 --efsearch 768 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r6_c4_np256_ef768.json 2> gpurun_out/r6_c4_np256_ef768.err
rc=$?; echo "bench c4 grid rc=$rc"; head -c 2500 gpurun_out/r6_c4_np256_ef768.json
fi
exit $rc
