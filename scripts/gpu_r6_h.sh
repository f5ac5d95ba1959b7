#!/bin/bash
# Round 6: the sequential kernel without the result heap — parity, then the c4 grid points and the wide diag.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_pq_hnsw_io.py tests/test_gpu_ref_fixtures.py tests/test_gpu_configs.py -k "hnsw or c4 or ref" -x -q -m gpu --timeout 600 --timeout-method thread > gpurun_out/r6h_suite.log 2>&1
rc=$?; tail -3 gpurun_out/r6h_suite.log; [ $rc -eq 0 ] || exit $rc
for pt in 256:768 1024:1024; do
  np=${pt%%:*}; ef=${pt##*:}
  for v in new old; do
    E=""; [ $v = old ] && E="FAISS_AMD_HNSW_NORB=0"
    env $E timeout -k 10 300 python -u bench.py --config c4 --nprobe $np --efsearch $ef --steps 10 --warmup 2 --no-cpu-baseline --recall-queries 0 > gpurun_out/h_c4_${np}_$v.json 2> gpurun_out/h_c4_${np}_$v.err
    rc=$?; [ $rc -eq 0 ] || { echo "bench $pt $v rc=$rc"; exit $rc; }
    python -c "import json;d=json.load(open('gpurun_out/h_c4_${np}_$v.json'));print('c4 $pt $v', round(d['value']/1e3,1), round(d['ms_per_step'],3), [(k['name'],round(k['ms_per_step'],3)) for k in d['kernels']])"
  done
done
