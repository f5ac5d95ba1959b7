#!/bin/bash
# Round 6: flagged HNSW queries searched again inside the wide kernel
# (FAISS_AMD_HNSW_INPLACE=1) — parity, then the c4 grid points both ways.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_pq_hnsw_io.py -k "wide_edges" -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r6m_edges.log 2>&1
rc=$?; tail -3 gpurun_out/r6m_edges.log; [ $rc -eq 0 ] || exit $rc
FAISS_AMD_HNSW_INPLACE=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_ref_fixtures.py -k "c4 or hnsw" -x -q -m gpu --timeout 500 --timeout-method thread > gpurun_out/r6m_c4.log 2>&1
rc=$?; tail -3 gpurun_out/r6m_c4.log; [ $rc -eq 0 ] || exit $rc
for pt in 256:768 1024:1024; do
  np=${pt%%:*}; ef=${pt##*:}
  for v in 1 0; do
    FAISS_AMD_HNSW_INPLACE=$v timeout -k 10 300 python -u bench.py --config c4 --nprobe $np --efsearch $ef --steps 10 --warmup 2 --no-cpu-baseline --recall-queries 0 > gpurun_out/m_c4_${np}_$v.json 2> gpurun_out/m_c4_${np}_$v.err
    rc=$?; [ $rc -eq 0 ] || { echo "bench $pt $v rc=$rc"; exit $rc; }
    python -c "import json;d=json.load(open('gpurun_out/m_c4_${np}_$v.json'));print('c4 $pt inplace=$v', round(d['value']/1e3,1), round(d['ms_per_step'],3), [(k['name'],round(k['ms_per_step'],3)) for k in d['kernels']])"
  done
done
