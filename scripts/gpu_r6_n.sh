#!/bin/bash
# Round 6: keys per filter stream (FAISS_AMD_IVF_KT) on c4 / c2 / c3 — stats, step times, parity.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in c4 c2 c3; do
  for kt in 4 8; do
    FAISS_AMD_IVF_KT=$kt timeout -k 10 300 python -u bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline --recall-queries 0 > gpurun_out/n_${c}_$kt.json 2> gpurun_out/n_${c}_$kt.err
    rc=$?; [ $rc -eq 0 ] || { echo "bench $c $kt rc=$rc"; tail -3 gpurun_out/n_${c}_$kt.err; exit $rc; }
    python -c "import json;d=json.load(open('gpurun_out/n_${c}_$kt.json'));print('$c KT=$kt', round(d['value']/1e6,3), round(d['ms_per_step'],4), [(k['name'],round(k['ms_per_step'],3)) for k in d['kernels']])"
  done
done
FAISS_AMD_IVF_KT=8 FAISS_AMD_IVF_STATS=1 timeout -k 10 300 python -u bench.py --config c4 --steps 1 --warmup 1 --no-cpu-baseline --recall-queries 0 > gpurun_out/n_c4_st.json 2> gpurun_out/n_c4_st.err || exit 1
grep "ivf mfma scan" gpurun_out/n_c4_st.err | tail -1
FAISS_AMD_IVF_KT=8 timeout -k 10 500 python -u -m pytest tests/test_gpu_configs.py -k "c2 or c3 or c4_hnsw32 or c4_full_10m" -x -q -m gpu --timeout 400 --timeout-method thread > gpurun_out/r6n_parity.log 2>&1
rc=$?; tail -2 gpurun_out/r6n_parity.log; exit $rc
