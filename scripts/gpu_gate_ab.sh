#!/bin/bash
# A/B of the wave-gated queue pushes (lib/ab/libfaiss_amd_gate.so): parity, then c2 / c3 / c5 bench lines per library.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
G=hnsw-ivf_amd/lib/ab/libfaiss_amd_gate.so
FAISS_AMD_LIB=$G timeout -k 10 600 python -u -m pytest tests/test_gpu_golden.py tests/test_gpu_ref_fixtures.py tests/test_gpu_wide_nprobe.py tests/test_gpu_idselector.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/gate_suite.log 2>&1
rc=$?; tail -2 gpurun_out/gate_suite.log; [ $rc -eq 0 ] || exit $rc
for c in ${CFGS:-c2 c3 c5}; do
  extra=""; st="--steps 200 --warmup 5"
  [ "$c" = c5 ] && { extra="--shard-of 8"; st="--steps 20 --warmup 2"; }
  for v in default gate; do
    L=""; [ $v = gate ] && L=$G
    FAISS_AMD_LIB=$L timeout -k 10 400 python -u bench.py --config $c $extra $st --no-cpu-baseline --recall-queries 0 > gpurun_out/gate_${c}_$v.json 2> gpurun_out/gate_${c}_$v.err
    rc=$?; [ $rc -eq 0 ] || { echo "bench $c $v rc=$rc"; exit $rc; }
    python -c "import json;d=json.load(open('gpurun_out/gate_${c}_$v.json'));print('$c $v', round(d['value']/1e6,3), round(d['ms_per_step'],4), [(k['name'],round(k['ms_per_step']*1e3,1)) for k in d['kernels']])"
  done
done
