#!/bin/bash
# Round 6: the many-group bucket scan / 128 KB count ranges: parity (configs with 16384 / 65536 lists), then c5 and c4 bench lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_max_codes.py -x -q -m gpu --timeout 600 --timeout-method thread > gpurun_out/r6f_suite.log 2>&1
rc=$?; tail -2 gpurun_out/r6f_suite.log; [ $rc -eq 0 ] || exit $rc
for c in c5 c4; do
  extra=""; [ "$c" = c5 ] && extra="--shard-of 8"
  for v in new old; do
    E=""; [ $v = old ] && E="FAISS_AMD_SCAN_PAR=0 FAISS_AMD_BC_BIG=0"
    env $E timeout -k 10 400 python -u bench.py --config $c $extra --steps 20 --warmup 2 --no-cpu-baseline --recall-queries 0 > gpurun_out/f_${c}_$v.json 2> gpurun_out/f_${c}_$v.err
    rc=$?; [ $rc -eq 0 ] || { echo "bench $c $v rc=$rc"; exit $rc; }
    python -c "import json;d=json.load(open('gpurun_out/f_${c}_$v.json'));print('$c $v', round(d['value']/1e6,3), round(d['ms_per_step'],4), [(k['name'],round(k['ms_per_step']*1e3,1)) for k in d['kernels']])"
  done
done
