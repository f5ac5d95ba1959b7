#!/bin/bash
# Round 6: the coarse re-rank's locality order — parity, then c5 with / without it.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py -k "locality or c5 or c4_hnsw32" -x -q -m gpu --timeout 600 --timeout-method thread > gpurun_out/r6g_suite.log 2>&1
rc=$?; tail -2 gpurun_out/r6g_suite.log; [ $rc -eq 0 ] || exit $rc
for v in on off; do
  E=""; [ $v = off ] && E="FAISS_AMD_CRERANK_ORDER=0"
  env $E timeout -k 10 400 python -u bench.py --config c5 --shard-of 8 --steps 20 --warmup 2 --no-cpu-baseline --recall-queries 0 > gpurun_out/g_c5_$v.json 2> gpurun_out/g_c5_$v.err
  rc=$?; [ $rc -eq 0 ] || { echo "bench $v rc=$rc"; exit $rc; }
  python -c "import json;d=json.load(open('gpurun_out/g_c5_$v.json'));print('c5 $v', round(d['value']/1e6,3), round(d['ms_per_step'],4), [(k['name'],round(k['ms_per_step']*1e3,1)) for k in d['kernels']])"
done
if [ -n "$PMC" ]; then
  rm -rf gpurun_out/pmc[0-9]*
  PMC_KERNEL="k_coarse_rerank" PMC_BENCH_ARGS="--config c5 --shard-of 8" T_PMC=400 PMC_SETS="FETCH_SIZE" bash scripts/pmc_passes.sh > gpurun_out/g_pmc.txt 2>&1; tail -12 gpurun_out/g_pmc.txt
fi
