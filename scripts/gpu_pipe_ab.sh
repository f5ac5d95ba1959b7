#!/bin/bash
# FAISS_AMD_PIPE A/B on the bench configs (after the pipelined-batch parity test).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_pipe.py tests/test_gpu_search_graph.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pipe_suite.log 2>&1
rc=$?; tail -2 gpurun_out/pipe_suite.log; [ $rc -eq 0 ] || exit $rc
for c in ${CFGS:-c2 c3}; do
for P in ${PS:-1 2 3 4}; do
  FAISS_AMD_PIPE=$P timeout -k 10 300 python -u bench.py --config $c --steps 200 --warmup 5 --no-cpu-baseline --recall-queries 0 > gpurun_out/pipe_${c}_$P.json 2> gpurun_out/pipe_${c}_$P.err
  rc=$?; [ $rc -eq 0 ] || { echo "bench $c P=$P rc=$rc"; exit $rc; }
  python -c "import json;d=json.load(open('gpurun_out/pipe_${c}_$P.json'));print('$c P=$P', round(d['value']/1e6,3), round(d['ms_per_step'],4), [(k['name'],round(k['ms_per_step']*1e3,1)) for k in d['kernels']])"
done
done
