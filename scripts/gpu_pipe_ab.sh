#!/bin/bash
# c4 bench lines for several FAISS_AMD_HNSW_PIPE chunk counts (same box)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for P in ${PIPES:-1 2 4}; do
  FAISS_AMD_HNSW_PIPE=$P timeout -k 10 300 python bench.py --config c4 --steps 30 --warmup 3 --no-cpu-baseline --recall-queries 0 > gpurun_out/bench_c4_p$P.json 2> gpurun_out/bench_c4_p$P.err
  rc=$?; echo "bench c4 pipe $P rc=$rc"; [ "$rc" -eq 0 ] || exit $rc
  python -c "import json;d=json.load(open('gpurun_out/bench_c4_p$P.json'));print(d['value'],d['ms_per_step'],[(k['name'],round(k['ms_per_step'],3)) for k in d['kernels']])"
done
