#!/bin/bash
# A/B of the IVF-PQ filter forms on c3 (and c5 with C5=1): wave-independent
# (default) vs the 4-wave work-group form.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for f in w wg; do
  FAISS_AMD_PQ_FILTER=$f timeout -k 10 300 python -u bench.py --config c3 --steps 50 --warmup 3 --no-cpu-baseline --recall-queries 0 > gpurun_out/ab_pq_c3_$f.json 2> gpurun_out/ab_pq_c3_$f.err
  rc=$?; echo "c3 $f rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python -c "import json;d=json.load(open('gpurun_out/ab_pq_c3_$f.json'));print('c3 $f', round(d['ms_per_step'],4), [(k['name'],round(k['ms_per_step'],4)) for k in d['kernels']])"
done
