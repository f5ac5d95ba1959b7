#!/bin/bash
# IVF-PQ filter A/B: codes (default) / decode (k_ivfpq_filter_w) / image, c3 and c5
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for c in ${CFGS:-c3 c5}; do
  for f in codes decode image; do
    if [ "$f" = codes ]; then unset FAISS_AMD_PQ_FILTER; else export FAISS_AMD_PQ_FILTER=$f; fi
    timeout -k 10 400 python bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/ab_${c}_$f.json 2> gpurun_out/ab_${c}_$f.err || exit 1
    echo "$c $f $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_${c}_$f.json | head -1) $(grep -o '"name": "ivfpq_filter", "ms_per_step": [0-9.]*' gpurun_out/ab_${c}_$f.json)"
  done
done
