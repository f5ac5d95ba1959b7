#!/bin/bash
# c2 / c4 bench lines for the in-tree library and each ab_libs/*.so (re-rank A/B)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for L in default ab_libs/*.so; do
  n=$(basename $L .so)
  for c in c2 c4; do
    if [ "$L" = default ]; then E=""; else E="FAISS_AMD_LIB=$PWD/$L"; fi
    env $E timeout -k 10 300 python bench.py --config $c --steps 30 --warmup 3 --no-cpu-baseline --recall-queries 0 > gpurun_out/rr_${n}_$c.json 2> gpurun_out/rr_${n}_$c.err
    rc=$?; echo "$n $c rc=$rc"; [ "$rc" -eq 0 ] || exit $rc
    python -c "import json;d=json.load(open('gpurun_out/rr_${n}_$c.json'));print(round(d['ms_per_step'],4),[(k['name'],round(k['ms_per_step'],4)) for k in d['kernels']])"
  done
done
