set -o pipefail
# A/B: non-temporal tile stream (Flat filter) / code loads (PQ filter) vs default
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for c in c2 c3; do
  timeout -k 10 200 python bench.py --config $c --steps 100 --warmup 3 --no-cpu-baseline > gpurun_out/ab_${c}_def.json 2>/dev/null || exit 1
  FAISS_AMD_LIB=$PWD/hnsw-ivf_amd/lib_ab/libfaiss_amd.so timeout -k 10 200 python bench.py --config $c --steps 100 --warmup 3 --no-cpu-baseline > gpurun_out/ab_${c}_nt.json 2>/dev/null || exit 1
done
timeout -k 10 300 python bench.py --config c5 --shard-of 8 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ab_c5_def.json 2>/dev/null || exit 1
FAISS_AMD_LIB=$PWD/hnsw-ivf_amd/lib_ab/libfaiss_amd.so timeout -k 10 300 python bench.py --config c5 --shard-of 8 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ab_c5_nt.json 2>/dev/null || exit 1
