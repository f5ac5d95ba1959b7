set -o pipefail
# A/B: coarse filter with two accumulator chains (lib_ab) vs default
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
AB=$PWD/hnsw-ivf_amd/lib_ab/libfaiss_amd.so
FAISS_AMD_LIB=$AB timeout -k 10 400 python -u -m pytest -x -q --timeout 250 --timeout-method thread -m gpu tests/test_gpu_flat_ivf.py tests/test_gpu_configs.py -k "coarse or c5_ivf or c2 or c1" > gpurun_out/t_split.log 2>&1 || { echo tests failed; exit 1; }
for c in c2; do
  timeout -k 10 200 python bench.py --config $c --steps 200 --warmup 3 --no-cpu-baseline > gpurun_out/sab_${c}_def.json 2>/dev/null || exit 1
  FAISS_AMD_LIB=$AB timeout -k 10 200 python bench.py --config $c --steps 200 --warmup 3 --no-cpu-baseline > gpurun_out/sab_${c}_ab.json 2>/dev/null || exit 1
done
timeout -k 10 300 python bench.py --config c5 --shard-of 8 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/sab_c5_def.json 2>/dev/null || exit 1
FAISS_AMD_LIB=$AB timeout -k 10 300 python bench.py --config c5 --shard-of 8 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/sab_c5_ab.json 2>/dev/null || exit 1
