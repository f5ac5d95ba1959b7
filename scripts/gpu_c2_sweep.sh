# c2 coarse split-count sweep (FAISS_AMD_COARSE_NSPLIT) and bucket-scan E
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for ns in 0 4 8 12 16; do
  if [ $ns = 0 ]; then unset FAISS_AMD_COARSE_NSPLIT; else export FAISS_AMD_COARSE_NSPLIT=$ns; fi
  timeout -k 10 200 python bench.py --config c2 --steps 200 --warmup 3 --no-cpu-baseline > gpurun_out/sw_ns$ns.json 2>/dev/null || exit 1
done
unset FAISS_AMD_COARSE_NSPLIT
for e in 4 8 16; do
  FAISS_AMD_SCAN_E=$e timeout -k 10 200 python bench.py --config c2 --steps 200 --warmup 3 --no-cpu-baseline > gpurun_out/sw_e$e.json 2>/dev/null || exit 1
done
