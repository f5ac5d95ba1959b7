cd $GRAFT_REPO_ROOT
for m in 0 3 4 5; do
  FAISS_AMD_RERANK_DEBUG=$m timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/rr$m -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline --recall-queries 0 > gpurun_out/rr$m.log 2>&1 || exit 1
done
