#!/bin/bash
# Per-query / per-item wave traces of one config (re-rank, coarse re-rank,
# filter), summarised on the box.   CFG=c2 bash scripts/gpu_traces.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
CFG=${CFG:-c2}
FAISS_AMD_RERANK_TRACE=gpurun_out/rtrace_$CFG.bin FAISS_AMD_CRERANK_TRACE=gpurun_out/crtrace_$CFG.bin \
FAISS_AMD_FILTER_TRACE=gpurun_out/ftrace_$CFG.bin \
  timeout -k 10 300 python bench.py --config $CFG --steps 3 --warmup 1 --no-cpu-baseline --recall-queries 0 \
  > gpurun_out/trace_$CFG.json 2> gpurun_out/trace_$CFG.err || exit $?
for f in rtrace crtrace; do
  [ -f gpurun_out/${f}_$CFG.bin ] && python scripts/rtrace_summary.py gpurun_out/${f}_$CFG.bin > gpurun_out/${f}_$CFG.txt 2>&1
done
[ -f gpurun_out/ftrace_$CFG.bin ] && python scripts/ftrace_summary.py gpurun_out/ftrace_$CFG.bin > gpurun_out/ftrace_$CFG.txt 2>&1
exit 0
