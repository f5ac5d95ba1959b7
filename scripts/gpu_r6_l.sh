#!/bin/bash
# Round 6: c5's rocprof kernel trace again (the step window now stops before the bench's host-buffer calls).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=c5; rm -rf gpurun_out/prof_$tag
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$tag -o run --output-format csv -- python bench.py --config c5 --shard-of 8 --steps 5 --warmup 1 --no-cpu-baseline --recall-queries 0 > gpurun_out/prof_$tag.json 2> gpurun_out/prof_$tag.err
rc=$?; echo "rocprof $tag rc=$rc"; [ "$rc" -eq 0 ] || exit $rc
f=$(find gpurun_out/prof_$tag -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/r06_${tag}_kernel_stats_all.csv
python scripts/step_kernels.py gpurun_out/prof_$tag --window-stats gpurun_out/r06_${tag}_kernel_stats.csv > gpurun_out/r06_${tag}_step_kernels.txt 2>&1; cat gpurun_out/r06_${tag}_step_kernels.txt
rm -rf gpurun_out/prof_$tag
