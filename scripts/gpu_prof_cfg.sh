#!/bin/bash
# rocprofv3 kernel trace + stats of a bench config; per-step kernel list.
#   CONFIGS="c3 c5" bash scripts/gpu_prof_cfg.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in ${CONFIGS:-c3}; do
  rm -rf gpurun_out/prof_$c
  timeout -k 10 ${T_PROF:-600} rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$c -o run --output-format csv -- python bench.py --config $c --steps ${PSTEPS:-5} --warmup 1 --no-cpu-baseline --recall-queries 0 > gpurun_out/prof_$c.json 2> gpurun_out/prof_$c.err
  rc=$?; echo "rocprof $c rc=$rc"; [ "$rc" -eq 0 ] || exit $rc
  python scripts/step_kernels.py gpurun_out/prof_$c ${MARKER:-} > gpurun_out/prof_${c}_step.txt 2>&1; tail -3 gpurun_out/prof_${c}_step.txt
done
