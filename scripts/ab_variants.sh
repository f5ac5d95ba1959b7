#!/bin/bash
# A/B of library variants and env settings on one GPU: per variant a short
# rocprofv3 kernel trace of bench.py (c2 unless CFG is set) and its per-step
# kernel list.  VARIANTS="name:libpath:ENV=val,ENV2=val ..." (libpath may be
# empty = the in-tree library).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in $VARIANTS; do
  name=${v%%:*}; rest=${v#*:}; lib=${rest%%:*}; envs=${rest#*:}
  envargs=$(echo "$envs" | tr ',' ' ')
  rm -rf gpurun_out/ab_$name
  env $envargs ${lib:+FAISS_AMD_LIB=$PWD/$lib} timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ab_$name -o run --output-format csv -- python bench.py --config ${CFG:-c2} --steps ${STEPS:-20} --warmup 2 --no-cpu-baseline --recall-queries 0 ${AB_ARGS:-} > gpurun_out/ab_$name.json 2> gpurun_out/ab_$name.err
  rc=$?; echo "== $name rc=$rc $(python -c "import json;d=json.load(open('gpurun_out/ab_$name.json'));print(d['value'],d['ms_per_step'])" 2>/dev/null)"
  [ "$rc" -eq 0 ] || exit $rc
  python scripts/step_kernels.py gpurun_out/ab_$name 2>&1 | tail -12
  python - gpurun_out/ab_$name <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if int(r["Calls"]) >= 10:
        print(f"  avg {float(r['AverageNs'])/1e3:8.1f} us x{r['Calls']:>4}  {r['Name'][:80]}")
PY
done
