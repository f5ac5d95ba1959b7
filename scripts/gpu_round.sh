#!/bin/bash
# One GPU session: parity tests, smoke, bench, rocprof summary.
# Stops at the first fault / abort / timeout (rc not in {0,1}).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
PYTEST_ARGS=${PYTEST_ARGS:-"tests -v -m gpu -x --timeout 300 --timeout-method thread"}
if [ -z "$SKIP_TEST" ]; then
timeout -k 10 ${T_TEST:-900} python -u -m pytest $PYTEST_ARGS > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log; ok $rc || exit $rc
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log; ok $rc || exit $rc
fi
if [ -z "$SKIP_BENCH" ]; then
timeout -k 10 ${T_BENCH:-600} python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench.json; tail -3 gpurun_out/bench.err; ok $rc || exit $rc
fi
if [ -n "$PROFILE" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline --recall-queries 0 > gpurun_out/prof.log 2>&1
  rc=$?; echo "rocprof rc=$rc"; ok $rc || exit $rc
  find gpurun_out/prof -name "*stats*" | head
fi
if [ -n "$PMC" ]; then
  BA="--steps 2 --warmup 1 --no-cpu-baseline --recall-queries 0 ${PMC_BENCH_ARGS:-}"
  KR=${PMC_KERNEL:-ivf}
  i=0
  for ctrs in "FETCH_SIZE" "WRITE_SIZE" \
      "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS" \
      "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAIT_INST_LDS"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $ctrs --kernel-include-regex "$KR" --output-format csv -d gpurun_out/pmc$i -o pmc -- python bench.py $BA > gpurun_out/pmc$i.log 2>&1
    rc=$?; echo "pmc$i rc=$rc"; ok $rc || exit $rc
  done
  python scripts/pmc_summary.py gpurun_out gpurun_out/pmc_summary.json > gpurun_out/pmc_summary.txt 2>&1; cat gpurun_out/pmc_summary.txt
fi
exit 0
