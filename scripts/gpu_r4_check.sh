#!/bin/bash
# round-4 check: parity tests of the changed paths, then c3 / c4 bench lines
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T="tests/test_gpu_ref_fixtures.py tests/test_gpu_golden.py tests/test_gpu_pq_hnsw_io.py tests/test_gpu_configs.py tests/test_gpu_stats.py tests/test_c_harness.py"
timeout -k 10 ${T_TEST:-600} python -u -m pytest $T -k "${TK:-pq or c3 or c5 or hnsw or c4 or harness or nprobe_beyond}" -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/r4_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASSED|FAILED|ERROR" gpurun_out/r4_tests.log | tail -8; tail -3 gpurun_out/r4_tests.log; [ "$rc" -eq 0 ] || exit $rc
for cfg in ${CFGS:-c3 c4}; do
  timeout -k 10 300 python bench.py --config $cfg --steps 30 --warmup 3 --no-cpu-baseline --recall-queries 200 > gpurun_out/bench_$cfg.json 2> gpurun_out/bench_$cfg.err
  rc=$?; echo "bench $cfg rc=$rc"; python -c "import json;d=json.load(open('gpurun_out/bench_$cfg.json'));print(d['value'],d['ms_per_step'],d['config']['recall_at_10'],[(k['name'],round(k['ms_per_step'],3)) for k in d['kernels']])"; [ "$rc" -eq 0 ] || exit $rc
done
if [ -n "$C4B" ]; then
  FAISS_AMD_HNSW=batched timeout -k 10 300 python bench.py --config c4 --steps 30 --warmup 3 --no-cpu-baseline --recall-queries 0 > gpurun_out/bench_c4b.json 2> gpurun_out/bench_c4b.err
  rc=$?; echo "bench c4 batched rc=$rc"; python -c "import json;d=json.load(open('gpurun_out/bench_c4b.json'));print(d['value'],d['ms_per_step'],[(k['name'],round(k['ms_per_step'],3)) for k in d['kernels']])"
fi
