#!/bin/bash
# Round 6: paged host-buffer search — parity tests, the Python-composed
# experiment, then c2's PCIe-inclusive rate at several page counts.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_host_pages.py tests/test_gpu_interrupt.py tests/test_gpu_stats.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r6j_suite.log 2>&1
rc=$?; tail -5 gpurun_out/r6j_suite.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/exp_host_pages.py > gpurun_out/host_pages.txt 2>&1
rc=$?; cat gpurun_out/host_pages.txt; [ $rc -eq 0 ] || exit $rc
for P in default 1 2 3 8; do
  E=""; [ $P = default ] || E="FAISS_AMD_HOST_PAGES=$P"
  env $E timeout -k 10 300 python -u bench.py --config c2 --steps 20 --warmup 5 --no-cpu-baseline --recall-queries 0 > gpurun_out/j_c2_$P.json 2> gpurun_out/j_c2_$P.err
  rc=$?; [ $rc -eq 0 ] || { echo "bench pages $P rc=$rc"; exit $rc; }
  python -c "import json;d=json.load(open('gpurun_out/j_c2_$P.json'));print('c2 pages $P', round(d['value']/1e6,2), round(d['ms_per_step'],4), d['pcie_inclusive'])"
done
