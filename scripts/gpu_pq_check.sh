set -o pipefail
# PQ filter parity (configs, fixtures, selectors, wide nprobe) + c3 / c5 bench lines
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 500 python -u -m pytest -x -q --timeout 250 --timeout-method thread -m gpu tests/test_gpu_configs.py tests/test_gpu_wide_nprobe.py tests/test_gpu_ref_fixtures.py tests/test_gpu_idselector.py tests/test_gpu_pq_hnsw_io.py tests/test_gpu_search_graph.py -k "c3 or c5 or pq or PQ or preassigned or sel or graph" > gpurun_out/t_pq.log 2>&1 || { echo tests failed; exit 1; }
timeout -k 10 200 python bench.py --config c3 --steps 100 --warmup 3 --no-cpu-baseline > gpurun_out/b_c3.json 2> gpurun_out/b_c3.err || { echo c3 failed; exit 1; }
timeout -k 10 350 python bench.py --config c5 --shard-of 8 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/b_c5.json 2> gpurun_out/b_c5.err || { echo c5 failed; exit 1; }
