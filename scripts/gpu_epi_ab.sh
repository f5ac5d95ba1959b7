set -o pipefail
# Flat filter epilogue by lane swap: parity + c2 / c1 / c4 bench + trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 500 python -u -m pytest -x -q --timeout 250 --timeout-method thread -m gpu tests/test_gpu_flat_ivf.py tests/test_gpu_configs.py tests/test_gpu_ref_fixtures.py tests/test_gpu_wide_nprobe.py tests/test_gpu_golden.py tests/test_gpu_idselector.py > gpurun_out/t_epi.log 2>&1 || { echo tests failed; exit 1; }
timeout -k 10 200 python bench.py --config c2 --steps 200 --warmup 3 --no-cpu-baseline > gpurun_out/epi_c2.json 2>/dev/null || exit 1
FAISS_AMD_FILTER_TRACE=gpurun_out/ft_c2.bin FAISS_AMD_GRAPH=0 timeout -k 10 200 python bench.py --config c2 --steps 3 --warmup 2 --no-cpu-baseline > /dev/null 2>&1 || exit 1
python scripts/ftrace_summary.py gpurun_out/ft_c2.bin > gpurun_out/ft_c2.txt 2>&1
