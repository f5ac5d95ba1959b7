set -o pipefail
# r05: folded PQ filter (shared positions) + coarse plan up to 32 splits — parity, traces, A/B
timeout -k 10 500 python -u -m pytest -x -v --timeout 250 --timeout-method thread -m gpu tests/test_gpu_flat_ivf.py tests/test_gpu_configs.py -k "coarse or c5 or c2 or c1" > gpurun_out/t_pq.log 2>&1 || { echo tests failed; exit 1; }
timeout -k 10 350 python bench.py --config c5 --shard-of 8 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/b_c5.json 2> gpurun_out/b_c5.err || { echo c5 failed; exit 1; }
FAISS_AMD_COARSE_WIDE=0 timeout -k 10 350 python bench.py --config c5 --shard-of 8 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/b_c5n.json 2> gpurun_out/b_c5n.err || { echo c5n failed; exit 1; }
FAISS_AMD_IVF_STATS=1 timeout -k 10 350 python bench.py --config c5 --shard-of 8 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/b_c5_st.json 2> gpurun_out/b_c5_st.err
