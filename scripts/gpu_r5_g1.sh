set -o pipefail
# PQ filter: snake static schedule — parity, c3/c5 traces, c3 A/B (snake vs stride), c5
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_configs.py tests/test_gpu_wide_nprobe.py tests/test_gpu_ref_fixtures.py -k "c3 or c5 or pq or preassigned" > gpurun_out/t_pq.log 2>&1 || { echo tests failed; exit 1; }
FAISS_AMD_PQ_TRACE=gpurun_out/pq_c3.trace timeout -k 10 200 python bench.py --config c3 --steps 3 --warmup 2 --no-cpu-baseline > gpurun_out/b_c3_tr.json 2> gpurun_out/b_c3_tr.err || { echo c3 trace failed; exit 1; }
timeout -k 10 200 python bench.py --config c3 --steps 50 --warmup 3 --no-cpu-baseline > gpurun_out/b_c3.json 2> gpurun_out/b_c3.err || { echo c3 failed; exit 1; }
FAISS_AMD_PQ_SCHED=stride timeout -k 10 200 python bench.py --config c3 --steps 50 --warmup 3 --no-cpu-baseline > gpurun_out/b_c3s.json 2> gpurun_out/b_c3s.err || { echo c3s failed; exit 1; }
timeout -k 10 350 python bench.py --config c5 --shard-of 8 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/b_c5.json 2> gpurun_out/b_c5.err || { echo c5 failed; exit 1; }
FAISS_AMD_PQ_TRACE=gpurun_out/pq_c5.trace timeout -k 10 350 python bench.py --config c5 --shard-of 8 --steps 2 --warmup 2 --no-cpu-baseline > gpurun_out/b_c5_tr.json 2> gpurun_out/b_c5_tr.err
