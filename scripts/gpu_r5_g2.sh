set -o pipefail
# c3 bench line (this round's PMC summary committed) and the c4 grid point
timeout -k 10 300 python -u bench.py --config c3 > gpurun_out/r05_c3_bench.json 2> gpurun_out/r05_c3_bench.err || { echo c3 failed; exit 1; }
timeout -k 10 600 python -u bench.py --config c4 --nprobe 256 --efsearch 768 --steps 10 --warmup 2 > gpurun_out/r05_c4_np256_ef768_bench.json 2> gpurun_out/r05_c4_np256_ef768_bench.err || { echo c4 grid failed; exit 1; }
