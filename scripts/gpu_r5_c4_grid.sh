set -o pipefail
# c4 grid point (nprobe 256 / efSearch 768): PMC passes of its kernels, then its bench line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
rm -rf gpurun_out/pmc[0-9]* gpurun_out/pmcdbg
SETS="FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS"
PMC_KERNEL="k_hnsw_exact|k_ivf_bf2_stream|k_ivf_rerank" PMC_BENCH_ARGS="--config c4 --nprobe 256 --efsearch 768" T_PMC=400 PMC_SETS="$SETS" bash scripts/pmc_passes.sh > gpurun_out/r05_c4_np256_ef768_pmc_run.txt 2>&1 || { echo pmc failed; exit 1; }
cp gpurun_out/pmc_summary.json profiles/r05_c4_np256_ef768_pmc.json
cp gpurun_out/pmc_summary.txt gpurun_out/r05_c4_np256_ef768_pmc_summary.txt
rm -rf gpurun_out/pmc[0-9]*
timeout -k 10 600 python -u bench.py --config c4 --nprobe 256 --efsearch 768 --steps 10 --warmup 2 > gpurun_out/r05_c4_np256_ef768_bench.json 2> gpurun_out/r05_c4_np256_ef768_bench.err || { echo c4 grid failed; exit 1; }
