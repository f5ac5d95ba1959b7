#!/bin/bash
# Round-6 evidence per config: PMC passes of the dominant kernels (first, so
# the bench line's `traffic` reads this round's summary), the bench line
# (with the reference CPU baseline), then a rocprofv3 kernel trace + stats
# and the per-step kernel list.  Results under gpurun_out/r06_<tag>_*.
#   CFGS="c2 c3" bash scripts/gpu_r6_evidence.sh
#   CFGS="c4g256 c4g1024" bash scripts/gpu_r6_evidence.sh   (c4 grid points)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out profiles
export TMPDIR=/tmp
SETS="FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS;SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
for c in ${CFGS:-c1 c2 c3 c5 c4}; do
  args="--config $c"; tag=$c; steps=""
  case $c in
    c1|c2) KR="k_ivf_bf2_stream|k_ivf_rerank|k_coarse_stream|k_coarse_rerank" ;;
    c3) KR="k_ivfpq_filter_w|k_ivf_rerank|k_coarse_stream|k_coarse_rerank" ;;
    c4) KR="k_hnsw_exact_reg|k_ivf_bf2_stream|k_ivf_rerank" ;;
    c5) KR="k_coarse_stream|k_ivfpq_filter_w|k_ivf_rerank|k_coarse_rerank"; args="--config c5 --shard-of 8" ;;
    c4g256) KR="k_hnsw_wide|k_hnsw_exact|k_ivf_bf2_stream|k_ivf_rerank"; args="--config c4 --nprobe 256 --efsearch 768"; tag=c4_np256_ef768; steps="--steps 10 --warmup 2" ;;
    c4g1024) KR="k_hnsw_wide|k_hnsw_exact|k_ivf_bf2_stream|k_ivf_rerank"; args="--config c4 --nprobe 1024 --efsearch 1024"; tag=c4_np1024_ef1024; steps="--steps 10 --warmup 2" ;;
  esac
  if [ -z "$NO_PMC" ]; then
    rm -rf gpurun_out/pmc[0-9]*
    PMC_KERNEL="$KR" PMC_BENCH_ARGS="$args" T_PMC=${T_PMC:-400} PMC_SETS="$SETS" bash scripts/pmc_passes.sh > gpurun_out/r06_${tag}_pmc_run.txt 2>&1
    rc=$?; echo "pmc $tag rc=$rc"; [ "$rc" -eq 0 ] || exit $rc
    cp gpurun_out/pmc_summary.json gpurun_out/r06_${tag}_pmc.json
    cp gpurun_out/pmc_summary.txt gpurun_out/r06_${tag}_pmc_summary.txt
    cp gpurun_out/pmc_summary.json profiles/r06_${tag}_pmc.json
    rm -rf gpurun_out/pmc[0-9]*
  fi
  timeout -k 10 ${T_CFG:-600} python -u bench.py $args $steps ${BARGS:-} > gpurun_out/r06_${tag}_bench.json 2> gpurun_out/r06_${tag}_bench.err
  rc=$?; echo "bench $tag rc=$rc"; [ "$rc" -eq 0 ] || exit $rc
  python -c "import json;d=json.load(open('gpurun_out/r06_${tag}_bench.json'));print(d['value'],d['ms_per_step'],d['roofline'].get('frac'),d['roofline'].get('traffic'),d['cpu_baseline']['value'] if d.get('cpu_baseline') else None,[(k['name'],round(k['ms_per_step'],3)) for k in d['kernels']])"
  if [ -z "$NO_PROF" ]; then
  rm -rf gpurun_out/prof_$tag
  timeout -k 10 ${T_PROF:-600} rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$tag -o run --output-format csv -- python bench.py $args --steps 5 --warmup 1 --no-cpu-baseline --recall-queries 0 > gpurun_out/prof_$tag.json 2> gpurun_out/prof_$tag.err
  rc=$?; echo "rocprof $tag rc=$rc"; [ "$rc" -eq 0 ] || exit $rc
  f=$(find gpurun_out/prof_$tag -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/r06_${tag}_kernel_stats_all.csv
  python scripts/step_kernels.py gpurun_out/prof_$tag --window-stats gpurun_out/r06_${tag}_kernel_stats.csv > gpurun_out/r06_${tag}_step_kernels.txt 2>&1; tail -1 gpurun_out/r06_${tag}_step_kernels.txt
  rm -rf gpurun_out/prof_$tag
  fi
done
