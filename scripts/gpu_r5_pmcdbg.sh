# one PMC pass on c3's PQ filter with its log kept
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
rm -rf gpurun_out/pmcdbg
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "ivfpq" --output-format csv -d gpurun_out/pmcdbg -o pmc -- python bench.py --config c3 --steps 2 --warmup 1 --no-cpu-baseline --recall-queries 0 > gpurun_out/pmcdbg.log 2>&1
echo "pmcdbg rc=$?"
find gpurun_out/pmcdbg -name "*.csv" | head; f=$(find gpurun_out/pmcdbg -name "*counter_collection*.csv" | head -1); [ -n "$f" ] && cut -d, -f1-30 "$f" | grep -o "k_ivfpq[^(]*" | sort | uniq -c
