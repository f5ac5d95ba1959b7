#!/bin/bash
# PMC passes over one kernel of a short program: PROG (python args), KR (kernel regex)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-pmc}
i=0
for ctrs in "FETCH_SIZE" "WRITE_SIZE" \
    "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS" \
    "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAIT_INST_LDS"; do
  i=$((i+1))
  rm -rf gpurun_out/${TAG}_p$i
  timeout -s KILL ${T_PMC:-240} rocprofv3 --pmc $ctrs --kernel-include-regex "$KR" --output-format csv -d gpurun_out/${TAG}_p$i -o pmc -- python $PROG > gpurun_out/${TAG}_p$i.log 2>&1
  rc=$?; echo "pmc$i rc=$rc"; [ "$rc" -eq 0 ] || exit $rc
done
mkdir -p gpurun_out/${TAG}_all && for j in $(seq 1 $i); do cp -r gpurun_out/${TAG}_p$j gpurun_out/${TAG}_all/pmc$j; done
python scripts/pmc_summary.py gpurun_out/${TAG}_all gpurun_out/${TAG}_summary.json > gpurun_out/${TAG}_summary.txt 2>&1; cat gpurun_out/${TAG}_summary.txt
