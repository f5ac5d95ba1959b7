#!/bin/bash
# Multi-rank bench rehearsal on a one-GPU box: 2 ranks over gloo (RCCL
# refuses two ranks on one device).  Replicas + rccl_shards figure (c1), the
# --shard form (c1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp FAISS_AMD_BENCH_BACKEND=gloo
for extra in "" "--shard"; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --config ${CFG:-c1} --steps 20 \
    --warmup 3 $extra > gpurun_out/rehearse$extra.json 2> gpurun_out/rehearse$extra.err
  rc=$?; echo "rehearse '$extra' rc=$rc"; cat gpurun_out/rehearse$extra.json; tail -3 gpurun_out/rehearse$extra.err
  [ $rc -eq 0 ] || exit $rc
done
