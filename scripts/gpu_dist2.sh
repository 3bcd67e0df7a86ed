#!/bin/bash
# 2-rank rehearsal of the multi-GPU bench path on one MI355X: gloo lets two ranks share the
# card (RCCL refuses that); the driver's N-GPU runs use "nccl" (RCCL) with one GPU per rank
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out; export PYTHONDONTWRITEBYTECODE=1
for preset in c3 c2; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 --dist-backend gloo --preset $preset \
    --no-cpu-baseline --no-per-call > gpurun_out/dist2_$preset.log 2>&1 || { tail -5 gpurun_out/dist2_$preset.log; exit 1; }
  tail -1 gpurun_out/dist2_$preset.log | cut -c1-400
done
