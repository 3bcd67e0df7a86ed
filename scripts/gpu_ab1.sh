#!/bin/bash
# tests + smoke, then in-process A/Bs of the XCD split and the static priority knob, then the bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
bash scripts/gpu_check.sh tests || exit $?
timeout -k 10 400 python scripts/env_ab.py --rounds 5 \
  --variants "CWQ_FG_QG=8;CWQ_FG_QG=4;CWQ_FG_QG=2;CWQ_FG_DBG=512" > gpurun_out/env_ab1.log 2>&1 || exit $?
tail -6 gpurun_out/env_ab1.log
bash scripts/gpu_check.sh bench
# 2-rank rehearsal of the multi-GPU bench path on this one GPU (gloo over CUDA tensors)
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 --dist-backend gloo --preset c2 \
  --no-cpu-baseline --no-per-call --recall-queries 0 > gpurun_out/dist2_gloo.log 2>&1
echo "dist2 rc=$?"; tail -2 gpurun_out/dist2_gloo.log
