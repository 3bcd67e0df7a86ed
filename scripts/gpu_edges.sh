#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out; export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_edges.py -m gpu -v -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pyt_edges.log 2>&1; rc=$?; tail -15 gpurun_out/pyt_edges.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
# 2-rank rehearsal of the multi-GPU bench path on this one GPU (gloo over CUDA tensors)
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 --dist-backend gloo --preset c2 \
  --no-cpu-baseline --no-per-call --recall-queries 0 > gpurun_out/dist2_gloo.log 2>&1
echo "dist2 rc=$?"; tail -2 gpurun_out/dist2_gloo.log
