#!/bin/bash
# stream filter ping-pong buffers vs the previous build at the C5 shape (D=256, one chunk
# per group) and C2 size
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out; export PYTHONDONTWRITEBYTECODE=1
for cfg in "8800000 256" "100000 768"; do set -- $cfg
for nq in 1 8 64; do
timeout -k 10 300 python -u scripts/ab_libs.py --n $1 --dim $2 --queries $nq --rounds 40 \
  --libs rag-cobweb_amd/libcwq_base.so --libs rag-cobweb_amd/libcwq.so > gpurun_out/ab8_$1_$2_$nq.log 2>&1 || exit $?
echo "n=$1 d=$2 nq=$nq"; grep -v amdgpu gpurun_out/ab8_$1_$2_$nq.log | tail -2
done; done
