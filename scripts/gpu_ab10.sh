#!/bin/bash
# stream filter, one-query-block instantiation at 4 waves per SIMD (2 workgroups per CU)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out; export PYTHONDONTWRITEBYTECODE=1
for cfg in "1000000 768" "8800000 256"; do set -- $cfg
for nq in 1 16; do
timeout -k 10 300 python -u scripts/ab_libs.py --n $1 --dim $2 --queries $nq --rounds 40 \
  --libs rag-cobweb_amd/libcwq.so --libs rag-cobweb_amd/libcwq_w4.so > gpurun_out/ab10_$1_$2_$nq.log 2>&1 || exit $?
echo "n=$1 d=$2 nq=$nq"; grep -v amdgpu gpurun_out/ab10_$1_$2_$nq.log | tail -2
done; done
