#!/bin/bash
# stream filter with ping-pong register buffers: parity tests on the new product build,
# then per-call A/B against the previous build (libcwq_base.so) at C3 and D=384 shapes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out; export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 500 python -u -m pytest tests/test_gpu_smallbatch.py tests/test_gpu_edges.py tests/test_gpu_configs.py tests/test_gpu_filter.py -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pyt_ab7.log 2>&1; rc=$?; tail -3 gpurun_out/pyt_ab7.log; [ $rc -eq 0 ] || exit $rc
for cfg in "1000000 768" "200000 384" "1000000 1024"; do set -- $cfg
for nq in 1 8 64; do
timeout -k 10 300 python -u scripts/ab_libs.py --n $1 --dim $2 --queries $nq --rounds 40 \
  --libs rag-cobweb_amd/libcwq_base.so --libs rag-cobweb_amd/libcwq.so > gpurun_out/ab7_$1_$2_$nq.log 2>&1 || exit $?
echo "n=$1 d=$2 nq=$nq"; grep -v amdgpu gpurun_out/ab7_$1_$2_$nq.log | tail -2
done; done
