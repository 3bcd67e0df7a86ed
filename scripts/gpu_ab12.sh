#!/bin/bash
# sb_prep with the centre staged in LDS: GPU tests, then per-call A/B vs the previous build
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out; export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pyt_ab12.log 2>&1; rc=$?; tail -2 gpurun_out/pyt_ab12.log; [ $rc -eq 0 ] || exit $rc
for cfg in "1000000 768 1" "1000000 768 64" "100000 768 1" "100000 768 8"; do set -- $cfg
timeout -k 10 300 python -u scripts/ab_libs.py --n $1 --dim $2 --queries $3 --rounds 40 \
  --libs rag-cobweb_amd/libcwq_base.so --libs rag-cobweb_amd/libcwq.so > gpurun_out/ab12_$1_$3.log 2>&1 || exit $?
echo "n=$1 d=$2 nq=$3"; grep -v amdgpu gpurun_out/ab12_$1_$3.log | tail -2
done
