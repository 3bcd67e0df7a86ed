#!/bin/bash
# select/tighten: empty lists filled by a wave-wide bitonic sort; GPU tests, then
# in-process A/B vs the previous build (batch C3 and per-call)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out; export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pyt_ab11.log 2>&1; rc=$?; tail -3 gpurun_out/pyt_ab11.log; [ $rc -eq 0 ] || exit $rc
for cfg in "1000000 768 10000 8" "1000000 768 1 40" "1000000 768 64 40" "100000 768 1 40"; do set -- $cfg
timeout -k 10 300 python -u scripts/ab_libs.py --n $1 --dim $2 --queries $3 --rounds $4 \
  --libs rag-cobweb_amd/libcwq_base.so --libs rag-cobweb_amd/libcwq.so > gpurun_out/ab11_$1_$3.log 2>&1 || exit $?
echo "n=$1 d=$2 nq=$3"; grep -v amdgpu gpurun_out/ab11_$1_$3.log | tail -2
done
