#!/bin/bash
# stream filter pretest: parity tests, then per-call A/B (pretest on / off) at C3, C2, C5 shapes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out; export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 500 python -u -m pytest tests/test_gpu_smallbatch.py tests/test_gpu_filter.py tests/test_gpu_edges.py tests/test_gpu_configs.py tests/test_gpu_parity.py -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pyt_ab6.log 2>&1; rc=$?; tail -3 gpurun_out/pyt_ab6.log; [ $rc -eq 0 ] || exit $rc
for cfg in "1000000 768" "100000 768" "8800000 256"; do set -- $cfg
for nq in 1 64; do
timeout -k 10 300 python -u scripts/env_ab.py --n $1 --dim $2 --queries $nq --rounds 6 --reps 20 \
  --variants "CWQ_DUMMY=0;CWQ_STREAM_NO_PRETEST=1" > gpurun_out/ab_pre_$1_$nq.log 2>&1 || exit $?
echo "n=$1 d=$2 nq=$nq"; grep -v amdgpu gpurun_out/ab_pre_$1_$nq.log | tail -3
done; done
