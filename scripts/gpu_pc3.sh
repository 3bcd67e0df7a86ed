#!/bin/bash
# per-call path: select fused into the probe, early panel loads, root prefix prefetch
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out; export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_smallbatch.py tests/test_gpu_filter.py tests/test_gpu_edges.py tests/test_gpu_streams.py tests/test_gpu_configs.py -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pyt_pc3.log 2>&1; rc=$?; tail -3 gpurun_out/pyt_pc3.log; [ $rc -eq 0 ] || exit $rc
for n in 100000 1000000; do
  timeout -k 10 200 python -u scripts/percall_probe.py --n $n --dim 768 --nq 1,8,64 --reps 50 --modes -1 > gpurun_out/pc3_$n.log 2>&1 || exit $?
  CWQ_STREAM_SELECT=1 timeout -k 10 200 python -u scripts/percall_probe.py --n $n --dim 768 --nq 1,8,64 --reps 50 --modes -1 > gpurun_out/pc3s_$n.log 2>&1 || exit $?
  grep 'us/call' gpurun_out/pc3_$n.log; grep 'us/call' gpurun_out/pc3s_$n.log
done
