#!/bin/bash
# GPU ifit: parity with the reference trees, then throughput with and without the speculative single launch per level
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out; export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_fit.py -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pyt_fit.log 2>&1; rc=$?; tail -3 gpurun_out/pyt_fit.log; [ $rc -eq 0 ] || exit $rc
: > gpurun_out/fit_probe.log
for cfg in "1000 768 0" "2000 768 20" "5000 384 50"; do set -- $cfg
  timeout -k 10 300 python -u scripts/fit_probe.py --n $1 --dim $2 --clusters $3 >> gpurun_out/fit_probe.log 2>&1 || exit $?
done
grep -v amdgpu gpurun_out/fit_probe.log
