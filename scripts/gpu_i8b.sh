#!/bin/bash
# int8 pass on hierarchical trees: tests, per-call A/B (b4/d9, b10/d5), then the bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out; export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
V="CWQ_STREAM_I8=0;CWQ_STREAM_I8=1"
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_filter.py tests/test_gpu_smallbatch.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/i8b_pytest.log 2>&1 || { tail -30 gpurun_out/i8b_pytest.log; exit 1; }
tail -1 gpurun_out/i8b_pytest.log
for t in 4,9 10,5; do
  timeout -k 10 400 python3 -u scripts/percall_ab.py --n 1000000 --nq 1 --calls 100 --rounds 3 --balanced $t --variants "$V" > gpurun_out/i8b_ab_$t.log 2>&1 || { tail -20 gpurun_out/i8b_ab_$t.log; exit 1; }
  grep -v amdgpu gpurun_out/i8b_ab_$t.log | grep -v "^round"
done
timeout -k 10 600 python3 -u bench.py --steps 10 --warmup 3 > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log | cut -c1-300
