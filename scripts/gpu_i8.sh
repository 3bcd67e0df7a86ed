#!/bin/bash
# int8 stream filter pass: stream-path GPU tests, then in-process per-call A/Bs (bf16 vs int8 pass)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out; export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
V="${V:-CWQ_STREAM_I8=0;CWQ_STREAM_I8=1;CWQ_STREAM_I8=1&CWQ_STREAM_CH8=1}"
timeout -k 10 400 python3 -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/i8_pytest.log 2>&1 || { tail -30 gpurun_out/i8_pytest.log; exit 1; }
tail -2 gpurun_out/i8_pytest.log
timeout -k 10 300 python3 -u scripts/percall_ab.py --n 1000000 --nq 1 --variants "$V" > gpurun_out/i8_ab_c3_nq1.log 2>&1 || { tail -20 gpurun_out/i8_ab_c3_nq1.log; exit 1; }
grep -v amdgpu gpurun_out/i8_ab_c3_nq1.log
timeout -k 10 300 python3 -u scripts/percall_ab.py --n 100000 --nq 1 --variants "$V" > gpurun_out/i8_ab_c2_nq1.log 2>&1 || { tail -20 gpurun_out/i8_ab_c2_nq1.log; exit 1; }
grep -v amdgpu gpurun_out/i8_ab_c2_nq1.log
timeout -k 10 300 python3 -u scripts/percall_ab.py --n 1000000 --nq 64 --calls 50 --variants "$V" > gpurun_out/i8_ab_c3_nq64.log 2>&1 || { tail -20 gpurun_out/i8_ab_c3_nq64.log; exit 1; }
grep -v amdgpu gpurun_out/i8_ab_c3_nq64.log
