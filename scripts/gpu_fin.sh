#!/bin/bash
# round-3 final check: all GPU tests, smoke, bench (N=1), per-call A/B at C3
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out; export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/fin_pytest.log 2>&1 || { tail -30 gpurun_out/fin_pytest.log; exit 1; }
tail -1 gpurun_out/fin_pytest.log
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fin_smoke.log 2>&1 || { tail -20 gpurun_out/fin_smoke.log; exit 1; }
tail -1 gpurun_out/fin_smoke.log | cut -c1-200
timeout -k 10 600 python3 -u bench.py --steps 10 --warmup 3 > gpurun_out/fin_bench.log 2>&1 || { tail -20 gpurun_out/fin_bench.log; exit 1; }
tail -1 gpurun_out/fin_bench.log | cut -c1-200
