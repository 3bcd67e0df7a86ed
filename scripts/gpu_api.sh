#!/bin/bash
# Host + device timeline of the per-call path (C3 shape, nq = 1): HIP runtime API calls and
# kernels on one clock (rocprofv3 --hip-runtime-trace --kernel-trace; no counters).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out; export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
N=${1:-1000000}
timeout -k 10 300 rocprofv3 --hip-runtime-trace --kernel-trace --output-format csv -d gpurun_out/api -o run -- \
  python3 scripts/percall_probe.py --n "$N" --dim 768 --nq 1 --reps 30 --modes -1 > gpurun_out/api_prof.log 2>&1 || exit $?
p=$(find gpurun_out/api -name 'run_kernel_trace.csv' | head -1); p=${p%kernel_trace.csv}
python3 scripts/api_timeline.py "$p" --last 2 > gpurun_out/api_timeline.txt 2>&1; tail -80 gpurun_out/api_timeline.txt
