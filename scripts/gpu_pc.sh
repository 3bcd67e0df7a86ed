#!/bin/bash
# kernel timeline of the per-call path (C2 shape, nq = 1): where the fixed cost goes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out; export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
timeout -k 10 300 python3 -u scripts/percall_probe.py --n 100000 --dim 768 --nq 1 --reps 50 --modes -1 > gpurun_out/pc_c2.log 2>&1 || exit $?
grep -v amdgpu gpurun_out/pc_c2.log | tail -3
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format rocpd -d gpurun_out/pc -o run -- \
  python3 scripts/percall_probe.py --n 100000 --dim 768 --nq 1 --reps 50 --modes -1 > gpurun_out/pc_prof.log 2>&1 || exit $?
db=$(find gpurun_out/pc -name '*.db' | head -1); echo "db=$db"
python3 scripts/rocpd_summary.py "$db" --timeline 24 > gpurun_out/pc_timeline.txt 2>&1; tail -40 gpurun_out/pc_timeline.txt
