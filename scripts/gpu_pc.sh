#!/bin/bash
# kernel timeline of the per-call path (one query per call): where the fixed cost goes.
#   gpu_pc.sh [N rows (default 1000000)] [nq (default 1)] [extra percall_probe args, e.g. "--balanced 4,9"]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out; export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
N=${1:-1000000}; NQ=${2:-1}; EXTRA=${3:-}
timeout -k 10 300 python3 -u scripts/percall_probe.py --n "$N" --dim 768 --nq "$NQ" --reps 50 --modes -1 $EXTRA > gpurun_out/pc_$N.log 2>&1 || exit $?
grep -v amdgpu gpurun_out/pc_$N.log | tail -3
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format rocpd -d gpurun_out/pc_$N -o run -- \
  python3 scripts/percall_probe.py --n "$N" --dim 768 --nq "$NQ" --reps 50 --modes -1 $EXTRA > gpurun_out/pc_prof_$N.log 2>&1 || exit $?
db=$(find gpurun_out/pc_$N -name '*.db' | head -1); echo "db=$db"
python3 scripts/rocpd_summary.py "$db" --timeline 24 > gpurun_out/pc_timeline_$N.txt 2>&1; tail -40 gpurun_out/pc_timeline_$N.txt
