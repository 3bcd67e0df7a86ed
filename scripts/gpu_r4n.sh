#!/bin/bash
# Round 4, call N: hierarchical-tree Fast at HEAD -- b4/d9 and b10/d5 1M x 768,
# 10k-query batch calls and one-query calls, with a kernel-stats profile of the b4/d9 batch.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
python -c "import cobweb_pkg; cobweb_pkg.load()" || { echo "libcwq does not match the sources"; exit 4; }
step() {   # name, limit, command...
  local name=$1 lim=$2; shift 2
  echo "=== $name"
  timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1
  local rc=$?
  tail -4 gpurun_out/$name.log
  if [ $rc -ne 0 ]; then echo "stopping at $name (rc=$rc)"; exit $rc; fi
}
step r4n_fast_b4 300 python -u scripts/filter_probe.py --balanced 4,9 --modes 1 --reps 3
step r4n_pc_b4 300 python -u scripts/percall_probe.py --balanced 4,9 --nq 1,8,64 --modes -1 --reps 50 --wrapper
step r4n_fast_b10 300 python -u scripts/filter_probe.py --balanced 10,5 --modes 1 --reps 3
step r4n_pc_b10 300 python -u scripts/percall_probe.py --balanced 10,5 --nq 1,8,64 --modes -1 --reps 50
step r4n_fast_b4_prof 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r4n_b4prof -o run -- python3 -u scripts/filter_probe.py --balanced 4,9 --modes 1 --reps 3
f=$(find gpurun_out/r4n_b4prof -name '*kernel_stats.csv' | head -1); [ -n "$f" ] && cp "$f" gpurun_out/r4n_fast_b4_kernel_stats.csv && head -12 "$f"
echo done
