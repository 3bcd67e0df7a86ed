#!/bin/bash
# Round 4, call E: C1 (G8) and C2 at their shapes, Basic on b4/d9 with max_nodes raised
# (found-k = 1), each step under its own limit; stops at a failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
PT="python -u -m pytest -p no:cacheprovider -x -v -s --timeout 400 --timeout-method thread -m gpu"
step() {   # name, limit, command...
  local name=$1 lim=$2; shift 2
  echo "=== $name"
  timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1
  local rc=$?
  tail -4 gpurun_out/$name.log
  if [ $rc -ne 0 ]; then echo "stopping at $name (rc=$rc)"; exit $rc; fi
}
step r4e_c1 420 $PT tests/test_gpu_c1.py
step r4e_c2 600 $PT tests/test_gpu_c2.py
step r4e_cat_b4 240 python -u scripts/basic_probe.py --balanced 4,9 --queries 500 --reps 2 --max-nodes 1000000000 --rank-queries 8
echo done
