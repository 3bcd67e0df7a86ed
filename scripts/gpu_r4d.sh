#!/bin/bash
# Round 4, call D: group-centred filter + stratified sample, two-level categorize replay,
# the chip-wide device ifit tests, C1/C2 at their shapes, the C2 probe, and the flat 20k
# fit probe against one workgroup.  Each step under its own limit; stops at a failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
PT="python -u -m pytest -p no:cacheprovider -x -v -s --timeout 300 --timeout-method thread -m gpu"
step() {   # name, limit, command...
  local name=$1 lim=$2; shift 2
  echo "=== $name"
  timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1
  local rc=$?
  tail -4 gpurun_out/$name.log
  if [ $rc -ne 0 ]; then echo "stopping at $name (rc=$rc)"; exit $rc; fi
}
step r4d_group 240 $PT tests/test_gpu_group.py
step r4d_catcount 300 $PT tests/test_gpu_cat_count.py
step r4d_c2probe 240 python -u scripts/c2_probe.py --calls 100
step r4d_fit 420 $PT tests/test_gpu_fit.py
step r4d_fitflat 300 python -u scripts/fit_probe.py --n 20000 --dim 768 --clusters 0 --chunk 2000 --compare-every 5000
echo done
