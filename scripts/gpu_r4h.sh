#!/bin/bash
# Round 4, call H: fit pu sums in three waves -- the fit tests and the flat 20k profile --
# and where C2's Basic batch spends its time (kernel stats of the Basic legs).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
python -c "import cobweb_pkg; cobweb_pkg.load()" || { echo "libcwq does not match the sources"; exit 4; }
step() {   # name, limit, command...
  local name=$1 lim=$2; shift 2
  echo "=== $name"
  timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1
  local rc=$?
  tail -5 gpurun_out/$name.log
  if [ $rc -ne 0 ]; then echo "stopping at $name (rc=$rc)"; exit $rc; fi
}
step r4h_fit 400 python -u -m pytest -p no:cacheprovider -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_fit.py
CWQ_FIT_PROFILE=1 step r4h_fitflat 300 python -u scripts/fit_probe.py --n 20000 --dim 768 --clusters 0 --chunk 2000 --compare-every 5000
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT}"
step r4h_prof_basic 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4h_prof_basic -o r4h -- python3 -u scripts/c2_probe.py --basic-only --calls 20
echo done
