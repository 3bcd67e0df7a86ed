#!/bin/bash
# Round 4, call E: the whole -m gpu suite (C1/G8 and C2 included), then smoke, then Basic on
# b4/d9 with max_nodes raised (found-k = 1).  Each step under its own limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
python -c "import cobweb_pkg; cobweb_pkg.load()" || { echo "libcwq does not match the sources"; exit 4; }
step() {   # name, limit, command...
  local name=$1 lim=$2; shift 2
  echo "=== $name"
  timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1
  local rc=$?
  tail -6 gpurun_out/$name.log
  if [ $rc -ne 0 ]; then echo "stopping at $name (rc=$rc)"; exit $rc; fi
}
CWQ_FIT_PROFILE=1 step r4e_fitflat 300 python -u scripts/fit_probe.py --n 20000 --dim 768 --clusters 0 --chunk 2000 --compare-every 5000
step r4e_pytest_gpu 900 python -u -m pytest -p no:cacheprovider -v --timeout 400 --timeout-method thread -m gpu tests/
step r4e_smoke 240 python -u -c "import __graft_entry__ as g; g.smoke()"
step r4e_cat_b4 240 python -u scripts/basic_probe.py --balanced 4,9 --queries 500 --reps 2 --max-nodes 1000000000 --rank-queries 8
echo done
