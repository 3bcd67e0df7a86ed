#!/bin/bash
# Round 4, call J: ifit KL sums in torch's float32 order with correctly rounded logs -- the
# fit tests, C1 (G8, the reference's own tree), the flat 20k probe; then the rest of the suite.
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
step r4j_fit 600 python -u -m pytest -p no:cacheprovider -v --timeout 400 --timeout-method thread -m gpu tests/test_gpu_fit.py tests/test_gpu_c1.py
CWQ_FIT_PROFILE=1 step r4j_fitflat 300 python -u scripts/fit_probe.py --n 20000 --dim 768 --clusters 0 --chunk 2000 --compare-every 5000
step r4j_suite 900 python -u -m pytest -p no:cacheprovider -v --timeout 400 --timeout-method thread -m gpu tests/ --deselect tests/test_gpu_fit.py --deselect tests/test_gpu_c1.py
step r4j_cat_b4 240 python -u scripts/basic_probe.py --balanced 4,9 --queries 500 --reps 2 --max-nodes 1000000000 --rank-queries 8
echo done
