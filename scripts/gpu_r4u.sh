#!/bin/bash
# Round 4, call U: unforked KL terms staged over the whole master workgroup -- fit/C1/C2 parity,
# the clustered fit profile, the flat 20k probe, the C2 probe.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
python -c "import cobweb_pkg; cobweb_pkg.load()" || { echo "libcwq does not match the sources"; exit 4; }
step() {   # name, limit, command...
  local name=$1 lim=$2; shift 2
  echo "=== $name"
  timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1
  local rc=$?
  tail -3 gpurun_out/$name.log
  if [ $rc -ne 0 ]; then echo "stopping at $name (rc=$rc)"; exit $rc; fi
}
step r4u_fit 600 python -u -m pytest -p no:cacheprovider -v --timeout 400 --timeout-method thread -m gpu tests/test_gpu_fit.py tests/test_gpu_c1.py
CWQ_FIT_PROFILE=all step r4u_fitclu 300 python -u scripts/fit_probe.py --n 20000 --dim 768 --clusters 100 --chunk 5000
step r4u_c2test 600 python -u -m pytest -p no:cacheprovider -v --timeout 400 --timeout-method thread -m gpu tests/test_gpu_c2.py
step r4u_c2 400 python -u scripts/c2_probe.py --calls 100
step r4u_fitflat 300 python -u scripts/fit_probe.py --n 20000 --dim 768 --clusters 0 --chunk 2000 --compare-every 5000
echo done
