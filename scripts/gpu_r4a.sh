#!/bin/bash
# Round 4, call A: the new GPU tests (G9 interleaved, pool reloads/fallback, C2 at shape),
# the C2 probe, the single-workgroup device ifit on flat N(0,I) trees (fan-out ~ N), the
# whole GPU suite, smoke and a bench line.  Each GPU step has its own limit; the script
# stops at the first fault / abort / timeout (exit codes other than 0 and 1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
step() {  # step <name> <timeout_s> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -4 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
PT="python -u -m pytest -p no:cacheprovider -x -v --timeout 600 --timeout-method thread"
step new_tests 900 $PT tests/test_gpu_fit.py tests/test_gpu_c2.py -m gpu
step c2_probe 400 python -u scripts/c2_probe.py
step fit_flat_5k 300 python -u scripts/fit_probe.py --n 5000 --dim 768 --clusters 0
step fit_flat_20k 600 python -u scripts/fit_probe.py --n 20000 --dim 768 --clusters 0
step pytest_gpu 1500 $PT tests -m gpu
step smoke 600 python -c "import __graft_entry__ as g; g.smoke()"
step bench 900 python bench.py --steps 10 --warmup 3
echo "=== done"
