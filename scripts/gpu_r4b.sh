#!/bin/bash
# Round 4, call B: the chip-wide device ifit (fit tests, then the flat 20k x 768 probe with
# one-workgroup comparisons), the C2 probe with the exact internal pass, the C1/C2 tests,
# the whole GPU suite, smoke and a bench line.  Stops at the first fault / abort / timeout.
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
step fit_tests 900 $PT tests/test_gpu_fit.py -m gpu
step fit_flat_20k 900 python -u scripts/fit_probe.py --n 20000 --dim 768 --clusters 0 --chunk 2000 --compare-every 5000 --compare-rows 100
step c2_probe_exactint 400 env CWQ_INT_BOUND=0 python -u scripts/c2_probe.py --calls 100
step c1c2_tests 600 $PT tests/test_gpu_c1.py tests/test_gpu_c2.py -m gpu
step pytest_gpu 1500 $PT tests -m gpu
step smoke 600 python -c "import __graft_entry__ as g; g.smoke()"
step bench 900 python bench.py --steps 10 --warmup 3
echo "=== done"
