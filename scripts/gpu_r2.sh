#!/bin/bash
# One gpurun call: GPU tests (verbose, per-test timeout), smoke, bench.  Stops at the
# first fault / abort / timeout (exit codes other than 0 and 1); never retries.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
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
MODE=${1:-all}
TESTS=${TESTS:-tests}
if [[ $MODE == all || $MODE == tests ]]; then
  step pytest_gpu 900 python -u -m pytest $TESTS -m gpu -x -v -s --timeout 240 --timeout-method thread -p no:cacheprovider
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
if [[ $MODE == all || $MODE == bench ]]; then
  step bench 600 python bench.py --steps 10 --warmup 3
fi
echo "=== done"
