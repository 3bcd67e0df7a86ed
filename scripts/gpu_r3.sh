#!/bin/bash
# Round-3 GPU pass: the GPU tests (new ones first, so a failure there shows fast), smoke,
# the default bench line.  Each step has its own time limit; stops at the first fault /
# abort / timeout; never retries a GPU step.  Usage: gpu_r3.sh [tests-selector] [bench args...]
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
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
SEL=${1:-all}
shift
PYT="python -u -m pytest -x -v -p no:cacheprovider --timeout 400 --timeout-method thread"
if [[ $SEL == all || $SEL == new ]]; then
  step pytest_new 900 $PYT tests/test_gpu_fullsize.py
fi
if [[ $SEL == all ]]; then
  step pytest_gpu 1200 $PYT tests -m gpu --ignore=tests/test_gpu_fullsize.py
  step smoke 600 python -c "import __graft_entry__ as g; g.smoke()"
fi
if [[ $SEL == all || $SEL == bench ]]; then
  step bench 900 python bench.py --steps 10 --warmup 3 "$@"
  tail -1 gpurun_out/bench.log
fi
