#!/bin/bash
# One gpurun call: GPU tests, smoke, a short bench and (optionally) a rocprofv3 pass.
# Each GPU step has its own time limit; the script stops at the first fault /
# abort / timeout (exit codes other than 0 and 1) and never retries a GPU step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
step() {  # step <name> <timeout_s> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
MODE=${1:-all}
if [[ $MODE == all || $MODE == tests ]]; then
  step pytest_gpu 1200 python -m pytest tests -m gpu -q -x -p no:cacheprovider
  step smoke 600 python -c "import __graft_entry__ as g; g.smoke()"
fi
if [[ $MODE == all || $MODE == bench ]]; then
  step bench 900 python bench.py --steps 5 --warmup 2
fi
if [[ $MODE == all || $MODE == prof ]]; then
  export TMPDIR=/tmp
  step rocprof 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \
      python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --recall-queries 0
fi
echo "=== done"
