#!/bin/bash
# rocprofv3 PMC passes (one counter group per pass, kernel-trace only; never
# combined with sys/runtime tracing) over a short bench run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
BENCH="python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --recall-queries 0"
timeout -k 10 120 rocprofv3 -L > gpurun_out/pmc/counters.txt 2>&1; echo "list rc=$?"
i=0
for set in "$@"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --kernel-trace --output-format csv -d gpurun_out/pmc/p$i -o run -- $BENCH \
      > gpurun_out/pmc/p$i.log 2>&1
  rc=$?; echo "pass $i ($set) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmc/p$i.log; exit $rc; fi
done
