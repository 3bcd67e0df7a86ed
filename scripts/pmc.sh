#!/bin/bash
# rocprofv3 PMC passes over the filter probe (one counter group per pass,
# kernel-trace only; never combined with sys/runtime tracing).
#   bash scripts/pmc.sh "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE SQ_WAVES ..."
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
i=0
for set in "$@"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $set --kernel-trace --output-format csv -d gpurun_out/pmc/p$i -o run -- \
      python3 scripts/filter_probe.py --modes 1 --reps 1 > gpurun_out/pmc/p$i.log 2>&1
  rc=$?; echo "pass $i ($set) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmc/p$i.log; exit $rc; fi
done
