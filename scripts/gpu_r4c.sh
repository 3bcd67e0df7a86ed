#!/bin/bash
# Round 4, call C: the chip-wide device ifit under 3 s spin bounds with the progress
# watchdog, one case per process (each under its own short limit); then the group-centred
# filter tests and the C2 probe.  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
for c in 64,300,64,1 64,300,64,-1 64,600,64,-1 384,400,256,-1; do
  echo "=== case $c"
  CWQ_FIT_SPIN_MS=3000 CWQ_FIT_WATCH=1 timeout -k 5 45 python -u scripts/fit_debug.py $c > gpurun_out/fit_debug_$c.log 2>&1
  rc=$?
  tail -3 gpurun_out/fit_debug_$c.log
  if [ $rc -ne 0 ]; then echo "stopping (rc=$rc)"; exit $rc; fi
done
echo "=== group tests"
timeout -k 10 300 python -u -m pytest -p no:cacheprovider -x -v --timeout 240 --timeout-method thread tests/test_gpu_group.py -m gpu > gpurun_out/group_tests.log 2>&1
rc=$?; tail -5 gpurun_out/group_tests.log; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
echo "=== c2 probe"
timeout -k 10 300 python -u scripts/c2_probe.py --calls 100 > gpurun_out/c2_probe_grp.log 2>&1
rc=$?; cat gpurun_out/c2_probe_grp.log | tail -12; exit $rc
