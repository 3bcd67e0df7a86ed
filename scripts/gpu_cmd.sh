cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for d in 0 2 3; do
CWQ_FG_DBG=$d timeout -k 10 300 python -u scripts/filter_probe.py --modes 1 > gpurun_out/probe_d$d.log 2>&1; rc=$?; echo "dbg $d $(grep -o "'fgemm_ms[^,]*" gpurun_out/probe_d$d.log)"; [ $rc -eq 0 ] || exit $rc
done
