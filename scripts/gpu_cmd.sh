cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/t_gpu.log 2>&1; rc=$?; tail -1 gpurun_out/t_gpu.log; [ $rc -eq 0 ] || exit $rc
for G in 1024 100000; do
timeout -k 10 300 python -u scripts/filter_probe.py --clusters $G > gpurun_out/probe_g$G.log 2>&1; rc=$?; grep "mode\|identical\|differ" gpurun_out/probe_g$G.log; [ $rc -eq 0 ] || exit $rc
done
