cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
R=rag-cobweb_amd
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/t_gpu.log 2>&1; rc=$?; tail -1 gpurun_out/t_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/filter_probe.py --clusters 100000 > gpurun_out/probe_g.log 2>&1; rc=$?; grep "mode 1\|equal" gpurun_out/probe_g.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u scripts/ab_libs.py --rounds 4 --clusters 100000 --libs $R/libcwq_head.so,$R/libcwq.so > gpurun_out/ab.log 2>&1; rc=$?; tail -2 gpurun_out/ab.log; exit $rc
