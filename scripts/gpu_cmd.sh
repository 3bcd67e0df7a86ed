cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
R=rag-cobweb_amd
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_filter.py > gpurun_out/t_f.log 2>&1; rc=$?; tail -1 gpurun_out/t_f.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/filter_probe.py --modes 1 > gpurun_out/probe.log 2>&1; rc=$?; grep "mode" gpurun_out/probe.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u scripts/ab_libs.py --rounds 10 --libs $R/libcwq_head.so,$R/libcwq.so,$R/libcwq_rdf.so,$R/libcwq_sprio.so,$R/libcwq_both.so > gpurun_out/ab.log 2>&1; rc=$?; tail -5 gpurun_out/ab.log; exit $rc
