cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_filter.py tests/test_gpu_parity.py -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pyt.log 2>&1; rc=$?; tail -3 gpurun_out/pyt.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u scripts/ab_libs.py --rounds 12 --libs "rag-cobweb_amd/libcwq_base.so,rag-cobweb_amd/libcwq.so" > gpurun_out/ab11.log 2>&1; rc=$?; tail -2 gpurun_out/ab11.log; grep -c MISMATCH gpurun_out/ab11.log; exit $rc
