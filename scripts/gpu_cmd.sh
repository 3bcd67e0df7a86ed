cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_filter.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/filt_tests.log 2>&1; rc=$?; tail -30 gpurun_out/filt_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/filter_probe.py --modes 1,0 > gpurun_out/probe.log 2>&1; rc=$?; cat gpurun_out/probe.log | grep -v amdgpu.ids; exit $rc
