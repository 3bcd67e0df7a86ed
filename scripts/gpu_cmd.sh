cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_whitening.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/whiten_tests.log 2>&1; rc=$?; tail -15 gpurun_out/whiten_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/whiten_probe.py > gpurun_out/whiten_probe.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/whiten_probe.log; exit $rc
