cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_filter.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/filt_tests.log 2>&1; rc=$?; tail -2 gpurun_out/filt_tests.log; [ $rc -eq 0 ] || exit $rc
for o in "0 1" "2 1" "0 0"; do set -- $o
CWQ_FG_ORDER=$1 CWQ_FG_PHASES=$2 timeout -k 10 300 python -u scripts/filter_probe.py --modes 1 > gpurun_out/probe_$1$2.log 2>&1; rc=$?; echo "order $1 phases $2"; grep -v amdgpu.ids gpurun_out/probe_$1$2.log | grep -o "q/s.*"; [ $rc -eq 0 ] || exit $rc
done
