cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_filter.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/filt_tests.log 2>&1; rc=$?; tail -2 gpurun_out/filt_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
for v in libcwq_m32 libcwq; do
CWQ_LIB=$PWD/rag-cobweb_amd/$v.so timeout -k 10 300 python -u scripts/filter_probe.py --modes 1 > gpurun_out/ab_$v$r.log 2>&1; rc=$?; echo "$v r$r $(grep -o "'fgemm_ms[^,]*" gpurun_out/ab_$v$r.log) $(grep -o "[0-9]* q/s" gpurun_out/ab_$v$r.log)"; [ $rc -eq 0 ] || exit $rc
done; done
