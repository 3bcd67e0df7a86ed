cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
timeout -k 10 400 python -u scripts/small_scan_probe.py > gpurun_out/small_probe.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/small_probe.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --preset c1 --steps 20 --warmup 3 > gpurun_out/bench_c1.log 2>&1; rc=$?; tail -c 300 gpurun_out/bench_c1.log; exit $rc
