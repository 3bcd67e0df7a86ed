cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
timeout -k 10 600 python -u bench.py --n 10000000 --dim 1024 --queries 12500 --steps 3 --warmup 1 --no-cpu-baseline --recall-queries 256 > gpurun_out/bench_c4.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/bench_c4.log | tail -1; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/bench.log | tail -1; exit $rc
