cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/t_gpu.log 2>&1; rc=$?; tail -1 gpurun_out/t_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_f -o run -- python3 scripts/filter_probe.py --reps 2 > gpurun_out/prof_f.log 2>&1; rc=$?; grep "mode 1\|equal" gpurun_out/prof_f.log; exit $rc
