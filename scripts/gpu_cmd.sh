cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_filter.py -k "multi" -v > gpurun_out/t_m.log 2>&1; rc=$?; grep -E "PASS|FAIL|passed|failed|Error" gpurun_out/t_m.log | tail -6; exit $rc
