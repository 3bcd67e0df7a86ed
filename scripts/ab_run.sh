cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_filter.py -m gpu -v -x --timeout 120 --timeout-method thread -p no:cacheprovider -k "chunking" > gpurun_out/pyt.log 2>&1; rc=$?; grep -E "PASS|FAIL|Error|assert" gpurun_out/pyt.log | head; exit $rc
