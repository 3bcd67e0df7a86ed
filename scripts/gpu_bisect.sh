#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out; export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
T="tests/test_gpu_configs.py::test_c5_whitened_d256"
for e in "X=1" "CWQ_FW_ROWS=64" "CWQ_FW_NOPF=1" "CWQ_FW_ROWS=64 CWQ_FW_NOPF=1" "CWQ_STREAM_I8=0" "CWQ_STREAM_NOBUF=1"; do
  env $e timeout -k 10 200 python3 -u -m pytest "$T" -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/bis.log 2>&1
  echo "$e -> rc=$? $(tail -1 gpurun_out/bis.log)"
done
