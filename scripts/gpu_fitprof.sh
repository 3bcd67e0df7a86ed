#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out; export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 300 python -u -m cProfile -s tottime scripts/fit_probe.py --n 2000 --dim 768 --clusters 20 --spec 16 > gpurun_out/fit_cprofile.log 2>&1 || exit $?
head -45 gpurun_out/fit_cprofile.log
