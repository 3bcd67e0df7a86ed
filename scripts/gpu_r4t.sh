#!/bin/bash
# Round 4, call T: the clustered fit's level phases split finer (P + x, merge/split KL terms).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
python -c "import cobweb_pkg; cobweb_pkg.load()" || { echo "libcwq does not match the sources"; exit 4; }
echo "=== r4t_fitclu"
CWQ_FIT_PROFILE=all timeout -k 10 300 python -u scripts/fit_probe.py --n 20000 --dim 768 --clusters 100 --chunk 5000 > gpurun_out/r4t_fitclu.log 2>&1 || exit $?
grep -v amdgpu gpurun_out/r4t_fitclu.log
echo done
