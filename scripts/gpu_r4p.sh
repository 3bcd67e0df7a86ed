#!/bin/bash
# Round 4, call P: clustered fit without helper workgroups (do the helpers' polls slow the
# master's levels?), and the kernel timeline of one-query calls on the b4/d9 tree.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
python -c "import cobweb_pkg; cobweb_pkg.load()" || { echo "libcwq does not match the sources"; exit 4; }
echo "=== r4p_fitclu_h0"
CWQ_FIT_HELPERS=0 timeout -k 10 300 python -u scripts/fit_probe.py --n 20000 --dim 768 --clusters 100 --chunk 5000 > gpurun_out/r4p_fitclu_h0.log 2>&1 || exit $?
tail -2 gpurun_out/r4p_fitclu_h0.log
echo "=== r4p_pc_b4 timeline"
bash scripts/gpu_pc.sh 1000000 1 "--balanced 4,9" || exit $?
echo done
