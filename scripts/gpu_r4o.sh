#!/bin/bash
# Round 4, call O: split-pass KL terms two per wave + table log -- fit parity (incl. D = 5, 6),
# clustered fit profile, C2 probe; then the hierarchical-tree Fast lines of call N.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
python -c "import cobweb_pkg; cobweb_pkg.load()" || { echo "libcwq does not match the sources"; exit 4; }
step() {   # name, limit, command...
  local name=$1 lim=$2; shift 2
  echo "=== $name"
  timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1
  local rc=$?
  tail -4 gpurun_out/$name.log
  if [ $rc -ne 0 ]; then echo "stopping at $name (rc=$rc)"; exit $rc; fi
}
step r4o_fit 600 python -u -m pytest -p no:cacheprovider -v --timeout 400 --timeout-method thread -m gpu tests/test_gpu_fit.py tests/test_gpu_c1.py
CWQ_FIT_PROFILE=all step r4o_fitclu_fm256 300 python -u scripts/fit_probe.py --n 20000 --dim 768 --clusters 100 --chunk 5000
CWQ_FIT_PROFILE=all CWQ_FIT_FORK_MIN=64 step r4o_fitclu_fm64 300 python -u scripts/fit_probe.py --n 20000 --dim 768 --clusters 100 --chunk 5000
step r4o_c2 400 python -u scripts/c2_probe.py --calls 100
bash scripts/gpu_r4n.sh
