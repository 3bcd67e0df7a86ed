#!/bin/bash
# Round 4, call S: parallel draws + top-2 on unforked levels of >= 8 children -- the whole
# -m gpu suite, the clustered fit profile, the C2 probe; the per-call counters zeroed by the
# query prep (no memset launch) on the b4/d9 and b10/d5 one-query calls.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
python -c "import cobweb_pkg; cobweb_pkg.load()" || { echo "libcwq does not match the sources"; exit 4; }
step() {   # name, limit, command...
  local name=$1 lim=$2; shift 2
  echo "=== $name"
  timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1
  local rc=$?
  tail -3 gpurun_out/$name.log
  if [ $rc -ne 0 ]; then echo "stopping at $name (rc=$rc)"; exit $rc; fi
}
step r4s_pytest_gpu 900 python -u -m pytest -p no:cacheprovider -v --timeout 400 --timeout-method thread -m gpu tests
CWQ_FIT_PROFILE=all step r4s_fitclu 300 python -u scripts/fit_probe.py --n 20000 --dim 768 --clusters 100 --chunk 5000
step r4s_c2 400 python -u scripts/c2_probe.py --calls 100
step r4s_pc_b4 300 python -u scripts/percall_probe.py --balanced 4,9 --nq 1,8,64 --modes -1 --reps 50
step r4s_pc_b10 300 python -u scripts/percall_probe.py --balanced 10,5 --nq 1,8,64 --modes -1 --reps 50
echo done
