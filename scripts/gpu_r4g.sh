#!/bin/bash
# Round 4, call G: per-node internal prefixes (chain kernel), split sums staged, fused
# per-call prep/select; the affected GPU tests, the C2 probe, the flat 20k fit with its
# phase profile, and the C2-flat per-call A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
python -c "import cobweb_pkg; cobweb_pkg.load()" || { echo "libcwq does not match the sources"; exit 4; }
step() {   # name, limit, command...
  local name=$1 lim=$2; shift 2
  echo "=== $name"
  timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1
  local rc=$?
  tail -5 gpurun_out/$name.log
  if [ $rc -ne 0 ]; then echo "stopping at $name (rc=$rc)"; exit $rc; fi
}
step r4g_tests 600 python -u -m pytest -p no:cacheprovider -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_smallbatch.py tests/test_gpu_parity.py tests/test_gpu_group.py tests/test_gpu_cat_count.py tests/test_gpu_fit.py
step r4g_c2probe 240 python -u scripts/c2_probe.py --calls 100
step r4g_ab_c2 240 python -u scripts/percall_ab.py --n 100000 --calls 200 --rounds 5 \
  --variants "CWQ_SELECT_UNFUSED=1;CWQ_PROBE_PREP=0;CWQ_SELECT_UNFUSED=0;CWQ_STREAM_WGS=2;CWQ_STREAM_I8=1"
CWQ_FIT_PROFILE=1 step r4g_fitflat 300 python -u scripts/fit_probe.py --n 20000 --dim 768 --clusters 0 --chunk 2000 --compare-every 5000
echo done
