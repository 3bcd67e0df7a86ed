#!/bin/bash
# kernel stats of the per-call path, one variant per profiled process
#   gpu_i8prof.sh N NQ "VARIANT" ["N NQ VARIANT" ...] as triples: N NQ V N NQ V ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out; export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
i=0
while [ $# -ge 3 ]; do
  N=$1; NQ=$2; V=$3; shift 3; i=$((i+1))
  d=gpurun_out/i8prof_$i
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- \
    python3 scripts/percall_ab.py --n "$N" --nq "$NQ" --rounds 2 --calls 100 --variants "$V" > $d.log 2>&1 || exit $?
  f=$(find $d -name '*kernel_stats.csv' | head -1); echo "== N=$N nq=$NQ $V"
  grep -v amdgpu $d.log | grep "us/call"
  head -8 "$f" | cut -d, -f1-5 | cut -c1-160
done
