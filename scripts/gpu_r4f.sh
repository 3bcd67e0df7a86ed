#!/bin/bash
# Round 4, call F: per-call latency A/Bs (fused select, workgroups per CU) at C2 (100k x 768
# flat) and C3 (1M), and a kernel-stats profile of the default per-call path at C2.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
python -c "import cobweb_pkg; cobweb_pkg.load()" || { echo "libcwq does not match the sources"; exit 4; }
step() {   # name, limit, command...
  local name=$1 lim=$2; shift 2
  echo "=== $name"
  timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1
  local rc=$?
  tail -6 gpurun_out/$name.log
  if [ $rc -ne 0 ]; then echo "stopping at $name (rc=$rc)"; exit $rc; fi
}
step r4f_ab_c2 240 python -u scripts/percall_ab.py --n 100000 --calls 200 --rounds 5 \
  --variants "CWQ_SELECT_UNFUSED=1;CWQ_PROBE_PREP=0;CWQ_SELECT_UNFUSED=0;CWQ_STREAM_WGS=2;CWQ_STREAM_WGS=3;CWQ_STREAM_I8=1"
step r4f_ab_c3 300 python -u scripts/percall_ab.py --n 1000000 --calls 200 --rounds 4 \
  --variants "CWQ_SELECT_UNFUSED=1;CWQ_PROBE_PREP=0;CWQ_SELECT_UNFUSED=0;CWQ_STREAM_WGS=2"
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT}"
echo "=== r4f_prof_c2"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/r4f_prof_c2 -o r4f -- python3 -u scripts/percall_ab.py --n 100000 --calls 200 --rounds 2 --variants "CWQ_SELECT_UNFUSED=0" > gpurun_out/r4f_prof_c2.log 2>&1
rc=$?; tail -4 gpurun_out/r4f_prof_c2.log; [ $rc -ne 0 ] && exit $rc
echo "=== r4f_prof_c2_i8"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/r4f_prof_c2_i8 -o r4f -- python3 -u scripts/percall_ab.py --n 100000 --calls 200 --rounds 2 --variants "CWQ_STREAM_I8=1" > gpurun_out/r4f_prof_c2_i8.log 2>&1
rc=$?; tail -4 gpurun_out/r4f_prof_c2_i8.log; exit $rc
