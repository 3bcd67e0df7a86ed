#!/bin/bash
# One gpurun call for an in-process A/B of libcwq builds or env knobs (replaces the one-off
# gpu_ab1..12 / ab_run / gpu_pc2-3 drivers of rounds 1-2).
#   gpu_ab.sh [-t TESTS] [-T SECONDS] -- <ab_libs.py args> [ ::: <ab_libs.py args> ... ]
# -t: pytest selection run first (default "tests -m gpu"; "none" skips), stops the call on
#     failure; each ':::'-separated group is one ab_libs.py run (--libs lib[@ENV=V;...] ...).
# Each GPU step has its own time limit, the script stops at the first non-zero exit and
# never retries a GPU step.  Logs: gpurun_out/ab_<i>.log
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
TESTS="tests -m gpu"; TLIM=400
while [[ $# -gt 0 && $1 != -- ]]; do
  case $1 in
    -t) TESTS=$2; shift 2 ;;
    -T) TLIM=$2; shift 2 ;;
    *) echo "unknown option $1"; exit 2 ;;
  esac
done
shift
if [[ $TESTS != none ]]; then
  timeout -k 10 900 python -u -m pytest $TESTS -q -x --timeout 120 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/ab_pytest.log 2>&1
  rc=$?; tail -n 2 gpurun_out/ab_pytest.log; [ $rc -eq 0 ] || exit $rc
fi
i=0; args=()
run() {
  [ ${#args[@]} -eq 0 ] && return 0
  i=$((i + 1))
  echo "=== ab_$i: ${args[*]}"
  timeout -k 10 "$TLIM" python -u scripts/ab_libs.py "${args[@]}" > "gpurun_out/ab_$i.log" 2>&1
  local rc=$?
  grep -v amdgpu.ids "gpurun_out/ab_$i.log" | tail -n 4
  [ $rc -eq 0 ] || exit $rc
  args=()
}
for a in "$@"; do
  if [[ $a == ::: ]]; then run; else args+=("$a"); fi
done
run
echo "=== done"
