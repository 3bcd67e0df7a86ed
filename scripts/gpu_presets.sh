#!/bin/bash
# bench lines of the other BASELINE configs' synthetic stand-ins at HEAD (one GPU)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out; export PYTHONDONTWRITEBYTECODE=1
for p in c1 c2 c5; do
  timeout -k 10 400 python -u bench.py --preset $p --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/preset_$p.log 2>&1 || exit $?
  echo "== $p"; tail -1 gpurun_out/preset_$p.log | cut -c1-200
done
timeout -k 10 600 python -u bench.py --preset c4 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/preset_c4.log 2>&1 || exit $?
echo "== c4"; tail -1 gpurun_out/preset_c4.log | cut -c1-200
