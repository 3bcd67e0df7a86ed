#!/bin/bash
# per-call probe size (CWQ_STREAM_PROBE_DIV: probe groups = groups / div) at C3 and C2, nq = 1 and 64
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out; export PYTHONDONTWRITEBYTECODE=1
for nq in 1 64; do
timeout -k 10 300 python -u scripts/env_ab.py --n 1000000 --dim 768 --queries $nq --rounds 8 --reps 20 \
  --variants "CWQ_FW_UNFUSED=0;CWQ_STREAM_PROBE_DIV=16;CWQ_STREAM_PROBE_DIV=64;CWQ_STREAM_PROBE_DIV=128" > gpurun_out/ab_probe_c3_$nq.log 2>&1 || exit $?
grep -v amdgpu gpurun_out/ab_probe_c3_$nq.log | tail -4
done
