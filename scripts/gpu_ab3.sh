#!/bin/bash
# phase plans of the batch filter at the C2 (100k x 768, 1k queries) and C5 (8.8M x 256, 10k) shapes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out; export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 300 python -u scripts/env_ab.py --n 100000 --dim 768 --queries 1000 --rounds 6 --reps 10 \
  --variants "CWQ_FG_PHASES=1;CWQ_FG_PHASES=0;CWQ_FG_CUTS=256;CWQ_FG_CUTS=128,512;CWQ_FG_CUTS=64,256" > gpurun_out/ab_c2_phases.log 2>&1 || exit $?
grep -v amdgpu gpurun_out/ab_c2_phases.log | tail -5
timeout -k 10 400 python -u scripts/env_ab.py --n 8800000 --dim 256 --queries 10000 --rounds 4 --reps 2 \
  --variants "CWQ_FG_PHASES=1;CWQ_FG_PHASES=0;CWQ_FG_CUTS=64,256,512;CWQ_FG_CUTS=16,64,256,512" > gpurun_out/ab_c5_phases.log 2>&1 || exit $?
grep -v amdgpu gpurun_out/ab_c5_phases.log | tail -4
