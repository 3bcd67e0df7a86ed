#!/bin/bash
# rerank form on deep trees: wave per query (final_kernel, default above 256 queries) vs
# workgroup per query (final_wide_kernel, CWQ_FINAL_WIDE raises its query limit); the
# filter probe's rerank_ms, each arm twice, interleaved
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out; export PYTHONDONTWRITEBYTECODE=1
for t in "4,9" "10,5"; do
  for arm in 256 100000 256 100000; do
    CWQ_FINAL_WIDE=$arm timeout -k 10 300 python scripts/filter_probe.py --balanced $t --modes 1 --reps 3 > gpurun_out/fw_$arm.log 2>&1 || exit $?
    echo "tree $t CWQ_FINAL_WIDE=$arm: $(grep -o "mode 1: [0-9.]* ms/call" gpurun_out/fw_$arm.log) $(grep -o "'rerank_ms': [0-9.]*" gpurun_out/fw_$arm.log)"
  done
done
