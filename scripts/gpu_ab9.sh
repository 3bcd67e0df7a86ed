#!/bin/bash
# small-batch exact scan with software-pipelined row loads: GPU tests, then in-process A/Bs
# vs the previous build (rank_scores and the exact-scan Fast call)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out; export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pyt_ab9.log 2>&1; rc=$?; tail -3 gpurun_out/pyt_ab9.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/rank_probe.py --nq 1,16,64,256 --reps 9 \
  --libs rag-cobweb_amd/libcwq_base.so,rag-cobweb_amd/libcwq.so > gpurun_out/ab9_rank.log 2>&1 || exit $?
grep -v amdgpu gpurun_out/ab9_rank.log
for nq in 1 16 64; do
timeout -k 10 300 python -u scripts/ab_libs.py --queries $nq --rounds 12 \
  --libs "rag-cobweb_amd/libcwq_base.so@CWQ_FILTER=0;CWQ_STREAM=0" --libs "rag-cobweb_amd/libcwq.so@CWQ_FILTER=0;CWQ_STREAM=0" > gpurun_out/ab9_exact_$nq.log 2>&1 || exit $?
echo "exact nq=$nq"; grep -v amdgpu gpurun_out/ab9_exact_$nq.log | tail -2
done
