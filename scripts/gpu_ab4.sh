#!/bin/bash
# A/B: non-temporal row-panel loads in the per-call stream filter (SK_NT) vs the product build
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out; export PYTHONDONTWRITEBYTECODE=1
CWQ_LIB=rag-cobweb_amd/libcwq_nt.so timeout -k 10 300 python -u -m pytest tests/test_gpu_filter.py tests/test_gpu_smallbatch.py tests/test_gpu_edges.py -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pyt_nt.log 2>&1; rc=$?; tail -2 gpurun_out/pyt_nt.log; [ $rc -eq 0 ] || exit $rc
for nq in 1 64; do
timeout -k 10 300 python -u scripts/ab_libs.py --rounds 40 --queries $nq --libs rag-cobweb_amd/libcwq.so --libs rag-cobweb_amd/libcwq_nt.so > gpurun_out/ab_nt_$nq.log 2>&1 || exit $?
tail -2 gpurun_out/ab_nt_$nq.log; grep -c MISMATCH gpurun_out/ab_nt_$nq.log
done
