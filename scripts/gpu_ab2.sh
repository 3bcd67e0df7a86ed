#!/bin/bash
# A/B: LDS-DMA half-stage issued among the MFMA cluster (FG_CDMA) vs the product build
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out; export PYTHONDONTWRITEBYTECODE=1
CWQ_LIB=rag-cobweb_amd/libcwq_cdma.so timeout -k 10 300 python -u -m pytest tests/test_gpu_filter.py tests/test_gpu_parity.py -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pyt_cdma.log 2>&1; rc=$?; tail -2 gpurun_out/pyt_cdma.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u scripts/ab_libs.py --rounds 8 --libs rag-cobweb_amd/libcwq.so --libs rag-cobweb_amd/libcwq_cdma.so --libs rag-cobweb_amd/libcwq_cdma2.so > gpurun_out/ab_cdma.log 2>&1; rc=$?; tail -5 gpurun_out/ab_cdma.log; exit $rc
