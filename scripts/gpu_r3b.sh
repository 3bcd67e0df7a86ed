#!/bin/bash
# round-3 check: GPU tests, then in-process A/Bs of the filter build (HEAD vs the previous
# wave mapping vs the round-2 library) and of the per-call path, and the per-call
# host/device timeline
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
bash scripts/gpu_ab.sh -t "tests -m gpu" -- --libs rag-cobweb_amd/libcwq.so --libs rag-cobweb_amd/libcwq_wq0.so \
  --libs rag-cobweb_amd/libcwq_r2.so --rounds 10 ::: --libs rag-cobweb_amd/libcwq.so --libs rag-cobweb_amd/libcwq_r2.so \
  --queries 1 --rounds 60 && bash scripts/gpu_api.sh
