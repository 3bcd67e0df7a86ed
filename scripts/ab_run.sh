cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
timeout -k 10 900 python -u scripts/ab_libs.py --n 10000000 --dim 1024 --queries 12500 --rounds 4 --share-index --libs "rag-cobweb_amd/libcwq.so@CWQ_FG_CUTS=64,256" --libs "rag-cobweb_amd/libcwq.so" > gpurun_out/ab7.log 2>&1; rc=$?; tail -3 gpurun_out/ab7.log; exit $rc
