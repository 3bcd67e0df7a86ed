cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
CWQ_FG_STAMP=$PWD/gpurun_out/stamps.bin CWQ_LIB=$PWD/rag-cobweb_amd/libcwq_stamp.so timeout -k 10 300 python -u scripts/filter_probe.py --modes 1 --reps 1 > gpurun_out/probe_st.log 2>&1; rc=$?; grep mode gpurun_out/probe_st.log; [ $rc -eq 0 ] || exit $rc
python scripts/stamp_summary.py gpurun_out/stamps.bin
