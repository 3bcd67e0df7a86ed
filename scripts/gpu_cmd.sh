cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
for r in 1 2 3; do
for v in prev cur; do
L=rag-cobweb_amd/libcwq.so; [ $v = prev ] && L=rag-cobweb_amd/libcwq_prev.so
CWQ_LIB=$PWD/$L timeout -k 10 300 python -u scripts/filter_probe.py --modes 1 > gpurun_out/ab_$v$r.log 2>&1; rc=$?; echo "$v r$r $(grep -o "'fgemm_ms[^,]*" gpurun_out/ab_$v$r.log) $(grep -o "[0-9]* q/s" gpurun_out/ab_$v$r.log)"; [ $rc -eq 0 ] || exit $rc
done; done
