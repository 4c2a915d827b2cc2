cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for d in ${DBG:-2 0 2}; do
timeout -k 10 200 python -u scripts/debug_mt.py 3 23 $d > gpurun_out/dbg_mt_$d.log 2>&1; rc=$?
tail -8 gpurun_out/dbg_mt_$d.log
[ $rc -le 1 ] || exit $rc
done
