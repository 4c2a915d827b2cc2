cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/debug_stream.py 12800 23 256 --check > gpurun_out/dbg_12800.log 2>&1; rc=$?
tail -5 gpurun_out/dbg_12800.log
[ $rc -le 1 ] || exit $rc
for i in 1 2; do
timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu --streams 3 > gpurun_out/b3_$i.json 2> gpurun_out/b3_$i.err; echo "bench3 rc=$?"; tail -1 gpurun_out/b3_$i.err; cat gpurun_out/b3_$i.json
done
