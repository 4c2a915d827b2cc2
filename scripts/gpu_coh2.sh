cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
LM_ALLOC=uncached timeout -k 10 400 python -u scripts/debug_stream.py 6400 23 256 --check > gpurun_out/u1.log 2>&1; echo "single ctx uncached vs oracle: rc=$? $(tail -1 gpurun_out/u1.log)"; grep -m5 "differs\|error" gpurun_out/u1.log | cut -c1-250
LM_ALLOC=finegrained timeout -k 10 400 python -u scripts/debug_stream.py 6400 23 256 --check > gpurun_out/u2.log 2>&1; echo "single ctx finegrained vs oracle: rc=$? $(tail -1 gpurun_out/u2.log)"; grep -m5 "differs\|error" gpurun_out/u2.log | cut -c1-250
