cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/sy
for i in 1 2 3; do
LM_SYNC_INPUTS=1 LM_ALLOC=finegrained timeout -k 10 300 python -u scripts/debug_mt.py 3 23 0 > gpurun_out/sy/in_$i.log 2>&1; echo "sync inputs: rc=$? $(tail -1 gpurun_out/sy/in_$i.log)"
LM_SYNC_OUTPUTS=1 LM_ALLOC=finegrained timeout -k 10 300 python -u scripts/debug_mt.py 3 23 0 > gpurun_out/sy/out_$i.log 2>&1; echo "sync outputs: rc=$? $(tail -1 gpurun_out/sy/out_$i.log)"
LM_ALLOC=finegrained timeout -k 10 300 python -u scripts/debug_mt.py 3 23 0 > gpurun_out/sy/none_$i.log 2>&1; echo "no sync: rc=$? $(tail -1 gpurun_out/sy/none_$i.log)"
done
