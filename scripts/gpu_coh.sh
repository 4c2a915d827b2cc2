cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export LM_ALLOW_QUEUE_SHARING=1
for i in 1 2 3; do
LM_ALLOC=uncached timeout -k 10 300 python -u scripts/debug_mt.py 3 23 0 > gpurun_out/c1_$i.log 2>&1; echo "ns3 uncached: rc=$? $(tail -1 gpurun_out/c1_$i.log)"
LM_ALLOC=finegrained timeout -k 10 300 python -u scripts/debug_mt.py 3 23 0 > gpurun_out/c2_$i.log 2>&1; echo "ns3 finegrained: rc=$? $(tail -1 gpurun_out/c2_$i.log)"
timeout -k 10 300 python -u scripts/debug_mt.py 3 23 0 > gpurun_out/c3_$i.log 2>&1; echo "ns3 default: rc=$? $(tail -1 gpurun_out/c3_$i.log)"
done
