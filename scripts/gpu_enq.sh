cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export LM_ALLOW_QUEUE_SHARING=1
for i in 1 2 3; do
LM_SERIALIZE=2 LM_ALLOC=finegrained timeout -k 10 300 python -u scripts/debug_mt.py 3 23 0 > gpurun_out/e1_$i.log 2>&1; echo "ns3 fg enqueue-serialized: rc=$? $(tail -1 gpurun_out/e1_$i.log)"
LM_ALLOC=finegrained timeout -k 10 300 python -u scripts/debug_mt.py 3 23 0 > gpurun_out/e2_$i.log 2>&1; echo "ns3 fg concurrent: rc=$? $(tail -1 gpurun_out/e2_$i.log)"
done
