cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export LM_ALLOW_QUEUE_SHARING=1
for i in 1 2 3; do
for m in 3 4; do
LM_SERIALIZE=$m LM_ALLOC=finegrained timeout -k 10 300 python -u scripts/debug_mt.py 3 23 0 > gpurun_out/m${m}_$i.log 2>&1; echo "ns3 fg mode $m: rc=$? $(tail -1 gpurun_out/m${m}_$i.log)"
done; done
