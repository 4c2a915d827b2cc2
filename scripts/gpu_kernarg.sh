cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export LM_ALLOW_QUEUE_SHARING=1
for i in 1 2 3; do
HIP_FORCE_DEV_KERNARG=0 LM_ALLOC=finegrained timeout -k 10 300 python -u scripts/debug_mt.py 3 23 0 > gpurun_out/ka_$i.log 2>&1; echo "ns3 fg HIP_FORCE_DEV_KERNARG=0: rc=$? $(tail -1 gpurun_out/ka_$i.log)"
LM_ALLOC=finegrained timeout -k 10 300 python -u scripts/debug_mt.py 3 23 0 > gpurun_out/kb_$i.log 2>&1; echo "ns3 fg default: rc=$? $(tail -1 gpurun_out/kb_$i.log)"
done
