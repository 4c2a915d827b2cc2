cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export LM_ALLOW_QUEUE_SHARING=1
for i in 1 2; do
LM_SERIALIZE=1 timeout -k 10 300 python -u scripts/debug_mt.py 3 23 0 > gpurun_out/s1_$i.log 2>&1; echo "ns3 serialized: rc=$? $(tail -1 gpurun_out/s1_$i.log)"
timeout -k 10 300 python -u scripts/debug_mt.py 3 23 0 > gpurun_out/s2_$i.log 2>&1; echo "ns3 concurrent: rc=$? $(tail -1 gpurun_out/s2_$i.log)"
done
