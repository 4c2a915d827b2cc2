cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r01d
for i in 1 2; do
timeout -k 10 300 python -u scripts/debug_mt.py 4 20 0 > gpurun_out/r01d/mt4_$i.log 2>&1; echo "ns4 serialized default: rc=$? $(tail -1 gpurun_out/r01d/mt4_$i.log)"
done
TAG=r01d bash scripts/gpu_round.sh
