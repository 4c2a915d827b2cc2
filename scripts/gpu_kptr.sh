cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/kp_tests.log 2>&1; rc=$?; echo "parity: $(tail -1 gpurun_out/kp_tests.log)"; [ $rc -eq 0 ] || exit $rc
export LM_ALLOW_QUEUE_SHARING=1
for i in 1 2 3; do
LM_ALLOC=finegrained timeout -k 10 300 python -u scripts/debug_mt.py 3 23 0 > gpurun_out/k1_$i.log 2>&1; echo "ns3 fg concurrent, K by pointer: rc=$? $(tail -1 gpurun_out/k1_$i.log)"
done
