# Checks the per-device enqueue serialisation: multi-context runs that used to
# corrupt batches, then the GPU test suite and benches at 1-3 streams.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/fix
for i in 1 2 3; do
LM_ALLOC=finegrained timeout -k 10 300 python -u scripts/debug_mt.py 3 23 0 > gpurun_out/fix/fg_ns3_$i.log 2>&1; echo "ns3 finegrained: rc=$? $(tail -1 gpurun_out/fix/fg_ns3_$i.log)"
done
for i in 1 2; do
timeout -k 10 300 python -u scripts/debug_mt.py 4 20 0 > gpurun_out/fix/ns4_$i.log 2>&1; echo "ns4 default: rc=$? $(tail -1 gpurun_out/fix/ns4_$i.log)"
LM_CORR_VARIANT=8 timeout -k 10 300 python -u scripts/debug_mt.py 2 23 0 > gpurun_out/fix/v8_ns2_$i.log 2>&1; echo "ns2 variant 8: rc=$? $(tail -1 gpurun_out/fix/v8_ns2_$i.log)"
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/fix/gpu_tests.log 2>&1; rc=$?; echo "gpu tests: $(tail -1 gpurun_out/fix/gpu_tests.log)"; [ $rc -eq 0 ] || exit $rc
summ='import json,sys; d=json.load(sys.stdin); print(d["config"]["streams_per_gpu"], d["value"], "corr_ms", d["roofline"]["avg_launch_ms"], "TF", d["roofline"]["achieved"])'
for ns in 1 2 3 4; do
  echo -n "bench streams $ns: "; timeout -k 10 200 python bench.py --steps 30 --warmup 3 --no-cpu --streams $ns 2>gpurun_out/fix/b$ns.err | python -c "$summ" || { tail -3 gpurun_out/fix/b$ns.err; exit 1; }
done
