# After the k_nms tie-path fix: GPU tests, multi-context stress, streams x batch sweep.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/pf
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pf/gpu_tests.log 2>&1; rc=$?; echo "gpu tests: $(tail -1 gpurun_out/pf/gpu_tests.log)"; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_mt_stress.sh || exit 1
summ='import json,sys; d=json.load(sys.stdin); r=d["roofline"]; print(d["config"]["streams_per_gpu"], d["config"]["batch_frames"], d["value"], "corr_ms", r["avg_launch_ms"], "TF", r["achieved"])'
for ns in 1 2 3; do for b in 256 512; do
  echo -n "streams $ns batch $b: "; timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu --streams $ns --batch $b 2>gpurun_out/pf/b_${ns}_$b.err | python -c "$summ" || { tail -3 gpurun_out/pf/b_${ns}_$b.err; exit 1; }
done; done
