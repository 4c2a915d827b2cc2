cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
summ='import json,sys; d=json.load(sys.stdin); print(d["n_gpus"], d["config"]["streams_per_gpu"], d["value"], "corr_ms", d["roofline"]["avg_launch_ms"], "TF", d["roofline"]["achieved"], d["kernel_busy_ms_per_batch"])'
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_c5.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -4 gpurun_out/gpu_tests_c5.log; [ $rc -eq 0 ] || exit $rc
echo -n "c3 s2: "; timeout -k 10 200 python bench.py --steps 40 --warmup 5 --no-cpu > gpurun_out/b_c3.json 2>gpurun_out/b_c3.err && python -c "$summ" < gpurun_out/b_c3.json || exit 1
echo -n "c3 s1: "; timeout -k 10 200 python bench.py --steps 40 --warmup 5 --no-cpu --streams 1 > gpurun_out/b_c3s1.json 2>gpurun_out/b_c3s1.err && python -c "$summ" < gpurun_out/b_c3s1.json || exit 1
echo -n "c5 s2: "; timeout -k 10 300 python bench.py --config c5 --steps 20 --warmup 3 --no-cpu --resident 1600 > gpurun_out/b_c5.json 2>gpurun_out/b_c5.err && python -c "$summ" < gpurun_out/b_c5.json || { tail -5 gpurun_out/b_c5.err; exit 1; }
echo -n "N=2 rehearsal: "; timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 3 --no-cpu > gpurun_out/b_n2.json 2>gpurun_out/b_n2.err && python -c "$summ" < gpurun_out/b_n2.json || { tail -20 gpurun_out/b_n2.err; exit 1; }
