# A/B of correlation variants: parity under the candidate variant, then
# interleaved benches (streams 1) and one streams-2 bench each.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
V=${V:-6}
summ='import json,sys; d=json.load(sys.stdin); print(d["config"]["streams_per_gpu"], d["value"], "corr_ms", d["roofline"]["avg_launch_ms"], "TF", d["roofline"]["achieved"])'
LM_CORR_VARIANT=$V timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/var_tests.log 2>&1; rc=$?
tail -2 gpurun_out/var_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do for v in 3 $V; do
  echo -n "variant $v s1 round $r: "; LM_CORR_VARIANT=$v timeout -k 10 200 python bench.py --steps 30 --warmup 3 --no-cpu --streams 1 2>/dev/null | python -c "$summ" || exit 1
done; done
for v in 3 $V; do
  echo -n "variant $v s2: "; LM_CORR_VARIANT=$v timeout -k 10 200 python bench.py --steps 30 --warmup 3 --no-cpu 2>/dev/null | python -c "$summ" || exit 1
  echo -n "variant $v c5: "; LM_CORR_VARIANT=$v timeout -k 10 200 python bench.py --config c5 --steps 10 --warmup 2 --no-cpu --resident 800 2>/dev/null | python -c "$summ" || exit 1
done
