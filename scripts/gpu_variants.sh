# Parity + per-width rocprof durations + bench for several correlation variants.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
summ='import json,sys; d=json.load(sys.stdin); print(d["config"]["streams_per_gpu"], d["value"], "corr_ms", d["roofline"]["avg_launch_ms"], "TF", d["roofline"]["achieved"])'
for v in ${VARS:-3}; do
  LM_CORR_VARIANT=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/var_tests_$v.log 2>&1; rc=$?
  echo "variant $v parity: $(tail -1 gpurun_out/var_tests_$v.log)"; [ $rc -eq 0 ] || exit $rc
  rm -rf gpurun_out/vprof_$v
  LM_CORR_VARIANT=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/vprof_$v -o run -- python bench.py --steps 10 --warmup 2 --no-cpu --streams 1 > gpurun_out/vprof_$v.out 2>&1 || { echo "prof $v failed"; exit 1; }
  python -c "
import csv
for r in csv.DictReader(open('gpurun_out/vprof_$v/run_kernel_stats.csv')):
    if 'k_corr' in r['Name']: print('   ', r['Name'].split('(')[0][:34], round(float(r['AverageNs'])/1e3,1), 'us')"
  echo -n "   bench s2: "; LM_CORR_VARIANT=$v timeout -k 10 200 python bench.py --steps 30 --warmup 3 --no-cpu 2>gpurun_out/vbench_$v.err | python -c "$summ" || { tail -3 gpurun_out/vbench_$v.err; exit 1; }
done
