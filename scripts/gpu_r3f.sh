#!/bin/bash
# Tests of the touched kernels, k_nms phase profile, an isolated 1-stream
# kernel trace, and the bench across contexts x lanes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r3f}
[ -n "$NO_TESTS" ] || timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_edges.py tests/test_gpu_pipeline.py tests/test_golden.py > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
LM_KPROF=1 timeout -k 10 120 python bench.py --no-cpu --streams 1 --steps 3 --warmup 1 > gpurun_out/kprof_$TAG.json 2> gpurun_out/kprof_$TAG.txt || { tail -5 gpurun_out/kprof_$TAG.txt; exit 1; }
grep "k_nms bottom\|k_nms side" gpurun_out/kprof_$TAG.txt | tail -2 | cut -c1-300
rm -rf gpurun_out/p1_$TAG
timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/p1_$TAG -o run -- python3 bench.py --streams 1 --steps 12 --warmup 3 --no-cpu > gpurun_out/p1_$TAG.out 2>&1 || { echo "trace failed"; tail -20 gpurun_out/p1_$TAG.out; exit 1; }
python3 - "gpurun_out/p1_$TAG/run_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print(f"{r['Name'].split('(')[0][:28]:28s} {r['Calls']:>6s} {float(r['AverageNs'])/1e3:9.2f} us")
PY
for sl in ${SPLITS:-4x1 1x4 2x2 4x2 6x1}; do
  set -- ${sl/x/ }
  timeout -k 10 240 python bench.py --no-cpu --streams $1 --lanes $2 --steps 40 --warmup 5 > gpurun_out/bench_${TAG}_s$1_l$2.json 2> gpurun_out/bench_${TAG}_s$1_l$2.err \
    || { echo "bench s$1 l$2 failed"; tail -20 gpurun_out/bench_${TAG}_s$1_l$2.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print('bench s$1 l$2', d['value'], 'k_corr', r['avg_launch_ms'], r['frac'], r['algorithmic_frac'])" gpurun_out/bench_${TAG}_s$1_l$2.json
done
for prec in fp32 f16; do
  timeout -k 10 300 python bench.py --no-cpu --config c5 --precision $prec --steps 10 --warmup 2 > gpurun_out/bench_${TAG}_c5_$prec.json 2> gpurun_out/bench_${TAG}_c5_$prec.err \
    || { echo "bench c5 $prec failed"; tail -20 gpurun_out/bench_${TAG}_c5_$prec.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print('bench c5 $prec', d['value'], 'k_corr', r['avg_launch_ms'], r['frac'], r['algorithmic_frac'])" gpurun_out/bench_${TAG}_c5_$prec.json
done
