#!/bin/bash
# BB pass: host-class integration test, throughput, rocprof kernel stats.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/bbox
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_host_class.py tests/test_gpu_bbox.py -x -q --timeout 120 --timeout-method thread > gpurun_out/bbox/tests.log 2>&1 || { tail -30 gpurun_out/bbox/tests.log; exit 1; }
tail -3 gpurun_out/bbox/tests.log
timeout -k 10 180 python -u bench.py --workload bb --config c3 --steps 20 --warmup 3 > gpurun_out/bbox/bench_c3.json 2> gpurun_out/bbox/bench_c3.err || { cat gpurun_out/bbox/bench_c3.err; exit 1; }
cat gpurun_out/bbox/bench_c3.json
timeout -k 10 180 python -u bench.py --workload bb --config c3 --steps 20 --warmup 3 --bb-semantics 1 --no-cpu > gpurun_out/bbox/bench_c3_int.json 2>/dev/null && cat gpurun_out/bbox/bench_c3_int.json
timeout -k 10 180 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/bbox/prof -o bb -- python -u bench.py --workload bb --config c3 --steps 10 --warmup 2 --no-cpu > gpurun_out/bbox/prof.log 2>&1 || { tail -20 gpurun_out/bbox/prof.log; exit 1; }
find gpurun_out/bbox/prof -name "*kernel_stats.csv" | head -1 | xargs cat
