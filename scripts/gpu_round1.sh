set -o pipefail
mkdir -p gpurun_out
cd $GRAFT_REPO_ROOT
timeout -k 10 420 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1
echo "pytest rc=$?" >> gpurun_out/gpu_tests.log
tail -5 gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-seconds 5 > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/prof.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/prof.log; exit 1; }
find gpurun_out/prof -name "*stats*" | head
