#!/bin/bash
# bench.py over a few (streams, batch) settings, one line each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/sweep
# SWEEP: "streams:batch streams:batch ..."
for sb in ${SWEEP:-3:256 4:256 2:256 3:384 4:192 6:128}; do
  set -- ${sb/:/ }
  timeout -k 10 200 python bench.py --no-cpu --streams $1 --batch $2 --steps ${STEPS:-30} --warmup 5 > gpurun_out/sweep/s$1_b$2.json 2> gpurun_out/sweep/s$1_b$2.err || { echo "s$1 b$2 failed"; tail -3 gpurun_out/sweep/s$1_b$2.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print('streams', sys.argv[2], 'batch', sys.argv[3], d['value'], 'k_corr', d['roofline']['avg_launch_ms'])" gpurun_out/sweep/s$1_b$2.json $1 $2
done
