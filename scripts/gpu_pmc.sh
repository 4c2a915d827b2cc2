#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, kernel trace only) over a short bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
rocprofv3 -L > gpurun_out/pmc/counters_list.txt 2>&1 || true
i=0
while read -r line; do
  [ -z "$line" ] && continue
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $line -f csv -d gpurun_out/pmc/p$i -o run -- python bench.py --steps 4 --warmup 1 --no-cpu --batch 256 --streams 1 > gpurun_out/pmc/p$i.log 2>&1 || { echo "pass $i failed: $line"; tail -5 gpurun_out/pmc/p$i.log; exit 1; }
  echo "pass $i ok: $line"
done < "${PMC_FILE:-scripts/pmc_sets.txt}"
