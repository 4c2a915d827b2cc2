#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, kernel trace only) over a short
# 1-stream bench, for each VARIANTS entry "name:ENV=val,..." (env set for the profiled run).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
for v in ${VARIANTS:-default:}; do
  name=${v%%:*}; envs=${v#*:}
  for e in ${envs//,/ }; do export "$e"; done
  mkdir -p gpurun_out/pmc_$name
  i=0
  while read -r line; do
    [ -z "$line" ] && continue
    i=$((i+1))
    timeout -k 10 120 rocprofv3 --kernel-trace --pmc $line -f csv -d gpurun_out/pmc_$name/p$i -o run -- python bench.py ${PMC_BENCH_ARGS:---steps 4 --warmup 1 --no-cpu --no-check --batch 256 --streams 1} > gpurun_out/pmc_$name/p$i.log 2>&1 || { echo "$name pass $i failed: $line"; tail -5 gpurun_out/pmc_$name/p$i.log; exit 1; }
    echo "$name pass $i ok"
  done < "${PMC_FILE:-scripts/pmc_corr.txt}"
  python scripts/pmc_summary.py gpurun_out/pmc_$name k_corr > gpurun_out/pmc_$name/summary.txt
  for e in ${envs//,/ }; do unset "${e%%=*}"; done
done
