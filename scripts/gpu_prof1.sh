#!/bin/bash
# Isolated kernel profile (one stream per GPU, so dispatches do not share the
# chip): rocprofv3 kernel trace + stats, then one PMC pass per line of
# $PMC_FILE (kernel trace only, each pass its own time limit).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
TAG=${TAG:-p1}
OUT=gpurun_out/$TAG
rm -rf $OUT && mkdir -p $OUT
ARGS=${PROF_ARGS:---streams 1 --steps 12 --warmup 3 --no-cpu --no-check}
timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o run -- python3 bench.py $ARGS > $OUT/trace.out 2>&1 || { echo "trace failed"; tail -20 $OUT/trace.out; exit 1; }
cat $OUT/trace/run_kernel_stats.csv | cut -c1-160
python3 scripts/prof_union.py $OUT/trace/run_kernel_trace.csv 4 3 > $OUT/union.txt && cat $OUT/union.txt
[ -n "$NO_PMC" ] && exit 0
i=0
while read -r line; do
  [ -z "$line" ] && continue
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $line -f csv -d $OUT/p$i -o run -- python3 bench.py ${PMC_BENCH_ARGS:---streams 1 --steps 3 --warmup 1 --no-cpu --no-check} > $OUT/p$i.log 2>&1 || { echo "pass $i failed: $line"; tail -5 $OUT/p$i.log; exit 1; }
  echo "pass $i ok: $line"
done < "${PMC_FILE:-scripts/pmc_k_corr.txt}"
python3 scripts/pmc_summary.py $OUT > $OUT/pmc_summary.txt && cat $OUT/pmc_summary.txt
