#!/bin/bash
# Throughput sweep of bench.py's context / lane / batch shape (no CPU legs,
# no oracle check): SWEEP="streams:lanes:batch ..." REPS=n
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/sweep
mkdir -p $O
for rep in $(seq 1 ${REPS:-2}); do
  for cfg in ${SWEEP:-4:1:256 5:1:256 6:1:256 4:1:384 3:1:384}; do
    IFS=: read st ln b <<< "$cfg"
    timeout -k 10 180 python3 bench.py --no-cpu --no-check --streams $st --lanes $ln --batch $b ${BENCH_ARGS:---steps 40 --warmup 5} > $O/$st-$ln-$b.$rep.json 2> $O/$st-$ln-$b.$rep.err || { echo "$cfg failed"; tail -3 $O/$st-$ln-$b.$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/$st-$ln-$b.$rep.json')); print('$cfg', $rep, round(d['value']), d['roofline']['avg_launch_ms'])"
  done
done
