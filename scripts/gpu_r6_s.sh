#!/bin/bash
# Round-6: the default C3 shape re-checked on the final kernels: 8 x 448
# (default) vs 8 x 512 vs 10 x 448, every line checked.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
for rep in 1 2 3; do
  for v in 8:448 8:512 10:448; do
    IFS=: read ns nb <<< "$v"
    timeout -k 10 180 python3 bench.py --no-cpu --streams $ns --batch $nb --steps 40 --warmup 5 > gpurun_out/ab/r6s_${ns}x${nb}.$rep.json 2> gpurun_out/ab/r6s_${ns}x${nb}.$rep.err || { tail -5 gpurun_out/ab/r6s_${ns}x${nb}.$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/ab/r6s_${ns}x${nb}.$rep.json')); print('${ns}x${nb}', $rep, d['value'], d['roofline']['frac'], d['parity_sample']['bit_exact'])"
  done
done
