#!/bin/bash
# Round-6: rocprof kernel trace of the C4 whole-video pass at the default
# shape (where the pass loses time against the stream), and the k_nms phase
# profile alone at 256-frame batches (the size the verdict's target uses).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r6n
mkdir -p $O
rm -rf $O/prof
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $O/prof -o run -- python3 bench.py --video-frames 10000 --steps 3 --warmup 2 --no-cpu --no-check > $O/prof.out 2>&1 || { tail -20 $O/prof.out; exit 1; }
tail -c 300 $O/prof.out
LM_KPROF=1 timeout -k 10 240 python3 bench.py --streams 1 --batch 256 --steps 3 --warmup 1 --no-cpu --no-check > $O/kprof256.json 2> $O/kprof256.txt || { tail -5 $O/kprof256.txt; exit 1; }
grep "kprof k_nms" $O/kprof256.txt | tail -2
