#!/bin/bash
# Kernel phase profiles (LM_KPROF=1, one stream) of the in-tree library
# ("base") and of each experiment library, installed in turn.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/kprof_ab
mkdir -p $O
LIB=locomouse_cpp_amd/liblocomouse_hip.so
cp $LIB $O/orig.so
cp $LIB locomouse_cpp_amd/exp/liblocomouse_hip_base.so
for f in locomouse_cpp_amd/exp/liblocomouse_hip_*.so; do
  v=$(basename $f .so | sed 's/liblocomouse_hip_//')
  cp $f $LIB
  LM_KPROF=1 timeout -k 10 240 python3 bench.py --streams 1 --steps 3 --warmup 1 --no-cpu --no-check > $O/$v.json 2> $O/$v.txt || { echo "$v failed"; tail -5 $O/$v.txt; cp $O/orig.so $LIB; exit 1; }
  grep -E "${KPROF_PAT:-kprof k_ingest}" $O/$v.txt | tail -2 | sed "s/^/$v /"
done
cp $O/orig.so $LIB
