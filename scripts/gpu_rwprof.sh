#!/bin/bash
# Ring-kernel wave profiles (LM_RW_PROF builds: locomouse_cpp_amd/exp/
# liblocomouse_hip_rwprof*.so, LM_KPROF=1, one stream): how much of each
# correlation launch the SIMDs hold waves, and the pk-FMA issue rate while
# they do -- merged launch (plan 1) and per-width launches (plan 0).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/rwprof
mkdir -p $O
LIB=locomouse_cpp_amd/liblocomouse_hip.so
cp $LIB $O/orig.so
for f in locomouse_cpp_amd/exp/liblocomouse_hip_rwprof*.so; do
  v=$(basename $f .so | sed 's/liblocomouse_hip_//')
  cp $f $LIB
  for plan in ${PLANS:-1 0}; do
    LM_CORR_PLAN=$plan LM_KPROF=1 timeout -k 10 240 python3 bench.py --streams 1 --steps 3 --warmup 1 --no-cpu --no-check > $O/$v.plan$plan.json 2> $O/$v.plan$plan.txt || { echo "$v plan $plan failed"; tail -5 $O/$v.plan$plan.txt; cp $O/orig.so $LIB; exit 1; }
    grep "rwprof" $O/$v.plan$plan.txt | tail -2 | sed "s/^/$v plan$plan /"
  done
done
cp $O/orig.so $LIB
