#!/bin/bash
# A/B of (library, environment) combinations on one box, REPS rounds:
#   VARIANTS="name:lib:ENV=val,ENV2=val ..."  lib = base (the in-tree library)
#   or the <v> of locomouse_cpp_amd/exp/liblocomouse_hip_<v>.so
# Each runs bench.py (no CPU legs; no parity check unless CHECK=1, then a
# line whose timed batches differ from the oracle fails the run) with BENCH_ARGS; the
# in-tree library is restored at the end.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
LIB=locomouse_cpp_amd/liblocomouse_hip.so
cp $LIB gpurun_out/ab/orig.so
TAG=${TAG:-combo}
NOCHK=--no-check
[ -n "$CHECK" ] && NOCHK=
for rep in $(seq 1 ${REPS:-2}); do
for v in $VARIANTS; do
  name=${v%%:*}; rest=${v#*:}; lib=${rest%%:*}; envs=${rest#*:}
  if [ "$lib" = base ]; then cp gpurun_out/ab/orig.so $LIB; else cp locomouse_cpp_amd/exp/liblocomouse_hip_$lib.so $LIB; fi
  timeout -k 10 180 env ${envs//,/ } python3 bench.py --no-cpu $NOCHK ${BENCH_ARGS:---steps 40 --warmup 5} > gpurun_out/ab/${TAG}_$name.$rep.json 2> gpurun_out/ab/${TAG}_$name.$rep.err || { echo "$name failed"; tail -5 gpurun_out/ab/${TAG}_$name.$rep.err; cp gpurun_out/ab/orig.so $LIB; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/ab/${TAG}_$name.$rep.json')); r=d['roofline']; print('$name', '$rep', d['value'], d['ms_per_step'], r['avg_launch_ms'], r['frac'])"
done
done
cp gpurun_out/ab/orig.so $LIB
