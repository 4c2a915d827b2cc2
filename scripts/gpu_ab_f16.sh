#!/bin/bash
# C5 f16 (non-parity) throughput A/B of the experiment libraries against the
# in-tree one: frames/s, k_corr ms per launch, frac of the dense f16 peak.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/ab_f16
mkdir -p $O
LIB=locomouse_cpp_amd/liblocomouse_hip.so
cp $LIB $O/orig.so
cp $LIB locomouse_cpp_amd/exp/liblocomouse_hip_base.so
for rep in $(seq 1 ${REPS:-2}); do
  for f in locomouse_cpp_amd/exp/liblocomouse_hip_*.so; do
    v=$(basename $f .so | sed 's/liblocomouse_hip_//')
    cp $f $LIB
    timeout -k 10 300 python3 bench.py --config c5 --precision f16 --streams ${STREAMS:-8} --steps 8 --warmup 2 --no-cpu --no-check > $O/$v.$rep.json 2> $O/$v.$rep.err || { echo "$v failed"; tail -5 $O/$v.$rep.err; cp $O/orig.so $LIB; exit 1; }
    python3 -c "
import json,sys
d=json.loads(open('$O/$v.$rep.json').read().strip().splitlines()[-1])
print('$v', $rep, d['value'], d['roofline']['avg_launch_ms'], d['roofline']['frac'])"
  done
done
cp $O/orig.so $LIB
rm -f locomouse_cpp_amd/exp/liblocomouse_hip_base.so
