#!/bin/bash
# Round-6: k_nms blocks with long lists take issue priority (b128: n >= 128,
# b256: n >= 256) vs base: parity tests on b256, the phase profile alone at
# 256-frame batches, then frames/s at the default shape, checked.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r6q
E=locomouse_cpp_amd/exp
mkdir -p $O
cp locomouse_cpp_amd/liblocomouse_hip.so /tmp/orig_lib.so
cp $E/liblocomouse_hip_b256.so locomouse_cpp_amd/liblocomouse_hip.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_parity_b256.log 2>&1
rc=$?; cp /tmp/orig_lib.so locomouse_cpp_amd/liblocomouse_hip.so; tail -2 $O/gpu_parity_b256.log; [ $rc -eq 0 ] || exit $rc
for v in base b128 b256; do
  [ $v = base ] || cp $E/liblocomouse_hip_$v.so locomouse_cpp_amd/liblocomouse_hip.so
  LM_KPROF=1 timeout -k 10 240 python3 bench.py --streams 1 --batch 256 --steps 3 --warmup 1 --no-cpu --no-check > $O/$v.json 2> $O/$v.txt || { tail -5 $O/$v.txt; cp /tmp/orig_lib.so locomouse_cpp_amd/liblocomouse_hip.so; exit 1; }
  cp /tmp/orig_lib.so locomouse_cpp_amd/liblocomouse_hip.so
  grep "kprof k_nms" $O/$v.txt | tail -4 | sed "s/^/$v /"
done
CHECK=1 TAG=r6q REPS=3 VARIANTS="base:base: b128:b128: b256:b256:" bash scripts/gpu_ab_combo.sh
