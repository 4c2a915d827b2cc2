#!/bin/bash
# Round-6: k_nms tie blocks with issue priority (LM_NMS_TIE_PRIO=3, p3) vs
# without (p0): parity tests on p3, the k_nms phase profile alone (one
# stream, LM_KPROF=1), then frames/s at the default shape, checked.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r6j
E=locomouse_cpp_amd/exp
mkdir -p $O /tmp/held
cp locomouse_cpp_amd/liblocomouse_hip.so /tmp/orig_lib.so
cp $E/liblocomouse_hip_p3.so locomouse_cpp_amd/liblocomouse_hip.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_parity_p3.log 2>&1
rc=$?; cp /tmp/orig_lib.so locomouse_cpp_amd/liblocomouse_hip.so; tail -2 $O/gpu_parity_p3.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $O/gpu_parity_p3.log | head; exit $rc; }
mv $E/liblocomouse_hip_r5.so /tmp/held/
KPROF_PAT="kprof k_nms" bash scripts/gpu_kprof_ab.sh > $O/kprof_ab.txt 2>&1; rc=$?
mv /tmp/held/*.so $E/; rm -f $E/liblocomouse_hip_base.so
cat $O/kprof_ab.txt; [ $rc -eq 0 ] || exit $rc
CHECK=1 TAG=r6j REPS=3 VARIANTS="p0:p0: p3:p3:" bash scripts/gpu_ab_combo.sh
