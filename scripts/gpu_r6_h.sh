#!/bin/bash
# Round-6: correlation HBM traffic at the default shape (8 contexts x 448)
# for this tree (XCD runs of 16 workgroups), runs of 32 and 64, and round 5's
# library; the per-width ring kernels alone (one stream, LM_CORR_PLAN=0);
# then workgroups of 1, 2 and 8 waves against 4 (LDS now sized by the
# correlation unit itself), each line checked against the oracle.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r6h
mkdir -p $O /tmp/wlibs
E=locomouse_cpp_amd/exp
mv $E/liblocomouse_hip_w*.so /tmp/wlibs/
bash scripts/gpu_traffic_ab.sh > $O/traffic_ab.txt 2>&1 || { tail -5 $O/traffic_ab.txt; exit 1; }
cat $O/traffic_ab.txt
rm -f $E/liblocomouse_hip_x32.so $E/liblocomouse_hip_x64.so $E/liblocomouse_hip_base.so
LM_CORR_PLAN=0 KERNELS="k_corr" bash scripts/gpu_kstats_ab.sh > $O/kstats_perwidth_streams1.txt 2>&1 || { tail -5 $O/kstats_perwidth_streams1.txt; exit 1; }
grep -v "^\[" $O/kstats_perwidth_streams1.txt | sort -k2,2 -k1,1
rm -f $E/liblocomouse_hip_base.so
mv /tmp/wlibs/*.so $E/
CHECK=1 TAG=r6h REPS=2 VARIANTS="base:base: w1:w1: w2:w2: w8:w8:" bash scripts/gpu_ab_combo.sh
# f16 (C5, non-parity): 2 x 2 waves of two x-adjacent tiles (build/var_src/lm_corr_xt.hip) vs 4 x 1;
# the f16 GPU tests on the variant first (exact on f16-representable detectors)
cp locomouse_cpp_amd/liblocomouse_hip.so /tmp/orig_lib.so
cp $E/liblocomouse_hip_xt.so locomouse_cpp_amd/liblocomouse_hip.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_f16.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_f16_xt.log 2>&1
rc=$?; cp /tmp/orig_lib.so locomouse_cpp_amd/liblocomouse_hip.so; tail -2 $O/gpu_f16_xt.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $O/gpu_f16_xt.log | head; exit $rc; }
TAG=r6hf REPS=3 BENCH_ARGS="--config c5 --precision f16 --streams 8 --steps 12 --warmup 2" VARIANTS="base:base: xt:xt:" bash scripts/gpu_ab_combo.sh
