#!/bin/bash
# Round-6: correlation HBM traffic at the default shape (8 contexts x 448)
# for this tree (XCD runs of 16 workgroups), runs of 32 and 64, and round 5's
# library; then the per-width ring kernels alone (one stream, LM_CORR_PLAN=0).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r6h
mkdir -p $O
bash scripts/gpu_traffic_ab.sh > $O/traffic_ab.txt 2>&1 || { tail -5 $O/traffic_ab.txt; exit 1; }
cat $O/traffic_ab.txt
rm -f locomouse_cpp_amd/exp/liblocomouse_hip_x32.so locomouse_cpp_amd/exp/liblocomouse_hip_x64.so locomouse_cpp_amd/exp/liblocomouse_hip_base.so
LM_CORR_PLAN=0 KERNELS="k_corr" bash scripts/gpu_kstats_ab.sh > $O/kstats_perwidth_streams1.txt 2>&1 || { tail -5 $O/kstats_perwidth_streams1.txt; exit 1; }
grep -v "^\[" $O/kstats_perwidth_streams1.txt | sort -k2,2 -k1,1
