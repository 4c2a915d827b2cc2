#!/bin/bash
# Experiment library with a runtime translation unit (lm_runtime.hip, which
# holds the non-correlation kernels) built with extra -D flags, linked with
# the in-tree correlation and BB objects (build/hip, from runtime.build()):
# locomouse_cpp_amd/exp/liblocomouse_hip_<name>.so, for scripts/gpu_ab_lib.sh.
#   scripts/build_variant_rt.sh <name> [-DFOO=1 ...]
set -e
cd "$(dirname "$0")/.."
name=$1; shift
mkdir -p locomouse_cpp_amd/exp build/var
obj=build/var/lm_runtime_$name.o
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize -fvisibility=hidden -Wall \
  -Wno-unused-function -Wno-unused-variable -Iinclude -Ilocomouse_cpp_amd/csrc "$@" -c -o $obj locomouse_cpp_amd/csrc/lm_runtime.hip
hipcc --offload-arch=gfx950 -shared -fPIC -o locomouse_cpp_amd/exp/liblocomouse_hip_$name.so \
  $obj build/hip/lm_corr.o build/hip/lm_bbox.o
echo "locomouse_cpp_amd/exp/liblocomouse_hip_$name.so"
