#!/bin/bash
# Experiment library: locomouse_cpp_amd/exp/liblocomouse_hip_<name>.so from a
# given correlation source (default: the in-tree lm_corr.hip) and -D flags,
# linked with the in-tree runtime and BB objects (build/hip, from
# runtime.build()).  For A/B runs with scripts/gpu_ab_lib.sh.
#   scripts/build_variant.sh <name> [corr_source.hip] [-DFOO=1 ...]
set -e
cd "$(dirname "$0")/.."
name=$1; shift
src=locomouse_cpp_amd/csrc/lm_corr.hip
if [ $# -gt 0 ] && [[ "$1" != -* ]]; then src=$1; shift; fi
mkdir -p locomouse_cpp_amd/exp build/var
obj=build/var/lm_corr_$name.o
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize -fvisibility=hidden -Wall \
  -Wno-unused-function -Wno-unused-variable -Iinclude -Ilocomouse_cpp_amd/csrc "$@" -c -o $obj $src
hipcc --offload-arch=gfx950 -shared -fPIC -o locomouse_cpp_amd/exp/liblocomouse_hip_$name.so \
  build/hip/lm_runtime.o $obj build/hip/lm_bbox.o
echo "locomouse_cpp_amd/exp/liblocomouse_hip_$name.so"
