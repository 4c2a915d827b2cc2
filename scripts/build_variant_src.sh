#!/bin/bash
# Experiment library from a modified copy of the sources: the in-tree csrc/
# with the given files replaced, all three translation units compiled (with
# optional -D flags) into locomouse_cpp_amd/exp/liblocomouse_hip_<name>.so.
#   scripts/build_variant_src.sh <name> <file.hip|.h>=<replacement path> ... [-DFOO=1 ...]
set -e
cd "$(dirname "$0")/.."
name=$1; shift
src=build/var_src/$name
rm -rf $src && mkdir -p $src && cp locomouse_cpp_amd/csrc/* $src/
defs=()
for a in "$@"; do
  if [[ "$a" == -* ]]; then defs+=("$a"); else cp "${a#*=}" "$src/${a%%=*}"; fi
done
mkdir -p locomouse_cpp_amd/exp build/var/$name
objs=()
for u in lm_runtime lm_corr lm_bbox; do
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize -fvisibility=hidden -Wall \
    -Wno-unused-function -Wno-unused-variable -Iinclude -I$src "${defs[@]}" -c -o build/var/$name/$u.o $src/$u.hip &
  objs+=(build/var/$name/$u.o)
done
wait
hipcc --offload-arch=gfx950 -shared -fPIC -o locomouse_cpp_amd/exp/liblocomouse_hip_$name.so "${objs[@]}"
echo "locomouse_cpp_amd/exp/liblocomouse_hip_$name.so"
