#!/bin/bash
# Per-kernel average durations (rocprofv3 kernel trace, one stream, no CPU
# legs) of each experiment library locomouse_cpp_amd/exp/liblocomouse_hip_<v>.so
# and of the in-tree one ("base"), installed in turn as the product library.
#   KERNELS="k_ingest k_corr" bash scripts/gpu_kstats_ab.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/kstats
mkdir -p $O
LIB=locomouse_cpp_amd/liblocomouse_hip.so
cp $LIB $O/orig.so
cp $LIB locomouse_cpp_amd/exp/liblocomouse_hip_base.so
for f in locomouse_cpp_amd/exp/liblocomouse_hip_*.so; do
  v=$(basename $f .so | sed 's/liblocomouse_hip_//')
  cp $f $LIB
  rm -rf $O/$v
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -f csv -d $O/$v -o run -- python3 bench.py ${BENCH_ARGS:---streams 1 --steps 6 --warmup 2 --no-cpu --no-check} > $O/$v.out 2>&1 || { echo "$v failed"; tail -5 $O/$v.out; cp $O/orig.so $LIB; exit 1; }
  python3 - $O/$v/run_kernel_stats.csv $v ${KERNELS:-k_ingest} <<'PY'
import csv, sys
path, v, pats = sys.argv[1], sys.argv[2], sys.argv[3:]
for r in csv.DictReader(open(path)):
    n = r["Name"].split("(")[0]
    if any(p in n for p in pats):
        print(v, n, r["Calls"], round(float(r["AverageNs"]) / 1e3, 2), "us")
PY
done
cp $O/orig.so $LIB
