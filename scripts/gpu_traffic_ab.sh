#!/bin/bash
# HBM traffic of the correlation per experiment library: for the in-tree
# library ("base") and each locomouse_cpp_amd/exp/liblocomouse_hip_<v>.so,
# one --pmc pass per counter set (FETCH_SIZE; WRITE_SIZE; TCC_HIT_sum
# TCC_MISS_sum), kernel trace only, then scripts/pmc_traffic.py.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/traffic
mkdir -p $O
LIB=locomouse_cpp_amd/liblocomouse_hip.so
cp $LIB $O/orig.so
cp $LIB locomouse_cpp_amd/exp/liblocomouse_hip_base.so
for f in locomouse_cpp_amd/exp/liblocomouse_hip_*.so; do
  v=$(basename $f .so | sed 's/liblocomouse_hip_//')
  cp $f $LIB
  i=0
  for c in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum"; do
    i=$((i+1))
    rm -rf $O/$v/p$i
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c -f csv -d $O/$v/p$i -o run -- python3 bench.py --steps 4 --warmup 1 --no-cpu --no-check > $O/$v.p$i.out 2>&1 || { echo "$v pass $c failed"; tail -5 $O/$v.p$i.out; cp $O/orig.so $LIB; exit 1; }
  done
  mkdir -p $O/$v/pmc && cp -r $O/$v/p1 $O/$v/pmc/FETCH_SIZE && cp -r $O/$v/p2 $O/$v/pmc/WRITE_SIZE
  python3 scripts/pmc_traffic.py $O/$v/pmc ${TRAFFIC_BATCH:-448} $O/$v/pmc_k_corr.json > $O/$v/traffic.txt && echo "$v" && tail -3 $O/$v/traffic.txt
  python3 - $O/$v/p3 <<'PY'
import csv, glob, sys
from collections import defaultdict
d = defaultdict(lambda: defaultdict(float)); n = defaultdict(int)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0]
        if "k_corr" in k:
            d[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, c in d.items():
    h, m = c.get("TCC_HIT_sum", 0), c.get("TCC_MISS_sum", 0)
    print(f"  {k}: L2 hit {h:.0f} miss {m:.0f} hit-rate {h / max(1, h + m):.3f}")
PY
done
cp $O/orig.so $LIB
