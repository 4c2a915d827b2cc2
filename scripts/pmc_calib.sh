#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration per access width (scripts/ubench/fetch_calib.hip)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/calib
rm -rf $OUT && mkdir -p $OUT
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 60 rocprofv3 --kernel-trace --pmc $c -f csv -d $OUT/$c -o run -- ./scripts/ubench/fetch_calib > $OUT/$c.log 2>&1 || { echo "calib $c failed"; tail -5 $OUT/$c.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, json
from collections import defaultdict
res = {}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    f = glob.glob(f"gpurun_out/calib/{c}/**/*counter_collection.csv", recursive=True)[0]
    d = defaultdict(list)
    for r in csv.DictReader(open(f)):
        d[r["Kernel_Name"].split("(")[0]].append(float(r["Counter_Value"]))
    for k, v in d.items():
        res.setdefault(k, {})[c + "_bytes"] = sum(v) / len(v) * 1024
B = 1 << 30
out = {"bytes_per_dispatch": B, "note": "counter bytes (KiB x 1024) / distinct bytes touched", "ratios": {}}
for k, v in sorted(res.items()):
    key = "FETCH_SIZE_bytes" if k.startswith("rd") else "WRITE_SIZE_bytes"
    out["ratios"][k] = round(v.get(key, 0) / B, 4)
out["raw"] = res
json.dump(out, open("gpurun_out/calib/fetch_calib.json", "w"), indent=1)
print(json.dumps(out["ratios"]))
PY
