"""From a rocprofv3 --kernel-trace CSV: per kernel family, dispatch count,
mean dispatch duration and the union of the dispatch intervals (overlapping
streams counted once) -- the rocprof-side counterpart of bench.py's
roofline.avg_launch_ms (union of k_corr spans / launches; one launch = the
4 width-group k_corr dispatches of a batch).

Usage: python scripts/prof_union.py <run_kernel_trace.csv> [groups_per_launch=4] [skip_launches=0]
"""
import csv
import sys
from collections import defaultdict


def union(iv):
    tot, end = 0, None
    for a, b in sorted(iv):
        if end is None or a > end:
            tot += b - a
            end = b
        elif b > end:
            tot += b - end
            end = b
    return tot


def main(path, per_launch=4, skip=0):
    per_launch, skip = int(per_launch), int(skip)
    fam = defaultdict(list)
    with open(path) as fh:
        for r in csv.DictReader(fh):
            name = r["Kernel_Name"].split("(")[0].split("<")[0].replace("void ", "").strip()
            fam[name].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    print(f"{'kernel':16s} {'dispatches':>10s} {'mean_us':>10s} {'union_us':>12s}")
    for k in sorted(fam, key=lambda k: -sum(b - a for a, b in fam[k])):
        iv = sorted(fam[k])
        print(f"{k:16s} {len(iv):10d} {sum(b - a for a, b in iv) / len(iv) / 1e3:10.2f} {union(iv) / 1e3:12.1f}")
    corr = sorted(fam.get("k_corr_rw", []) or fam.get("k_corr_pk", []) or fam.get("k_corr", []))[skip * per_launch:]
    if corr:
        n = len(corr) / per_launch
        print(f"k_corr launches {n:.0f}: union per launch {union(corr) / n / 1e6:.5f} ms, "
              f"mean launch (sum of dispatches) {sum(b - a for a, b in corr) / n / 1e6:.5f} ms")


if __name__ == "__main__":
    main(*sys.argv[1:])
