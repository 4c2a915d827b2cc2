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
        # timeline over the window of the counted k_corr launches: how much of
        # it any kernel ran, k_corr ran, or the GPU had no kernel at all
        t0, t1 = corr[0][0], max(b for _, b in corr)
        clip = lambda iv: [(max(a, t0), min(b, t1)) for a, b in iv if b > t0 and a < t1]
        allk = clip([x for k, v in fam.items() if k != "k_synth" for x in v])
        span = t1 - t0
        u_all, u_corr = union(allk), union(clip(corr))
        print(f"window {span / 1e6:.3f} ms: any kernel {100 * u_all / span:.1f} %, k_corr {100 * u_corr / span:.1f} %, "
              f"no kernel {100 * (span - u_all) / span:.1f} %, other kernels only {100 * (u_all - u_corr) / span:.1f} %")


if __name__ == "__main__":
    main(*sys.argv[1:])
