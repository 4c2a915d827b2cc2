"""Where a C4 pass (bench.py --video-frames) spends its time, from a
rocprofv3 --kernel-trace CSV: the passes are found as the k_minmax bursts
(every batch starts with one), and for each pass the script prints its span
(first dispatch start to last end), the time some kernel runs, the time a
correlation runs, and that split into the pass's first / middle / last
fifths -- the fill and drain show up as low correlation coverage at the ends.

    python scripts/trace_passes.py run_kernel_trace.csv [batches_per_pass]
"""
import csv
import sys


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


def clip(iv, lo, hi):
    return [(max(a, lo), min(b, hi)) for a, b in iv if b > lo and a < hi]


def main(path, per_pass=32):
    per_pass = int(per_pass)
    rows = []
    with open(path) as fh:
        for r in csv.DictReader(fh):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0]))
    rows.sort()
    starts = [a for a, _, n in rows if n == "k_minmax"]
    # passes: consecutive groups of per_pass batches, from the end (the timed ones)
    npass = len(starts) // per_pass
    for p in range(npass):
        lo = starts[p * per_pass]
        hi_start = starts[(p + 1) * per_pass] if (p + 1) * per_pass < len(starts) else None
        ks = [(a, b, n) for a, b, n in rows if a >= lo and (hi_start is None or a < hi_start)]
        if not ks:
            continue
        t0, t1 = ks[0][0], max(b for _, b, _ in ks)
        allk = [(a, b) for a, b, _ in ks]
        corr = [(a, b) for a, b, n in ks if "k_corr" in n]
        span = t1 - t0
        line = f"pass {p}: span {span / 1e6:.3f} ms, any kernel {union(allk) / span:.3f}, correlation {union(corr) / span:.3f}"
        fifths = []
        for q in range(5):
            a, b = t0 + span * q // 5, t0 + span * (q + 1) // 5
            fifths.append(f"{union(clip(corr, a, b)) / (b - a):.2f}")
        gap = (hi_start - t1) / 1e6 if hi_start else None
        print(line + ", correlation by fifth " + " ".join(fifths) +
              (f", idle before the next pass {gap:.3f} ms" if gap is not None else ""))


if __name__ == "__main__":
    main(*sys.argv[1:])
