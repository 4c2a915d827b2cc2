"""HBM traffic per k_corr "launch" (the four width-group dispatches of one
batch) from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE; one counter
per pass, kernel trace only).  Writes profiles/pmc_k_corr.json, which
bench.py reports as roofline.traffic.

Units: rocprofv3 reports FETCH_SIZE / WRITE_SIZE in KiB.  MI355X_MICROARCH.md
(HBM section): FETCH_SIZE reads exactly 1/2 of the bytes only for 16-B/lane
coalesced streaming reads; other widths are uncalibrated.  k_corr's tile
loads are 1-byte-per-element reads of the u8 ext crops, so FETCH_SIZE is
taken as is (no x2) and the figure is labelled uncalibrated.

Usage: python scripts/pmc_traffic.py gpurun_out/pmc_<tag> <batch> [out.json]
"""
import csv
import json
import os
import sys
from collections import defaultdict


def per_kernel(path):
    d = defaultdict(list)
    with open(path) as fh:
        for r in csv.DictReader(fh):
            d[r["Kernel_Name"].split("(")[0]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in d.items()}


def main(root, batch, out=None):
    batch = int(batch)
    fetch = per_kernel(os.path.join(root, "FETCH_SIZE", "run_counter_collection.csv"))
    write = per_kernel(os.path.join(root, "WRITE_SIZE", "run_counter_collection.csv"))
    corr = sorted(k for k in fetch if "k_corr" in k)
    f_kib = sum(fetch[k] for k in corr)
    w_kib = sum(write.get(k, 0.0) for k in corr)
    res = {
        "kernel": "k_corr (sum of the width-group dispatches of one batch)",
        "dispatches": corr,
        "batch_frames": batch,
        "fetch_bytes_per_launch": int(f_kib * 1024),
        "write_bytes_per_launch": int(w_kib * 1024),
        "hbm_bytes_per_launch": int((f_kib + w_kib) * 1024),
        "hbm_bytes_per_frame": round((f_kib + w_kib) * 1024 / batch, 1),
        "correction": "none (1-byte loads; the x2 FETCH_SIZE correction is calibrated for 16-B/lane reads only)",
        "all_kernels_kib_per_dispatch": {k: {"fetch": round(fetch[k], 1), "write": round(write.get(k, 0.0), 1)}
                                         for k in sorted(fetch)},
    }
    text = json.dumps(res, indent=1)
    if out:
        with open(out, "w") as fh:
            fh.write(text + "\n")
    print(text)


if __name__ == "__main__":
    main(*sys.argv[1:])
