"""HBM traffic per k_corr "launch" (the four width-group dispatches of one
batch) from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE; one counter
per pass, kernel trace only).  Writes profiles/pmc_k_corr.json, which
bench.py reports as roofline.traffic.

Units: rocprofv3 reports FETCH_SIZE / WRITE_SIZE in KiB.  MI355X_MICROARCH.md
(HBM section, :298): on gfx950 FETCH_SIZE reports exactly 1/2 of the bytes of
a wide coalesced streaming read (16 B/lane; 128-B requests tallied at 64 B).
The other widths the kernels use were calibrated on a known byte count
(scripts/ubench/fetch_calib.hip, profiles/r03/fetch_calib.json): 4-B/lane
dword loads (k_corr_rw's ring rows), k_ingest's five-dword run gathers and
byte loads also read 0.50 of their bytes, and WRITE_SIZE is exact for 16-B
and 4-B stores.  So every FETCH_SIZE is doubled.  The per-kernel table lists
FETCH_SIZE as reported.

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
    # x2 for every read width the kernels use (MI355X_MICROARCH.md:298; profiles/r03/fetch_calib.json)
    scale = {k: 2 for k in corr}
    f_kib = sum(scale[k] * fetch[k] for k in corr)
    w_kib = sum(write.get(k, 0.0) for k in corr)
    res = {
        "kernel": "k_corr (sum of the width-group dispatches of one batch)",
        "dispatches": corr,
        "batch_frames": batch,
        "fetch_bytes_per_launch": int(f_kib * 1024),
        "write_bytes_per_launch": int(w_kib * 1024),
        "hbm_bytes_per_launch": int((f_kib + w_kib) * 1024),
        "hbm_bytes_per_frame": round((f_kib + w_kib) * 1024 / batch, 1),
        "correction": {k: "FETCH_SIZE x2: gfx950 tallies 128-B requests at 64 B (MI355X_MICROARCH.md:298); "
                          "calibrated for the kernel's 4-B/lane and 16-B/lane loads in profiles/r03/fetch_calib.json"
                       for k in corr},
        "write_correction": "WRITE_SIZE as reported",
        # k_ingest per batch (one dispatch): its 16-B and 4-B run loads and byte
        # loads are calibrated at 0.50 too (profiles/r03/fetch_calib.json)
        "k_ingest": ({"fetch_bytes_per_batch": int(2 * fetch["k_ingest"] * 1024),
                      "write_bytes_per_batch": int(write.get("k_ingest", 0.0) * 1024),
                      "hbm_bytes_per_batch": int((2 * fetch["k_ingest"] + write.get("k_ingest", 0.0)) * 1024),
                      "correction": "FETCH_SIZE x2, WRITE_SIZE as reported"} if "k_ingest" in fetch else None),
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
