"""Per-kernel effective clock and VALU busy from rocprofv3 PMC passes.

For every pass directory (OUT/p*/) holding GRBM_GUI_ACTIVE, the dispatches'
counter rows are joined with the same pass's kernel trace (durations):
    clock = GRBM_GUI_ACTIVE / 8 XCDs / duration         (MI355X_MICROARCH.md, DVFS give-back)
and, when the pass also holds SQ_ACTIVE_INST_VALU (quad-cycles summed over
waves), VALU busy = 4 * SQ_ACTIVE_INST_VALU / (1024 SIMDs * GRBM_GUI_ACTIVE / 8).
Usage: pmc_clock.py OUT [kernel-substring]"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main(root, filt=""):
    rows = defaultdict(lambda: defaultdict(list))
    for d in sorted(glob.glob(os.path.join(root, "p*"))):
        cc = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
        kt = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
        if not cc:
            continue
        dur = {}
        for f in kt:
            with open(f) as fh:
                for r in csv.DictReader(fh):
                    dur[r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        per = defaultdict(lambda: defaultdict(float))
        names = {}
        for f in cc:
            with open(f) as fh:
                for r in csv.DictReader(fh):
                    per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
                    names[r["Dispatch_Id"]] = r["Kernel_Name"].split("(")[0]
                    if "Start_Timestamp" in r and r["Dispatch_Id"] not in dur:
                        dur[r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        for disp, cs in per.items():
            if "GRBM_GUI_ACTIVE" not in cs or disp not in dur or dur[disp] <= 0:
                continue
            cyc = cs["GRBM_GUI_ACTIVE"] / 8
            r = rows[names[disp]]
            r["clock_ghz"].append(cyc / dur[disp])
            r["dur_us"].append(dur[disp] / 1e3)
            if "SQ_ACTIVE_INST_VALU" in cs:
                r["valu_busy"].append(4 * cs["SQ_ACTIVE_INST_VALU"] / (1024 * cyc))
            if "SQ_INSTS_VALU" in cs and "SQ_ACTIVE_INST_VALU" in cs and cs["SQ_INSTS_VALU"]:
                r["quad_cyc_per_valu"].append(cs["SQ_ACTIVE_INST_VALU"] / cs["SQ_INSTS_VALU"])
    for k in sorted(rows):
        if filt and filt not in k:
            continue
        r = rows[k]
        print(k + ": " + ", ".join(f"{m} {sum(v) / len(v):.3f} (n={len(v)})" for m, v in r.items()))


if __name__ == "__main__":
    main(*sys.argv[1:])
