"""Aggregate rocprofv3 --pmc counter CSVs (one dir per pass) per kernel:
mean over dispatches of each counter.  Usage: pmc_summary.py gpurun_out/pmc [kernel-substring]"""
import csv
import glob
import os
import sys
from collections import defaultdict


def load(root):
    data = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> [values per dispatch]
    for f in sorted(glob.glob(os.path.join(root, "p*", "*counter_collection.csv"))):
        per = defaultdict(float)
        names = {}
        with open(f) as fh:
            for row in csv.DictReader(fh):
                key = (row["Dispatch_Id"], row["Counter_Name"])
                per[key] += float(row["Counter_Value"])
                names[row["Dispatch_Id"]] = row["Kernel_Name"].split("(")[0]
        for (disp, cn), v in per.items():
            data[names[disp]][cn].append(v)
    return data


def main(root, filt=""):
    data = load(root)
    for k in sorted(data):
        if filt and filt not in k:
            continue
        print(k)
        for cn in sorted(data[k]):
            vals = data[k][cn]
            print(f"   {cn:28s} mean {sum(vals)/len(vals):16.1f}  n={len(vals)}")


if __name__ == "__main__":
    main(*sys.argv[1:])
