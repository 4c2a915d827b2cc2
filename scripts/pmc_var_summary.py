"""Summarise scripts/gpu_pmc_var.sh output: per variant and k_corr width,
counters per wave-cycle (SQ counters are sampled per SE; ratios only)."""
import csv, glob, collections, sys, re
root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pv"
for vdir in sorted(set(re.sub(r"_\d+$", "", p) for p in glob.glob(root + "/v*_*") if not p.endswith(".log"))):
    d = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(vdir + "_*/run_counter_collection.csv"):
        per = collections.defaultdict(float); names = {}
        for r in csv.DictReader(open(f)):
            per[(f, r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"]); names[(f, r["Dispatch_Id"])] = r["Kernel_Name"].split("(")[0]
        for (ff, di, cn), v in per.items(): d[names[(ff, di)]][cn].append(v)
    for k in sorted(d):
        if "k_corr" not in k: continue
        m = {cn: sum(v) / len(v) for cn, v in d[k].items()}
        wc = m["SQ_WAVE_CYCLES"]
        keys = ["SQ_ACTIVE_INST_VALU", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE", "SQ_INST_LEVEL_SMEM", "SQ_INST_LEVEL_LDS"]
        print(vdir.split("/")[-1], k[:28].ljust(28), " ".join(f"{c[3:]}={m.get(c, 0) / wc:.3f}" for c in keys),
              f"VALU/GRBM={m['SQ_INSTS_VALU'] * 4 / 1024 / m['GRBM_GUI_ACTIVE']:.3f}")
