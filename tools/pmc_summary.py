"""Summarise tools/pmc.sh output: per-dispatch counter values of the PBS kernel.
Usage: python tools/pmc_summary.py DIR [KERNEL_SUBSTRING (default pbs1024)]"""
import csv, glob, sys, collections
root = sys.argv[1]
kname = sys.argv[2] if len(sys.argv) > 2 else "pbs1024"
vals = collections.defaultdict(list)
for f in glob.glob(f"{root}/*/run_counter_collection.csv") + glob.glob(f"{root}/*/*/run_counter_collection.csv"):
    for row in csv.DictReader(open(f)):
        if kname not in row.get("Kernel_Name", ""):
            continue
        vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
for k in sorted(vals):
    v = vals[k]
    print(f"{k:28s} {sum(v)/len(v):.4g}  (n={len(v)})")
