"""Summarise tools/pmc.sh output: per-dispatch counter values of the PBS kernel."""
import csv, glob, sys, collections
root = sys.argv[1]
vals = collections.defaultdict(list)
for f in glob.glob(f"{root}/*/run_counter_collection.csv") + glob.glob(f"{root}/*/*/run_counter_collection.csv"):
    for row in csv.DictReader(open(f)):
        if "pbs1024" not in row.get("Kernel_Name", ""):
            continue
        vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
for k in sorted(vals):
    v = vals[k]
    print(f"{k:28s} {sum(v)/len(v):.4g}  (n={len(v)})")
