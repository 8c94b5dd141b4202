"""Per-kernel split of a PMC traffic pass (tools/pmc.sh passes d / e: FETCH_SIZE, WRITE_SIZE) over
one bench call: which launch of the general path moves which bytes (the
N >= 8192 two-launch path's X / Y / accumulator traffic).
  bytes read = 2 * FETCH_SIZE KB (gfx950 tallies 128-B requests at 64 B, MI355X_MICROARCH.md §HBM),
  bytes written = WRITE_SIZE KB.
Usage: python tools/pmc_split.py DIR BATCH STEPS(n) [OUT.json]"""
import collections
import csv
import glob
import json
import re
import sys

root, batch, n = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
acc = collections.defaultdict(lambda: {"dispatches": 0, "FETCH_SIZE_KB": 0.0, "WRITE_SIZE_KB": 0.0})
for f in glob.glob(f"{root}/**/run_counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        name = row.get("Kernel_Name", "")
        if "rocclr" in name:
            continue
        short = re.sub(r"<.*", "", name.split("(")[0]).replace("void ", "").strip()
        c = row["Counter_Name"]
        if c in ("FETCH_SIZE", "WRITE_SIZE"):
            acc[short][c + "_KB"] += float(row["Counter_Value"])
            if c == "FETCH_SIZE":
                acc[short]["dispatches"] += 1
out = {}
for k, v in sorted(acc.items(), key=lambda kv: -(2 * kv[1]["FETCH_SIZE_KB"] + kv[1]["WRITE_SIZE_KB"])):
    rd, wr = 2 * v["FETCH_SIZE_KB"] * 1024, v["WRITE_SIZE_KB"] * 1024
    out[k] = {"dispatches": v["dispatches"], "read_bytes": rd, "write_bytes": wr,
              "read_per_ct_step": rd / (batch * n), "write_per_ct_step": wr / (batch * n)}
    print(f"{k:60s} {v['dispatches']:6d}  read {rd / 1e9:9.2f} GB  write {wr / 1e9:9.2f} GB  "
          f"per ct-step read {rd / (batch * n) / 2**20:6.3f} MiB write {wr / (batch * n) / 2**20:6.3f} MiB")
if len(sys.argv) > 4:
    json.dump({"batch": batch, "n": n, "kernels": out}, open(sys.argv[4], "w"), indent=1)
