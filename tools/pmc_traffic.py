"""Turn a tools/pmc.sh run into the per-launch HBM traffic record bench.py reports.

traffic = 2 * FETCH_SIZE + WRITE_SIZE (KB -> bytes).  gfx950 tallies 128-B fabric read requests
at 64 B, so FETCH_SIZE is doubled for 16-B/lane streaming reads (MI355X_MICROARCH.md §HBM);
WRITE_SIZE is exact for 16-B/lane stores.  The record carries the hash of the kernel sources it
was measured on; bench.py reports it only while the sources are unchanged.
Usage: python tools/pmc_traffic.py gpurun_out/<tag> profiles/<round>_pbs_traffic.json [cfg2|cfg4]
"""
import csv, glob, json, os, sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import kernel_source_hash  # noqa: E402

src, dst = sys.argv[1], sys.argv[2]
config = sys.argv[3] if len(sys.argv) > 3 else "cfg2"
kname = "pbs1024" if config == "cfg2" else "pbs2048"
vals = {}
for f in glob.glob(f"{src}/**/run_counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        if kname in row.get("Kernel_Name", "") and row["Counter_Name"] in ("FETCH_SIZE", "WRITE_SIZE"):
            vals.setdefault(row["Counter_Name"], []).append(float(row["Counter_Value"]))
fetch = sum(vals["FETCH_SIZE"]) / len(vals["FETCH_SIZE"])
write = sum(vals["WRITE_SIZE"]) / len(vals["WRITE_SIZE"])
rec = {"kernel": kname, "config": config, "batch": 4096,
       "fetch_size_kb": fetch, "write_size_kb": write,
       "traffic_bytes": int(round((2 * fetch + write) * 1024)),
       "source_hash": kernel_source_hash(), "pmc_dir": src}
json.dump(rec, open(dst, "w"), indent=1)
print(json.dumps(rec))
