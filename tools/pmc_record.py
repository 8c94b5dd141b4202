"""Turn tools/pmc.sh passes into the per-launch PMC record bench.py reports (roofline.traffic,
roofline.valu, roofline.dram).

  traffic = 2 * FETCH_SIZE + WRITE_SIZE (KB -> bytes): gfx950 tallies 128-B fabric read requests at
            64 B, so FETCH_SIZE is doubled for 16-B/lane streaming reads (MI355X_MICROARCH.md
            §HBM); WRITE_SIZE is exact for 16-B/lane stores.
  f64_flop = 64 lanes * (2 * SQ_INSTS_VALU_FMA_F64 + SQ_INSTS_VALU_ADD_F64 + SQ_INSTS_VALU_MUL_F64)
            (the SQ_INSTS_* counters count wave-instructions, summed over the device).
The record carries the hash of the kernel sources it was measured on; bench.py uses it only while
the sources are unchanged.
Usage: python tools/pmc_record.py gpurun_out/<tag> profiles/<round>_<config>_pmc.json CONFIG BATCH [KERNEL]
       (<tag> holds the pass directories of tools/pmc.sh: d/e for traffic, b for the f64 mix)
"""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import kernel_source_hash  # noqa: E402

KERNEL = {"cfg2": "pbs1024_pair", "cfg4": "pbs2048", "opt5": "pbs2048", "opt4": "pbs1024k2", "opt1": "pbs_small",
          "opt2": "pbs_small", "opt3": "pbs_small"}
# the general path (optB configs) runs several launches per PBS call (pbs_generic.hip): the record
# sums every gen_* dispatch of the process's single call (tools/pmc.sh: --steps 1 --warmup 0 --no-e2e),
# except the once-per-key conversion
GENERIC_PREFIX = "chip::gen::gen_"
GENERIC_SKIP = ("gen_convert",)


def collect(src, kname):
    vals = {}
    generic = kname.startswith("opt")  # a config without a kernel of its own: the general path
    for f in glob.glob(f"{src}/**/run_counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            name = row.get("Kernel_Name", "")
            if generic:
                hit = GENERIC_PREFIX in name and not any(x in name for x in GENERIC_SKIP)
            else:
                hit = kname in name
            if hit:
                vals.setdefault(row["Counter_Name"], []).append(float(row["Counter_Value"]))
    if generic:  # one PBS call = the sum of its launches
        return {k: sum(v) for k, v in vals.items()}
    return {k: sum(v) / len(v) for k, v in vals.items()}


def main():
    src, dst, config, batch = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4])
    # optional 5th argument: the kernel-name substring (e.g. pbs1024_hex for cfg2 at B = 512)
    kname = sys.argv[5] if len(sys.argv) > 5 else KERNEL.get(config, config)
    v = collect(src, kname)
    rec = {"kernel": kname if not kname.startswith("opt") else "gen_* (sum over one PBS call)", "config": config, "batch": batch, "source_hash": kernel_source_hash(config), "pmc_dir": src,
           "counters": v}
    if "FETCH_SIZE" in v and "WRITE_SIZE" in v:
        rec["traffic_bytes"] = int(round((2 * v["FETCH_SIZE"] + v["WRITE_SIZE"]) * 1024))
    if "SQ_INSTS_VALU_FMA_F64" in v:
        rec["f64_flop"] = 64.0 * (2 * v["SQ_INSTS_VALU_FMA_F64"] + v.get("SQ_INSTS_VALU_ADD_F64", 0.0)
                                  + v.get("SQ_INSTS_VALU_MUL_F64", 0.0))
    # round 6: L2 and matrix-core passes (tools/pmc.sh f, g; the keyswitch's int8 MFMA kernel)
    if "TCP_TCC_READ_REQ_sum" in v:
        rec["l2_read_requests"] = v["TCP_TCC_READ_REQ_sum"]
        rec["l2_bytes"] = int(round(v["TCP_TCC_READ_REQ_sum"] * 128))  # 128-B L1 -> L2 read requests
    if "TCC_HIT_sum" in v and "TCC_MISS_sum" in v and v["TCC_HIT_sum"] + v["TCC_MISS_sum"] > 0:
        rec["l2_hit"] = round(v["TCC_HIT_sum"] / (v["TCC_HIT_sum"] + v["TCC_MISS_sum"]), 4)
    if "SQ_INSTS_VALU_MFMA_MOPS_I8" in v:
        rec["i8_ops"] = v["SQ_INSTS_VALU_MFMA_MOPS_I8"] * 512.0
    if "SQ_VALU_MFMA_BUSY_CYCLES" in v and v.get("GRBM_GUI_ACTIVE"):
        # rocprofv3's MfmaUtil: busy cycles summed over the 1,024 SIMDs / (GRBM_GUI_ACTIVE of one XCD
        # (the collected value sums the 8 XCDs) x 1,024)
        rec["mfma_busy"] = round(v["SQ_VALU_MFMA_BUSY_CYCLES"] / (v["GRBM_GUI_ACTIVE"] / 8 * 4 * 256), 4)
    json.dump(rec, open(dst, "w"), indent=1)
    print(json.dumps({k: rec[k] for k in rec if k != "counters"}))


if __name__ == "__main__":
    main()
