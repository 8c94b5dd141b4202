"""Collect the bench lines of tools/r06.sh bench1 / bench2 (r05: tools/r05_final.sh) into one record:
python tools/collect_bench.py gpurun_out/<tag> profiles/<round>_bench_all_configs.json"""
import glob
import json
import os
import sys

src, dst = sys.argv[1], sys.argv[2]
out = {"note": "bench.py lines of every config on the final sources, one MI355X box (tools/r06.sh bench1 + bench2; r05: tools/r05_final.sh); "
               "cfg2 = BASELINE configs[1] (the metric), cfg4 = configs[3], opt8 = configs[4]'s optimizer row; "
               "opt1..opt6 at batch 4096, opt7..opt9 at 1024, opt10 at 512; opt7_twolaunch = opt7 with "
               "CONCRETE_HIP_GEN_COOP=0 (the two-launch path, for the A/B of DESIGN.md §4.12)",
       "lines": {}}
for f in sorted(glob.glob(os.path.join(src, "bench_*.log"))):
    name = os.path.basename(f)[len("bench_"):-len(".log")]
    lines = [l for l in open(f).read().splitlines() if l.startswith("{")]
    if lines:
        out["lines"]["cfg2" if name == "default" else name] = json.loads(lines[-1])
# a line run with CONCRETE_HIP_GEN_COOP=0 is the two-launch path: the config's PMC record (bench.py attaches
# it by source hash) is the two-workgroup kernel's, so its traffic / dram / valu do not apply
for k, v in out["lines"].items():
    if k.endswith("_twolaunch"):
        for f in ("traffic", "traffic_src", "dram", "valu"):
            v.get("roofline", {}).pop(f, None)
        v.setdefault("roofline", {})["note_pmc"] = "no PMC record for the two-launch path on these sources (the config's record is the default kernel's)"
json.dump(out, open(dst, "w"), indent=1)
for k, v in out["lines"].items():
    r = v.get("roofline", {})
    print(f"{k:6s} {v['value']:>10} PBS/s  frac {r.get('frac')}  traffic {r.get('traffic')}  "
          f"valu {(r.get('valu') or {}).get('frac')}  cpu {(v.get('cpu_baseline') or {}).get('value')}  "
          f"bitexact {v.get('checks', {}).get('bitexact')}  decrypt {v.get('checks', {}).get('decrypt_ok')}")
