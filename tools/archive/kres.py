"""Per-kernel resource usage from hipcc -Rpass-analysis=kernel-resource-usage remarks.
Usage: hipcc ... -Rpass-analysis=kernel-resource-usage -c X.hip -o /tmp/x.o 2>&1 | python tools/kres.py [FILTER]"""
import re
import subprocess
import sys

flt = sys.argv[1] if len(sys.argv) > 1 else ""
rows, cur = [], None
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    m = re.search(r"remark:\s+([A-Za-z \[\]/]+?):\s*(\d+)", line)
    if m and cur is not None:
        cur[m.group(1).strip()] = int(m.group(2))
names = [r["name"] for r in rows]
try:
    dem = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout.split("\n")
except OSError:
    dem = names
for r, d in zip(rows, dem):
    if flt not in d:
        continue
    print(f"{d[:90]:90s} vgpr={r.get('VGPRs')} agpr={r.get('AGPRs')} spill={r.get('VGPRs Spill')} "
          f"lds={r.get('LDS Size [bytes/block]')} occ={r.get('Occupancy [waves/SIMD]')}")
