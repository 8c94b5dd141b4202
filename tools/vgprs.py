"""Print VGPR / spill counts of the PBS kernels in a hipcc -S output: python tools/vgprs.py file.s [filter]"""
import re, sys
s = open(sys.argv[1]).read()
flt = sys.argv[2] if len(sys.argv) > 2 else ""
for m in re.finditer(r"\n  - \.agpr_count:.*?\n    \.name:\s+(\S+).*?\.vgpr_count:\s+(\d+)\n\s+\.vgpr_spill_count:\s+(\d+)", s, re.S):
    blk = m.group(0)
    if flt in m.group(1):
        sp = re.search(r"\.sgpr_spill_count:\s+(\d+)", blk)
        print(m.group(1)[:60], "vgpr", m.group(2), "vspill", m.group(3), "sspill", sp.group(1) if sp else "?")
