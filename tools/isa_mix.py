"""Instruction mix of one kernel in a hipcc -S listing.

  python tools/isa_mix.py FILE.s KERNEL_SUBSTR [--loop]

--loop restricts the count to the outermost loop (from its "Loop Header: Depth=1" label to the
last branch back to it), i.e. one CMUX step of the PBS kernels (everything there is unrolled)."""
import collections, re, sys

path, key = sys.argv[1], sys.argv[2]
loop = "--loop" in sys.argv
lines = open(path).read().split("\n")
start = next(i for i, l in enumerate(lines)
             if l.startswith("_Z") and key in l and l.split(";")[0].rstrip().endswith(":"))
end = next(i for i in range(start + 1, len(lines)) if lines[i].strip().startswith(".Lfunc_end"))
body = lines[start:end]
if loop:
    # blocks of the outermost loop: its header and every block LLVM annotates
    # "in Loop: Header=<hdr> Depth=1" (the latch may be laid out before the header); inner
    # loops (the spin waits) are left out
    h = next(i for i, l in enumerate(body) if "Loop Header: Depth=1" in l)
    hdr = body[h].split(":")[0].strip().lstrip(".L")
    keep, on = [], False
    for i, l in enumerate(body):
        if re.match(r"^\.?\w+:", l) or l.startswith("; %bb."):
            on = i == h or ("Header=" + hdr + " Depth=1") in l
        if on:
            keep.append(l)
    body = keep
cnt = collections.Counter()
cls = collections.Counter()
for l in body:
    s = l.strip()
    if not s or s.startswith((";", ".", "_Z")) or s.split(";")[0].rstrip().endswith(":"):
        continue
    m = s.split()[0]
    cnt[m] += 1
    if m.startswith("v_") and "f64" in m: cls["valu_f64"] += 1
    elif m.startswith("v_"): cls["valu_other"] += 1
    elif m.startswith("ds_"): cls["lds"] += 1
    elif m.startswith(("global_", "buffer_")): cls["vmem"] += 1
    elif m.startswith("s_"): cls["salu/ctrl"] += 1
print(dict(cls))
for m, c in cnt.most_common(40):
    print(f"{c:6d} {m}")
