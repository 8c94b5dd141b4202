"""Extracts the parameter rows of the concrete optimizer's reference table
(compilers/concrete-optimizer/v0-parameters/ref/v0_last_128: per message width and log norm2,
k, log2 N, n, br_l, br_b, ks_l, ks_b) into tests/golden/v0_last_128_rows.json.  The rows are data
(the table's numbers), used by tests/test_keygen_abi.py and tests/test_gpu_pbs_generic.py; this
script runs in the build container only (the reference tree is not on the GPU boxes).
Usage: python tests/golden/make_v0_rows.py [/root/reference]"""
import json
import os
import re
import sys


def main():
    ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
    src = os.path.join(ref, "compilers/concrete-optimizer/v0-parameters/ref/v0_last_128")
    rows, width = [], None
    for line in open(src):
        m = re.match(r"\s*- (\d+): # bits", line)
        if m:
            width = int(m.group(1))
            continue
        m = re.match(r"\s*- (\d+)\s*:\s*(.*)", line)
        if m and width:
            k, log_n, n, br_l, br_b, ks_l, ks_b = (int(x) for x in m.group(2).split(",")[:7])
            rows.append({"bits": width, "log_norm2": int(m.group(1)), "k": k, "N": 1 << log_n, "n": n,
                         "br_l": br_l, "br_b": br_b, "ks_l": ks_l, "ks_b": ks_b})
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "v0_last_128_rows.json")
    with open(out, "w") as fh:  # one row per line
        fh.write('{"source": "compilers/concrete-optimizer/v0-parameters/ref/v0_last_128", "rows": [\n')
        fh.write(",\n".join(json.dumps(r) for r in rows))
        fh.write("\n]}\n")
    print(f"{len(rows)} rows -> {out}")


if __name__ == "__main__":
    main()
