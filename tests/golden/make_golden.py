"""Regenerate tests/golden/*.json from the reference's own fixture generators.

Runs (as subprocesses, read-only) the reference's numpy generators exactly as its GPU test
Makefile does (compilers/concrete-compiler/compiler/Makefile:299-303):
  end_to_end_apply_lookup_table_gen.py        --bitwidth 1 2 3 4 5 6 7 8
  end_to_end_linalg_apply_lookup_table_gen.py --bitwidth 1 2 3 4 5 6 7 8
and keeps the cleartext vectors (inputs, LUT, expected outputs) as JSON data fixtures.
The reference tree is only needed to regenerate; the tests read the committed JSON.
"""
import json
import os
import subprocess
import sys

import yaml

REF = "/root/reference/compilers/concrete-compiler/compiler/tests/end_to_end_fixture"
HERE = os.path.dirname(os.path.abspath(__file__))


def run(gen, args):
    out = subprocess.run([sys.executable, os.path.join(REF, gen)] + args, cwd=REF, check=True,
                         capture_output=True, text=True).stdout
    return [d for d in yaml.safe_load_all(out) if d]


def cases(docs):
    res = []
    for d in docs:
        for t in d["tests"]:
            ins = t["inputs"]
            x = ins[0].get("scalar", ins[0].get("tensor"))
            res.append({
                "description": d["description"],
                "input_signed": bool(ins[0].get("signed", False)),
                "output_signed": bool(t["outputs"][0].get("signed", False)),
                "input": x if isinstance(x, list) else [x],
                "lut": ins[1]["tensor"],
                "expected": (lambda o: o if isinstance(o, list) else [o])(
                    t["outputs"][0].get("scalar", t["outputs"][0].get("tensor"))),
            })
    return res


def main():
    bits = [str(b) for b in range(1, 9)]
    out = {
        "source": "reference fixture generators (see make_golden.py)",
        "apply_lookup_table": cases(run("end_to_end_apply_lookup_table_gen.py", ["--bitwidth"] + bits)),
        "linalg_apply_lookup_table": cases(run("end_to_end_linalg_apply_lookup_table_gen.py",
                                               ["--bitwidth"] + bits + ["--n-ct", "64"])),
    }
    with open(os.path.join(HERE, "reference_lut_fixtures.json"), "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", sum(len(v) for k, v in out.items() if isinstance(v, list)), "cases")


if __name__ == "__main__":
    main()
