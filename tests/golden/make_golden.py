"""Regenerate tests/golden/*.json from the reference's own fixture generators.

Runs (as subprocesses, read-only) the reference's numpy generators exactly as its GPU test
Makefile does (compilers/concrete-compiler/compiler/Makefile:299-303):
  end_to_end_apply_lookup_table_gen.py        --bitwidth 1 2 3 4 5 6 7 8
  end_to_end_linalg_apply_lookup_table_gen.py --bitwidth 1 2 3 4 5 6 7 8
and keeps the cleartext vectors (inputs, LUT, expected outputs) as JSON data fixtures.
reference_leveled_fixtures.json: the leveled (PBS-free) cases — BASELINE configs[0]'s add(x, y)
and its siblings — from end_to_end_leveled_gen.py --minimal 1 and the neg_eint cases of
tests_cpu/end_to_end_fhe.yaml: op, precision, constant, inputs, expected (data only).
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


LEVELED_OPS = ("FHE.add_eint_int", "FHE.add_eint", "FHE.sub_eint_int", "FHE.sub_int_eint", "FHE.sub_eint",
               "FHE.mul_eint_int", "FHE.neg_eint")


def leveled_cases(docs):
    """Single-op leveled programs (one encrypted scalar result): op, precision, constant, inputs."""
    import re
    res = []
    for d in docs:
        prog = d.get("program", "")
        ops = [o for o in LEVELED_OPS if f'"{o}"' in prog]
        if "tensor" in prog:
            continue
        if not ops and "return %arg0" in prog:
            ops = ["identity"]
        if len(ops) != 1:
            continue
        m = re.search(r"!FHE\.eint<(\d+)>", prog)
        if not m:  # signed (esint) programs are out of this set
            continue
        prec = int(m.group(1))
        cst = re.search(r"arith\.constant (\d+) : i\d+", prog)
        # argument order of the op (sub_int_eint takes the integer first)
        args = re.search(r"@main\(([^)]*)\)", prog).group(1)
        kinds = ["int" if re.search(r": i\d+$", a.strip()) else "eint" for a in args.split(",") if a.strip()]
        for t in d["tests"]:
            res.append({"description": d["description"], "op": ops[0].replace("FHE.", ""), "precision": prec,
                        "constant": int(cst.group(1)) if cst else None, "arg_kinds": kinds,
                        "inputs": [int(i["scalar"]) for i in t.get("inputs", [])],
                        "expected": int(t["outputs"][0]["scalar"])})
    return res


def leveled():
    gen = [d for d in run("end_to_end_leveled_gen.py", ["--minimal", "1"])]
    with open(os.path.join(REF, "tests_cpu", "end_to_end_fhe.yaml")) as f:
        fhe = [d for d in yaml.safe_load_all(f) if d and str(d.get("description", "")).startswith("neg_eint")]
    return {"source": "end_to_end_leveled_gen.py --minimal 1; tests_cpu/end_to_end_fhe.yaml neg_eint*",
            "cases": leveled_cases(gen) + leveled_cases(fhe)}


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
    lev = leveled()
    with open(os.path.join(HERE, "reference_leveled_fixtures.json"), "w") as f:
        json.dump(lev, f, indent=1)
    print("wrote", len(lev["cases"]), "leveled cases")


if __name__ == "__main__":
    main()
