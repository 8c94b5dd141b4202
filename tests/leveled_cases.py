"""The reference's leveled (PBS-free) cases as linear-operation programs.

tests/golden/reference_leveled_fixtures.json holds BASELINE configs[0]'s add(x, y) and its sibling
single-op circuits (end_to_end_leveled_gen.py --minimal 1, tests_cpu/end_to_end_fhe.yaml neg_eint):
op, precision p, constant, inputs, expected.  The compiler lowers each op to the runtime's LWE
linear operations (compiler lib/Conversion/FHEToTFHEScalar/FHEToTFHEScalar.cpp: add_eint ->
ciphertext add, add_eint_int -> plaintext add of the encoded integer, sub_* -> the same with a
negation, mul_eint_int -> cleartext multiply, neg_eint -> negate), which are the four
cuda_*_lwe_ciphertext_vector_64 entry points on the GPU route (GPUDFG.cpp:1286-1447).
`program(case)` returns that lowering as a list of steps; `cleartext(case)` evaluates the same
steps on integers modulo 2^(p+1) (one padding bit, Transformers.cpp:364-382).
"""
import json
import os

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "reference_leveled_fixtures.json")


def load():
    with open(GOLDEN) as f:
        return json.load(f)["cases"]


def operands(case):
    """(encrypted inputs, integer operand or None) in the op's argument order."""
    ints = [v for v, k in zip(case["inputs"], case["arg_kinds"]) if k == "int"]
    encs = [v for v, k in zip(case["inputs"], case["arg_kinds"]) if k == "eint"]
    integer = case["constant"] if case["constant"] is not None else (ints[0] if ints else None)
    return encs, integer


def program(case):
    """Steps over ciphertext registers: ("add", a, b), ("add_pt", a, value), ("mul", a, value),
    ("neg", a); register i < len(encs) is encrypted input i, each step appends a register; the last
    register is the result."""
    op = case["op"]
    encs, c = operands(case)
    if op == "identity":
        return []
    if op == "add_eint":
        return [("add", 0, 1)]
    if op == "add_eint_int":
        return [("add_pt", 0, c)]
    if op == "sub_eint_int":
        return [("add_pt", 0, -c)]
    if op == "sub_int_eint":
        return [("neg", 0), ("add_pt", 1, c)]
    if op == "sub_eint":
        return [("neg", 1), ("add", 0, 2)]
    if op == "mul_eint_int":
        return [("mul", 0, c)]
    if op == "neg_eint":
        return [("neg", 0)]
    raise ValueError(op)


def cleartext(case):
    mod = 1 << (case["precision"] + 1)
    regs, _ = operands(case)
    regs = list(regs)
    for st in program(case):
        if st[0] == "add":
            regs.append(regs[st[1]] + regs[st[2]])
        elif st[0] == "add_pt":
            regs.append(regs[st[1]] + st[2])
        elif st[0] == "mul":
            regs.append(regs[st[1]] * st[2])
        else:
            regs.append(-regs[st[1]])
        regs[-1] %= mod
    return regs[-1] % mod
