"""CPU check of the leveled-case lowering (tests/leveled_cases.py): evaluated on integers modulo
2^(p+1), every reference case (tests/golden/reference_leveled_fixtures.json) gives the reference's
expected output — this pins the op -> linear-operation mapping that tests/test_gpu_leveled.py runs
encrypted through the cuda_* entry points."""
import leveled_cases as LC


def test_fixture_covers_configs0_and_every_linear_op():
    cases = LC.load()
    ops = {c["op"] for c in cases}
    assert {"add_eint", "add_eint_int", "sub_eint_int", "sub_int_eint", "sub_eint", "mul_eint_int", "neg_eint"} <= ops
    assert any(c["op"] == "add_eint" for c in cases)  # configs[0]: add(x, y)
    assert len(cases) >= 150


def test_lowering_matches_reference_expectations():
    for c in LC.load():
        assert LC.cleartext(c) == c["expected"], c
