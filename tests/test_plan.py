"""The cfg2 batch planner (concrete_amd/csrc/pbs1024_plan.hpp, through the C-ABI query
concrete_hip_pbs1024_plan): host logic only, no GPU.  A call is cut into whole pair-kernel rounds
(4 ciphertexts per CU), six-wave rounds (2 per CU) and at most one round of one ciphertext per CU;
the plan's estimated time is never above either single-kernel choice, and every part size adds up
to the batch."""
import ctypes as C

import pytest

PAIR, HEX2, HEX1 = 1020, 545, 485  # round costs the planner uses (1/100 ms at n = 630)


@pytest.fixture(scope="module")
def L():
    from concrete_amd import _native
    return _native.lib()


def plan(L, nb, cus):
    parts = (C.c_uint32 * 3)()
    cost = L.concrete_hip_pbs1024_plan(nb, cus, parts)
    return list(parts), cost


@pytest.mark.parametrize("cus", [256, 304, 80, 1])
def test_plan_covers_the_batch_and_beats_single_kernels(L, cus):
    for nb in list(range(1, 9 * cus + 3, max(1, cus // 16))) + [4096, 65536 // 8, 12345]:
        parts, cost = plan(L, nb, cus)
        assert sum(parts) == nb, (nb, parts)
        assert parts[2] <= cus
        pair_only = -(-nb // (4 * cus)) * PAIR
        hex_rounds = -(-nb // (2 * cus))
        hex_only = hex_rounds * HEX2 if nb > cus or hex_rounds > 1 else HEX1
        assert cost <= min(pair_only, hex_only), (nb, parts, cost)
        # the estimate is the sum of the parts' rounds
        est = -(-parts[0] // (4 * cus)) * PAIR + -(-parts[1] // (2 * cus)) * HEX2 + (HEX1 if parts[2] else 0)
        assert est == cost, (nb, parts, cost, est)


def test_plan_at_the_sweep_points(L):
    """The batch sweep of profiles/r06/batch_sweep.json (B = 256 .. 4096 in steps of 256 on 256 CUs)."""
    want = {256: [0, 0, 256], 512: [0, 512, 0], 768: [768, 0, 0], 1024: [1024, 0, 0], 1280: [1024, 0, 256],
            1536: [1024, 512, 0], 2304: [2048, 0, 256], 2560: [2048, 512, 0], 4096: [4096, 0, 0]}
    for nb, parts in want.items():
        assert plan(L, nb, 256)[0] == parts, nb
