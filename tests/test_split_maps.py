"""Index maps of the N = 2^15 / 2^16 split path (concrete_amd/csrc/pbs_generic.hip, round 6), restated on
the host: every map must be a bijection, or a workgroup / lane would compute a polynomial class or a
frequency twice and leave another unwritten (the GPU parity tests would only see that on the shapes
they run)."""
import pytest


def split_block(b, polys, S, xcd=True):
    """split_block<S>: workgroup b -> (polynomial, class h); the S classes of a polynomial on one XCD
    (workgroups b and b + 8 share one under round-robin dispatch), plain order in a last partial group."""
    g, r = divmod(b, 8 * S)
    if xcd and (g + 1) * 8 <= polys:
        return g * 8 + (r & 7), r >> 3
    return b // S, b % S


def mac_lane(b, t, S):
    """gen_mac_split_kernel: (block b, thread t) -> (frequency row k1, position, class u of the lane)."""
    QW, PB = 64 // S, 256 // S
    kl = b // (2 * S)
    lane = t & 63
    u, pl = divmod(lane, QW)
    pos = (b % (2 * S)) * PB + (t >> 6) * QW + pl
    return kl + 16 * u, pos, u


@pytest.mark.parametrize("S", [2, 4])
@pytest.mark.parametrize("polys", [1, 2, 6, 8, 9, 16, 17, 134, 512])
def test_split_block_is_a_bijection(S, polys):
    seen = {split_block(b, polys, S) for b in range(polys * S)}
    assert seen == {(p, h) for p in range(polys) for h in range(S)}
    # the grouped part really shares XCDs: b and b + 8 (same XCD) hold two classes of one polynomial
    for b in range(polys * S):
        g = b // (8 * S)
        if (g + 1) * 8 <= polys and (b % (8 * S)) < 8 * (S - 1):
            assert split_block(b, polys, S)[0] == split_block(b + 8, polys, S)[0]


@pytest.mark.parametrize("S", [2, 4])
def test_mac_lane_map_covers_every_frequency_once(S):
    M = 16 * 512 * S
    blocks = M // 256
    seen = set()
    for b in range(blocks):
        for t in range(256):
            k1, pos, u = mac_lane(b, t, S)
            assert 0 <= pos < 512 and 0 <= k1 < 16 * S
            seen.add((k1, pos))
            # the lane holding the same position at class u' is lane u' 64 / S + (lane mod 64 / S)
            lane = t & 63
            for uu in range(S):
                src = (t & ~63) + uu * (64 // S) + lane % (64 // S)
                k1b, posb, ub = mac_lane(b, src, S)
                assert posb == pos and ub == uu and k1b % 16 == k1 % 16
    assert len(seen) == M
