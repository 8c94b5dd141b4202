"""CPU tests of libconcrete_hip.so: it loads, exports every symbol include/concrete_hip.h
declares, its host-side client helpers agree bit-for-bit with the oracle, and its
status-returning entry points reject bad arguments before touching a device."""
import ctypes as C
import os

import numpy as np
import pytest

from concrete_amd import _native
from concrete_amd import backend as B


def test_library_exports_every_declared_symbol():
    L = _native.lib()
    declared = _native.declared_symbols()
    assert len(declared) >= 30
    for name in declared:
        assert hasattr(L, name), name
    # and every declared symbol has a ctypes signature in the host binding
    assert set(declared) <= set(_native.SIGNATURES), set(declared) - set(_native.SIGNATURES)


def test_abi_version_and_queries():
    L = _native.lib()
    assert L.concrete_hip_abi_version() == 5
    assert L.concrete_hip_pbs_supported(1, 1024, 3, 7) == 1
    assert L.concrete_hip_pbs_supported(1, 1024, 3, 30) == 0  # l * logB >= 64
    # the pair kernel's exactness gate is (k+1) l 2^logB <= 4096 (3-limb rounding bound < 1/4);
    # wider digits run on the general path (a general-format companion key) while its bound holds
    assert L.concrete_hip_pbs_supported(1, 1024, 3, 9) == 1
    assert L.concrete_hip_pbs_supported(1, 1024, 3, 10) == 1
    assert L.concrete_hip_pbs_supported(1, 1024, 2, 10) == 1
    assert L.concrete_hip_pbs_supported(1, 1024, 1, 11) == 1
    assert L.concrete_hip_pbs_supported(1, 1024, 1, 15) == 1
    assert L.concrete_hip_pbs_supported(1, 1024, 1, 23) == 1
    assert L.concrete_hip_pbs_supported(1, 1024, 2, 33) == 0  # l * logB > 64
    assert L.concrete_hip_pbs_supported(2, 1024, 3, 7) == 1  # k = 2: the general path
    assert L.concrete_hip_pbs_supported(1, 131072, 1, 7) == 0  # N up to 2^16
    assert L.concrete_hip_bsk_limbs(1024, 3, 7) == 3
    p = B.CFG2
    # n * l * (k+1)^2 * LIMBS * N/2 complex f64
    assert B.fourier_bsk_bytes(p) == p.n * p.level * 4 * 3 * 512 * 16
    assert B.fourier_bsk_bytes(p) == 3 * p.bsk_len * 8  # 3 limbs x 8 B per coefficient


def test_status_codes_without_device():
    L = _native.lib()
    # unsupported parameters are rejected before any device call
    rc = L.concrete_hip_pbs(None, 0, 1, None, 1, None, 1, None, 1, 630, 1, 131072, 7, 3, 4, None)
    assert rc == -2 and b"unsupported" in L.concrete_hip_last_error()
    rc = L.concrete_hip_pbs(None, 0, None, None, None, None, None, None, None, 630, 1, 1024, 7, 3, 4, None)
    assert rc == -1
    assert L.concrete_hip_pbs(None, 0, None, None, None, None, None, None, None, 630, 1, 1024, 7, 3, 0, None) == 0
    rc = L.concrete_hip_convert_bsk(None, 0, None, None, 0, 630, 1, 3, 1024)
    assert rc == -1


def test_keygen_matches_oracle(oracle):
    p = B.PbsParams(n=32, k=1, N=1024, level=3, base_log=7, ks_level=4, ks_base_log=3)
    op = oracle.Params(n=32, k=1, N=1024, l=3, logB=7, ks_l=4, ks_logB=3)
    for seed in (1, 99):
        assert np.array_equal(B.binary_key(777, seed), oracle.binary_key(777, seed))
    lwe_sk = B.binary_key(p.n, 1)
    glwe_sk = B.binary_key(p.big_n, 2)
    bsk = B.bsk_generate(p, lwe_sk, glwe_sk, 3)
    assert np.array_equal(bsk, oracle.keygen_bsk(op, lwe_sk, glwe_sk, 3))
    ksk = B.ksk_generate(p, glwe_sk, lwe_sk, 4)
    assert np.array_equal(ksk, oracle.keygen_ksk(op, glwe_sk, lwe_sk, 4))
    pts = [int(B.encode(m, 3)) for m in range(8)]
    cts = B.lwe_encrypt(lwe_sk, pts, p.n, 2.0 ** -20, 5)
    assert np.array_equal(cts, oracle.lwe_encrypt_batch(lwe_sk, pts, p.n, 2.0 ** -20, 5))
    assert np.array_equal(B.lwe_decrypt(lwe_sk, cts, p.n), oracle.lwe_decrypt_batch(lwe_sk, cts, p.n))
    for bits in (1, 3, 4):
        for signed in (False, True):
            tab = np.arange(1 << bits, dtype=np.uint64)[::-1].copy()
            assert np.array_equal(B.expand_lut(tab, 1024, bits, signed), oracle.expand_lut(tab, 1024, bits, signed))


def test_encode_decode_match_oracle(oracle):
    for width in (1, 3, 4, 8):
        for m in range(1 << width):
            e = B.encode(m, width)
            assert int(e) == int(oracle.encode(m, width))
            assert B.decode(e, width) == oracle.decode(e, width) == m


def test_key_formats_and_exact_range():
    """Host-side key-format selection and exactness gate (pbs.hpp:key_format, pbs_generic.hip):
    the two hand-tuned layouts for cfg2/cfg4, the general path for the optimizer's other rows
    (v0_last_128 1..8-bit sets), and refusal where the certified bound would not hold."""
    import ctypes as C

    from concrete_amd import _native
    L = _native.lib()

    def fmt(k, N, l):
        a, b = C.c_uint32(), C.c_uint32()
        return L.concrete_hip_bsk_format(k, N, l, C.byref(a), C.byref(b)), a.value, b.value

    assert fmt(1, 1024, 3) == (1, 3, 22)
    assert fmt(1, 2048, 1) == (2, 4, 16)
    # cfg4 key: 4 limbs of g only (the digit is split on the limb grid, pbs2048.hip)
    assert L.concrete_hip_fourier_bsk_size_bytes(742, 1, 1, 2048) == 742 * 4 * 4 * 1024 * 16
    assert L.concrete_hip_pbs_supported(1, 2048, 1, 24) == 1
    assert L.concrete_hip_pbs_supported(1, 2048, 1, 25) == 1  # past the cfg4 kernel: the general path
    # l = 2 .. 4: the same kernel with whole-digit levels (l 2^(logB-1) <= 2^15), format code 2
    assert fmt(1, 2048, 2) == (2, 4, 16) and fmt(1, 2048, 4) == (2, 4, 16) and fmt(1, 2048, 5)[0] == 3
    assert L.concrete_hip_fourier_bsk_size_bytes(783, 1, 2, 2048) == 783 * 2 * 4 * 4 * 1024 * 16
    assert L.concrete_hip_pbs_supported(1, 2048, 2, 15) == 1 and L.concrete_hip_pbs_supported(1, 2048, 4, 9) == 1
    assert L.concrete_hip_pbs_supported(1, 2048, 2, 16) == 1  # past the levels gate: the companion key
    # the general-format key of the hand-tuned shapes (wide digits): its own limbs
    assert L.concrete_hip_generic_bsk_size_bytes(10, 1, 1, 2048) > 0
    assert L.concrete_hip_generic_bsk_size_bytes(10, 1, 1, 32768) > 0  # N = 2^15: the split path (round 4)
    assert L.concrete_hip_generic_bsk_size_bytes(10, 1, 1, 131072) == 0
    # the optimizer's 4-bit rows (k = 2, N = 1024, l = 1): their own kernel (pbs1024k2.hip, round 4),
    # 4 limbs of 16 bits, the digit split on the limb grid as at N = 2048
    assert fmt(2, 1024, 1) == (4, 4, 16) and fmt(2, 1024, 2) == (4, 4, 16)
    assert L.concrete_hip_pbs_supported(2, 1024, 2, 15) == 1  # two levels: whole digits up to 15 bits
    assert fmt(2, 1024, 3) == (4, 4, 16) and fmt(2, 1024, 4) == (4, 4, 16)  # l >= 4: one level at a time
    assert L.concrete_hip_fourier_bsk_size_bytes(727, 2, 44, 1024) == 727 * 44 * 4 * 9 * 512 * 16
    assert L.concrete_hip_pbs_supported(2, 1024, 3, 12) == 1
    assert L.concrete_hip_fourier_bsk_size_bytes(801, 2, 1, 1024) == 801 * 4 * 9 * 512 * 16
    assert L.concrete_hip_pbs_supported(2, 1024, 1, 24) == 1
    assert L.concrete_hip_generic_error_bound(2, 1024, 1, 23, 0.0) == -1.0
    # the optimizer's 1- to 3-bit rows (N = 256, k = 5 / 6, N = 512, k = 3 / 4, l = 1): the small-ring
    # kernels (pbs_small.hip, pbs512k4.hip, round 4), format code 5, digits up to 24 bits (wider: the
    # general path)
    assert fmt(3, 512, 1) == (5, 4, 16) and fmt(5, 256, 1) == (5, 4, 16) and fmt(6, 256, 1) == (5, 4, 16)
    assert fmt(4, 512, 1) == (5, 4, 16) and L.concrete_hip_pbs_supported(4, 512, 1, 23) == 1
    # levels on the small-ring kernels: whole digits with l 2^(logB-1) <= 2^15 (pbs.hpp pbs_small_ok);
    # k = 4, N = 512, l = 2 (logB = 16 rows): five 13-bit key limbs
    for k, N, l in [(5, 256, 2), (6, 256, 3), (3, 512, 3), (4, 512, 3), (4, 512, 5)]:
        assert fmt(k, N, l) == (5, 4, 16), (k, N, l)
    assert fmt(4, 512, 2) == (5, 5, 13) and fmt(5, 256, 4)[0] == 3 and fmt(4, 512, 6) == (5, 4, 16)
    assert fmt(4, 512, 44) == (5, 4, 16) and L.concrete_hip_pbs_supported(4, 512, 44, 1) == 1  # one level at a time
    assert L.concrete_hip_fourier_bsk_size_bytes(700, 4, 2, 512) == 700 * 2 * 5 * 25 * 256 * 16
    assert L.concrete_hip_pbs_supported(4, 512, 2, 16) == 1
    assert L.concrete_hip_fourier_bsk_size_bytes(700, 4, 3, 512) == 700 * 3 * 4 * 25 * 256 * 16
    assert L.concrete_hip_pbs_supported(6, 256, 3, 9) == 1 and L.concrete_hip_pbs_supported(4, 512, 5, 8) == 1
    assert L.concrete_hip_pbs_supported(6, 256, 3, 15) == 1  # past the levels gate: the companion key
    assert L.concrete_hip_fourier_bsk_size_bytes(722, 3, 1, 512) == 722 * 4 * 16 * 256 * 16
    assert L.concrete_hip_pbs_supported(3, 512, 1, 24) == 1 and L.concrete_hip_pbs_supported(5, 256, 1, 15) == 1
    assert L.concrete_hip_pbs_supported(5, 256, 1, 25) == 1  # past the small-ring gate: the general path
    for k, N, l, logB in [(6, 256, 4, 8), (1, 2048, 8, 5), (3, 512, 5, 8), (1, 4096, 1, 22),
                          (1, 8192, 1, 22), (1, 16384, 2, 15), (1, 2048, 5, 8)]:
        kind, limbs, bits = fmt(k, N, l)
        assert kind == 3 and limbs * bits >= 64, (k, N, l)
        assert L.concrete_hip_pbs_supported(k, N, l, logB) == 1, (k, N, l, logB)
        assert 0 < L.concrete_hip_generic_error_bound(k, N, l, logB, 0.0) < 0.25
        assert L.concrete_hip_fourier_bsk_size_bytes(10, k, l, N) == 10 * l * (k + 1) ** 2 * limbs * (N // 2) * 16
    assert fmt(1, 32768, 2)[0] == 3 and fmt(1, 65536, 2)[0] == 3
    assert L.concrete_hip_pbs_supported(1, 32768, 2, 15) == 1  # v0_last_128 9-bit row
    assert L.concrete_hip_pbs_supported(1, 65536, 2, 14) == 1  # 10-bit row
    assert fmt(1, 131072, 2)[0] == 0
    assert L.concrete_hip_pbs_supported(1, 4096, 1, 40) == 0


def test_committed_pmc_records_match_the_kernel_sources():
    """bench.py reports roofline.traffic / dram / valu only from a PMC record measured on the
    current kernel sources (bench.KERNEL_SOURCES, hashed per config): a kernel edit without a new
    record would silently drop those fields from the round's bench line."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    for config in ("cfg2", "cfg4"):
        assert bench.pmc_traffic(4096, config)[0], f"no PMC traffic record for the current {config} sources"
        assert bench.pmc_f64_flop(4096, config)[0], f"no PMC f64 record for the current {config} sources"


def test_pmc_records_not_attached_under_dispatch_overrides(monkeypatch):
    """A record measured on the default dispatch does not describe a run whose environment switches
    kernels (an A/B library, the two-launch path at N = 8192, a forced cfg2 kernel): bench.py then
    reports no traffic / f64 fields rather than another kernel's."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    assert bench.pmc_traffic(1024, "opt7")[0]
    for var, val in (("CONCRETE_HIP_GEN_COOP", "0"), ("CONCRETE_HIP_LIB", "/tmp/x.so"), ("CONCRETE_HIP_PBS_HEX", "2")):
        monkeypatch.setenv(var, val)
        assert bench.pmc_traffic(1024, "opt7") == (None, None) and bench.pmc_f64_flop(1024, "opt7") == (None, None)
        monkeypatch.delenv(var)
    # cfg2 at a batch split over two kernels has no single-kernel record to scale
    assert bench.dispatched_kernel(1280, "cfg2", 256) is None or bench.pmc_f64_flop(1280, "cfg2")[0] is None


def test_optimizer_table_coverage():
    """Every row of the optimizer's reference table (tests/golden/v0_last_128_rows.json, from
    v0-parameters/ref/v0_last_128 by tests/golden/make_v0_rows.py) from 1 to 8 bits, at every log
    norm2, has a PBS (k, N, br_l, br_b) and a keyswitch (ks_l, ks_b, kN -> n) the backend runs
    exactly, and so does every 9- and 10-bit row (N = 2^15, 2^16: the split path, round 4)."""
    import json

    L = _native.lib()
    rows = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "v0_last_128_rows.json")))["rows"]
    assert len(rows) == 235
    runs = lambda r: (L.concrete_hip_pbs_supported(r["k"], r["N"], r["br_l"], r["br_b"]) == 1 and  # noqa: E731
                      L.concrete_hip_keyswitch_supported(r["ks_l"], r["ks_b"], r["k"] * r["N"], r["n"]) == 1)
    small = [r for r in rows if r["bits"] <= 8]
    assert len(small) == 204
    assert [r for r in small if not runs(r)] == []
    big = [r for r in rows if r["bits"] > 8]
    assert len(big) == 31 and all(r["N"] >= 32768 for r in big)
    assert [r for r in big if not runs(r)] == []


def test_optimizer_rows_on_hand_tuned_kernels():
    """Round 4's dispatch census: 135 of the 235 table rows get a hand-tuned
    key format (small-ring 89, k = 2 at N = 1024: 27, N = 2048: 19); the rows left to the general
    path at N <= 2048 are N = 2048's many-level ones (l >= 5)."""
    import json
    from collections import Counter

    L = _native.lib()
    rows = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "v0_last_128_rows.json")))["rows"]
    fmt = lambda r: L.concrete_hip_bsk_format(r["k"], r["N"], r["br_l"], C.byref(C.c_uint32()),  # noqa: E731
                                              C.byref(C.c_uint32()))
    census = Counter(fmt(r) for r in rows)
    assert census[5] == 89 and census[4] == 27 and census[2] == 19 and census[3] == 100, census
    for r in rows:
        if fmt(r) == 3 and r["N"] <= 2048:
            assert r["N"] == 2048 and r["br_l"] >= 5, r
        if fmt(r) != 3:
            assert L.concrete_hip_pbs_supported(r["k"], r["N"], r["br_l"], r["br_b"]) == 1, r
