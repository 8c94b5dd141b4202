"""CPU tests of the oracle (the CPU restatement of concrete-cpu / tfhe 0.10 semantics).

Pinned by: the reference's own golden noise-model tests (blind_rotate.rs:38-109), the
reference fixture generators' cleartext vectors (tests/golden/reference_lut_fixtures.json),
closed-form restatements of simulation.cpp / Transformers.cpp / wrappers.cpp, and agreement
of two independent exact integer product paths (schoolbook definition, Karatsuba).
"""
import json
import math
import os

import numpy as np
import pytest

from oracle import noise_model as NM

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "reference_lut_fixtures.json")
M64 = (1 << 64) - 1


def test_noise_model_golden_bootstrap_1():
    # blind_rotate.rs:38-72 security_variance_bootstrap_1
    var_bsk = NM.minimal_variance_glwe(2, 1 << 12, 64)
    actual = NM.variance_blind_rotate(2048, 2, 1 << 12, 24, 2, 64, 53, var_bsk)
    assert math.isclose(NM.variance_to_modular_variance(actual, 64), 4.078_296_369_990_673e31, rel_tol=1e-8)


def test_noise_model_golden_bootstrap_2():
    # blind_rotate.rs:74-108 golden_python_prototype_security_variance_bootstrap_2 (log q = 128).
    # The golden value equals the formula WITHOUT the FFT term (rel. err 3e-15); with the FFT term
    # of external_product_glwe.rs:62-89 as written it would be 1.89e59.  The exact-arithmetic part
    # is the one that models this backend, so that is what the golden vector pins here.
    var_bsk = NM.minimal_variance_glwe(4, 1 << 12, 128)
    actual = NM.variance_blind_rotate(1024, 4, 1 << 12, 5, 9, 128, 53, var_bsk, exact=True)
    assert math.isclose(NM.variance_to_modular_variance(actual, 128), 3.269_722_907_894_341e55, rel_tol=1e-8)


def test_secure_std_matches_curve(oracle):
    for size in (450, 630, 742, 1024, 2048, 4096):
        assert math.isclose(oracle.lib().ora_secure_log2_std(1, size), NM.secure_log2_std(size, 64.0))


def py_modswitch_simulation(x, N):
    # compiler lib/Runtime/simulation.cpp:64-75 (noise-free part)
    shift = 64 - int(math.log2(N)) - 2
    ms = x >> shift
    ms += ms & 1
    ms >>= 1
    return ms % (2 * N)


def test_modswitch_matches_simulation(oracle):
    rng = np.random.RandomState(1)
    xs = [int(v) for v in rng.randint(0, 2 ** 63, size=2000, dtype=np.int64)] + [0, M64, 1 << 63, (1 << 52) - 1, 1 << 52]
    xs += [int(v) * 2 for v in rng.randint(0, 2 ** 62, size=500, dtype=np.int64)]
    for N in (256, 1024, 2048):
        for x in xs:
            assert oracle.lib().ora_modswitch(x, N) == py_modswitch_simulation(x, N)


def py_decompose(x, l, logB):
    """Independent restatement of tfhe 0.10 SignedDecomposer (closest_representable + balanced digits)."""
    nrep = 64 - l * logB
    state = (x >> nrep) + ((x >> (nrep - 1)) & 1)
    B = 1 << logB
    out = []
    for _ in range(l):
        res = state & (B - 1)
        state >>= logB
        carry = (((res - 1) & M64) | state) & res
        carry >>= logB - 1
        state += carry
        out.append(res - (carry << logB))
    return out


@pytest.mark.parametrize("l,logB", [(3, 7), (1, 23), (4, 3), (5, 3), (2, 15)])
def test_decomposition(oracle, l, logB):
    import ctypes as C
    rng = np.random.RandomState(l * 100 + logB)
    xs = [int(v) for v in rng.randint(-2 ** 63, 2 ** 63 - 1, size=3000, dtype=np.int64).view(np.uint64)]
    xs += [0, M64, 1 << 63, (1 << 63) - 1]
    dig = np.zeros(l, dtype=np.int64)
    nrep = 64 - l * logB
    for x in xs:
        oracle.lib().ora_decompose(C.c_uint64(x), l, logB, dig.ctypes.data_as(oracle.i64p))
        ref = py_decompose(x, l, logB)
        assert list(dig) == ref
        assert all(-(1 << (logB - 1)) <= d <= (1 << (logB - 1)) for d in ref)
        # recomposition == closest representable value (round half up at the dropped bits)
        rec = sum(d << (64 - logB * (l - q)) for q, d in enumerate(ref)) & M64
        closest = (((x >> nrep) + ((x >> (nrep - 1)) & 1)) << nrep) & M64
        assert rec == closest


def negacyclic_py(d, g, N):
    out = [0] * N
    for m in range(N):
        if d[m] == 0:
            continue
        for j in range(N):
            if j >= m:
                out[j] += d[m] * g[j - m]
            else:
                out[j] -= d[m] * g[N + j - m]
    return [v & M64 for v in out]


def test_polymul_paths_agree(oracle):
    rng = np.random.RandomState(7)
    for N in (16, 64, 256):
        d = rng.randint(-64, 65, size=N).astype(np.int64)
        g = rng.randint(0, 2 ** 63, size=N, dtype=np.int64).astype(np.uint64) * np.uint64(2) + np.uint64(1)
        a = np.zeros(N, dtype=np.uint64)
        b = np.zeros(N, dtype=np.uint64)
        oracle.lib().ora_polymul_acc_schoolbook(oracle.P(a), d.ctypes.data_as(oracle.i64p), oracle.P(g), N)
        oracle.lib().ora_polymul_acc_karatsuba(oracle.P(b), d.ctypes.data_as(oracle.i64p), oracle.P(g), N)
        ref = negacyclic_py([int(v) for v in d], [int(v) for v in g], N) if N <= 64 else None
        assert np.array_equal(a, b)
        if ref is not None:
            assert [int(v) for v in a] == ref


def test_monomial_roundtrip(oracle):
    N = 64
    rng = np.random.RandomState(3)
    p = rng.randint(0, 2 ** 62, size=N, dtype=np.int64).astype(np.uint64)
    t = np.zeros(N, dtype=np.uint64)
    u = np.zeros(N, dtype=np.uint64)
    for d in (0, 1, 5, N - 1, N, N + 3, 2 * N - 1):
        oracle.lib().ora_monomial_mul(oracle.P(t), oracle.P(p), d, N)
        oracle.lib().ora_monomial_div(oracle.P(u), oracle.P(t), d, N)
        assert np.array_equal(u, p)
        # X^d * p == schoolbook product with the monomial
        mono = [0] * N
        sign = 1 if (d // N) % 2 == 0 else -1
        mono[d % N] = sign
        assert [int(v) for v in t] == negacyclic_py(mono, [int(v) for v in p], N)


def test_limb_split_recombines(oracle):
    rng = np.random.RandomState(5)
    xs = [int(v) for v in rng.randint(-2 ** 63, 2 ** 63 - 1, size=2000, dtype=np.int64).view(np.uint64)] + [0, M64, 1 << 63]
    for L in (3, 4, 6):
        w = [64 // L + (1 if i < 64 % L else 0) for i in range(L)]
        limbs = np.zeros(L, dtype=np.int64)
        for x in xs:
            oracle.lib().ora_limb_split(x, L, limbs.ctypes.data_as(oracle.i64p))
            s = 0
            sh = 0
            for i in range(L):
                assert -(1 << (w[i] - 1)) <= limbs[i] < (1 << (w[i] - 1))
                s += int(limbs[i]) << sh
                sh += w[i]
            assert s & M64 == x


def test_encode_decode_transformers(oracle):
    for width in range(1, 9):
        for m in range(1 << width):
            e = int(oracle.encode(m, width))
            assert e == (m << (64 - (width + 1))) & M64
            assert oracle.decode(e, width) == m
            # noise within half a box decodes to m
            assert oracle.decode((e + (1 << (64 - width - 3))) & M64, width) == m


def py_expand_lut(table, out_size, bits, signed=False):
    # compiler lib/Runtime/wrappers.cpp:388-450
    n_in = len(table)
    mega = out_size // n_in
    idx = (lambda i: i + n_in // 2 if i < n_in // 2 else i - n_in // 2) if signed else (lambda i: i)
    out = [0] * out_size
    sh = 64 - bits - 1
    for o in range(mega // 2):
        out[o] = (table[idx(0)] << sh) & M64
    for o in range((n_in - 1) * mega + mega // 2, out_size):
        out[o] = (-(table[idx(0)] << sh)) & M64
    for li in range(1, n_in):
        v = (table[idx(li)] << sh) & M64
        st = mega * (li - 1) + mega // 2
        for o in range(st, st + mega):
            out[o] = v
    return out


@pytest.mark.parametrize("signed", [False, True])
def test_expand_lut(oracle, signed):
    rng = np.random.RandomState(2)
    for bits in (1, 2, 3, 5):
        table = [int(v) for v in rng.randint(0, 1 << bits, size=1 << bits)]
        got = oracle.expand_lut(np.array(table, dtype=np.uint64), 1024, bits, signed)
        assert [int(v) for v in got] == py_expand_lut(table, 1024, bits, signed)


def small_setup(oracle, p, std_bsk=2.0 ** -40):
    lwe_sk = oracle.binary_key(p.n, 11)
    glwe_sk = oracle.binary_key(p.k * p.N, 12)
    bsk = oracle.keygen_bsk(p, lwe_sk, glwe_sk, 13, std=std_bsk)
    fbsk = oracle.bsk_to_fourier(p, bsk)
    return lwe_sk, glwe_sk, bsk, fbsk


def test_pbs_three_paths_agree_small(oracle):
    p = oracle.SMALL
    lwe_sk, glwe_sk, bsk, fbsk = small_setup(oracle, p)
    width = 3
    table = np.array([3, 1, 4, 1, 5, 0, 2, 6], dtype=np.uint64)
    acc = oracle.trivial_glwe(p, oracle.expand_lut(table, p.N, width))[None, :]
    msgs = np.arange(8)
    cts = oracle.lwe_encrypt_batch(lwe_sk, [oracle.encode(m, width) for m in msgs], p.n, 2.0 ** -30, 5)
    cts[3, :4] = 0  # zero mask elements exercise the tfhe skip rule
    outs = [oracle.pbs_batch(p, cts, acc, bsk=bsk, fbsk=fbsk, mode=m)[0] for m in (0, 1, 2)]
    assert np.array_equal(outs[0], outs[1]) and np.array_equal(outs[1], outs[2])
    dec = oracle.lwe_decrypt_batch(glwe_sk, outs[2], p.big_n)
    assert [oracle.decode(d, width) for d in dec] == [int(table[m]) for m in msgs]


def test_fft_product_exact_adversarial_digits(oracle):
    """Exact-limb FFT == Karatsuba for the worst-case digit magnitudes at cfg2's N."""
    import ctypes as C
    from dataclasses import replace
    p = replace(oracle.CFG2, n=2)
    lwe_sk = oracle.binary_key(p.n, 1)
    glwe_sk = oracle.binary_key(p.N, 2)
    bsk = oracle.keygen_bsk(p, lwe_sk, glwe_sk, 3)
    fbsk = oracle.bsk_to_fourier(p, bsk)
    assert oracle.fft_error_bound(p, fbsk) < 0.5
    gsz = (p.k + 1) * p.N
    for trial in range(4):
        # ct1 whose digits all sit at +-B/2 (largest ||d||_2) or random
        rng = np.random.RandomState(trial)
        if trial < 2:
            half = 1 << (p.logB - 1)
            digs = rng.choice([-half, half], size=(gsz, p.l))
            ct1 = np.array([sum(int(d) << (64 - p.logB * (p.l - q)) for q, d in enumerate(row)) & M64
                            for row in digs], dtype=np.uint64)
        else:
            ct1 = rng.randint(-2 ** 63, 2 ** 63 - 1, size=gsz, dtype=np.int64).view(np.uint64)
        a = np.zeros(gsz, dtype=np.uint64)
        b = np.zeros(gsz, dtype=np.uint64)
        resid = C.c_double(0)
        L = oracle.lib()
        L.ora_external_product_acc(oracle.P(a), oracle.P(bsk), None, oracle.P(ct1), p.k, p.N, p.l, p.logB, p.limbs,
                                   oracle.MODE_KARATSUBA, None)
        L.ora_external_product_acc(oracle.P(b), None, oracle.P(fbsk, oracle.f64p), oracle.P(ct1), p.k, p.N, p.l,
                                   p.logB, p.limbs, oracle.MODE_FFT, C.byref(resid))
        assert np.array_equal(a, b)
        assert resid.value < 0.01


def test_pbs_cfg2_fft_equals_karatsuba_and_decrypts(oracle):
    p = oracle.CFG2
    lwe_sk = oracle.binary_key(p.n, 101)
    glwe_sk = oracle.binary_key(p.k * p.N, 102)
    bsk = oracle.keygen_bsk(p, lwe_sk, glwe_sk, 103)
    fbsk = oracle.bsk_to_fourier(p, bsk)
    bound = oracle.fft_error_bound(p, fbsk)
    assert bound < 0.5
    width = 3
    rng = np.random.RandomState(0)
    table = rng.randint(0, 8, size=8).astype(np.uint64)
    acc = oracle.trivial_glwe(p, oracle.expand_lut(table, p.N, width))[None, :]
    msgs = np.arange(16) % 8
    cts = oracle.lwe_encrypt_batch(lwe_sk, [oracle.encode(m, width) for m in msgs], p.n, oracle.lwe_std_torus(p), 104)
    out, resid = oracle.pbs_batch(p, cts, acc, bsk=bsk, fbsk=fbsk, mode=oracle.MODE_FFT)
    assert resid < bound
    kara, _ = oracle.pbs_batch(p, cts[:1], acc, bsk=bsk, mode=oracle.MODE_KARATSUBA)
    assert np.array_equal(kara, out[:1])
    dec = oracle.lwe_decrypt_batch(glwe_sk, out, p.big_n)
    assert [oracle.decode(d, width) for d in dec] == [int(table[m]) for m in msgs]


def test_reference_fixtures_through_oracle_pbs(oracle):
    """Decrypt-level parity with the reference generators' cleartext vectors (p <= 3 at cfg2)."""
    from dataclasses import replace
    fx = json.load(open(GOLDEN))
    p = oracle.CFG2
    lwe_sk = oracle.binary_key(p.n, 201)
    glwe_sk = oracle.binary_key(p.k * p.N, 202)
    bsk = oracle.keygen_bsk(p, lwe_sk, glwe_sk, 203)
    fbsk = oracle.bsk_to_fourier(p, bsk)
    cases = [c for c in fx["linalg_apply_lookup_table"] if c["description"].endswith("_1layer")]
    cases = [c for c in cases if len(c["lut"]) <= 8]
    assert cases
    for ci, c in enumerate(cases):
        width = int(math.log2(len(c["lut"])))
        xs = c["input"][:8]
        acc = oracle.trivial_glwe(p, oracle.expand_lut(np.array(c["lut"], dtype=np.uint64), p.N, width))[None, :]
        cts = oracle.lwe_encrypt_batch(lwe_sk, [oracle.encode(x, width) for x in xs], p.n,
                                       oracle.lwe_std_torus(p), 300 + ci)
        out, _ = oracle.pbs_batch(p, cts, acc, fbsk=fbsk, mode=oracle.MODE_FFT)
        dec = oracle.lwe_decrypt_batch(glwe_sk, out, p.big_n)
        assert [oracle.decode(d, width) for d in dec] == c["expected"][:8], c["description"]


def test_keyswitch_decrypts(oracle):
    p = oracle.CFG2
    big_sk = oracle.binary_key(p.big_n, 401)
    small_sk = oracle.binary_key(p.n, 402)
    ksk = oracle.keygen_ksk(p, big_sk, small_sk, 403)
    width = 2
    msgs = [0, 1, 2, 3, 3, 2, 1, 0]
    cts = oracle.lwe_encrypt_batch(big_sk, [oracle.encode(m, width) for m in msgs], p.big_n, 2.0 ** -40, 404)
    out = oracle.keyswitch_batch(p, cts, ksk)
    dec = oracle.lwe_decrypt_batch(small_sk, out, p.n)
    assert [oracle.decode(d, width) for d in dec] == msgs


def test_pbs_output_noise_matches_model(oracle):
    """P4: empirical PBS output noise vs the reference model without the FFT term."""
    from dataclasses import replace
    p = replace(oracle.CFG2, n=64)
    lwe_sk = oracle.binary_key(p.n, 501)
    glwe_sk = oracle.binary_key(p.k * p.N, 502)
    bsk = oracle.keygen_bsk(p, lwe_sk, glwe_sk, 503)
    fbsk = oracle.bsk_to_fourier(p, bsk)
    width = 2
    table = np.array([0, 1, 2, 3], dtype=np.uint64)
    acc = oracle.trivial_glwe(p, oracle.expand_lut(table, p.N, width))[None, :]
    msgs = np.arange(48) % 4
    cts = oracle.lwe_encrypt_batch(lwe_sk, [oracle.encode(m, width) for m in msgs], p.n, 2.0 ** -30, 504)
    out, _ = oracle.pbs_batch(p, cts, acc, fbsk=fbsk)
    dec = oracle.lwe_decrypt_batch(glwe_sk, out, p.big_n)
    err = [((int(d) - int(oracle.encode(table[m], width)) + (1 << 63)) % (1 << 64) - (1 << 63)) / 2.0 ** 64
           for d, m in zip(dec, msgs)]
    emp = float(np.var(err))
    var_bsk = 2.0 ** (2 * oracle.lib().ora_secure_log2_std(p.k, p.N))
    model = NM.variance_blind_rotate(p.n, p.k, p.N, p.logB, p.l, 64, 53, var_bsk, exact=True)
    # 48 samples: the sample variance is within a factor ~2 of the model with overwhelming probability
    assert model / 3 < emp < model * 3, (emp, model)


def test_cfg4_shape_fft_equals_karatsuba(oracle):
    """N = 2048, l = 1, logB = 23 (BASELINE configs[3]) with the oracle's 8-limb FFT path: its
    certified bound is < 1/2 and it agrees bit-for-bit with the integer Karatsuba product."""
    from dataclasses import replace
    p = replace(oracle.CFG4, n=10)
    assert p.limbs == oracle.limbs_for(p.N) == 8
    lwe = oracle.binary_key(p.n, 1)
    glwe = oracle.binary_key(p.big_n, 2)
    bsk = oracle.keygen_bsk(p, lwe, glwe, 3, std=2.0 ** -45)
    f = oracle.bsk_to_fourier(p, bsk)
    assert oracle.fft_error_bound(p, f) < 0.5
    width = 5
    table = np.arange(32, dtype=np.uint64)[::-1].copy()
    acc = oracle.trivial_glwe(p, oracle.expand_lut(table, p.N, width))
    msgs = np.array([0, 1, 17, 31])
    cts = oracle.lwe_encrypt_batch(lwe, [oracle.encode(int(m), width) for m in msgs], p.n, 2.0 ** -30, 7)
    r_fft, _ = oracle.pbs_batch(p, cts, acc[None, :], fbsk=f, mode=oracle.MODE_FFT)
    r_kar, _ = oracle.pbs_batch(p, cts, acc[None, :], bsk=bsk, mode=1)
    assert np.array_equal(r_fft, r_kar)
    dec = oracle.lwe_decrypt_batch(glwe, r_fft, p.big_n)
    assert [oracle.decode(int(d), width) for d in dec] == [int(table[m]) for m in msgs]


def test_generic_error_bound_matches_the_kernel_gate(oracle):
    """The certified bound the GPU tests evaluate (oracle/pyoracle.py) is the same formula the
    library's exactness gate uses (concrete_amd/csrc/pbs_generic.hip:generic_error_bound)."""
    import ctypes as C

    from concrete_amd import _native
    L = _native.lib()
    for k, N, l, logB in [(6, 256, 4, 8), (1, 2048, 8, 5), (3, 512, 5, 8), (1, 4096, 1, 22), (1, 16384, 2, 15),
                          (3, 512, 4, 9), (1, 2048, 5, 8)]:
        limbs, bits = C.c_uint32(), C.c_uint32()
        assert L.concrete_hip_bsk_format(k, N, l, C.byref(limbs), C.byref(bits)) == 3
        for maxg in (0.0, 1e5, 3e6):
            c_val = L.concrete_hip_generic_error_bound(k, N, l, logB, maxg)
            if maxg == 0.0:
                py = oracle.generic_error_bound(k, N, l, logB, bits.value)
            else:  # a one-value "key" whose spectrum magnitude is maxg (scaled by 1/M like the device key)
                py = oracle.generic_error_bound(k, N, l, logB, bits.value, np.array([maxg / (N / 2), 0.0]))
            assert abs(c_val - py) <= 1e-12 * max(1.0, abs(py)), (k, N, l, logB, maxg, c_val, py)


@pytest.mark.parametrize("cfg", ["CFG2", "CFG4"])
def test_pbs_fft64_mode_decrypts(oracle, cfg):
    """ORA_MODE_FFT64 (the CPU baseline bench.py times): concrete-cpu's fft64 arithmetic — one f64
    spectrum of the u64 key, f64 products rounded mod 2^64.  Not exact (its ciphertexts diverge from
    the exact path's after the first rounding difference changes a digit), but every output decrypts
    to the LUT value."""
    from dataclasses import replace
    p0 = getattr(oracle, cfg)
    p = replace(p0, n=64, limbs=1)
    lwe_sk = oracle.binary_key(p.n, 201)
    glwe_sk = oracle.binary_key(p.k * p.N, 202)
    bsk = oracle.keygen_bsk(p, lwe_sk, glwe_sk, 203)
    width = 3 if cfg == "CFG2" else 5
    rng = np.random.RandomState(1)
    table = rng.randint(0, 1 << width, size=1 << width).astype(np.uint64)
    acc = oracle.trivial_glwe(p, oracle.expand_lut(table, p.N, width))[None, :]
    msgs = np.arange(12) % (1 << width)
    cts = oracle.lwe_encrypt_batch(lwe_sk, [oracle.encode(m, width) for m in msgs], p.n, 2.0 ** -25, 204)
    out, _ = oracle.pbs_batch(p, cts, acc, fbsk=oracle.bsk_to_fourier(p, bsk), mode=oracle.MODE_FFT64)
    dec = oracle.lwe_decrypt_batch(glwe_sk, out, p.big_n)
    assert [oracle.decode(d, width) for d in dec] == [int(table[m]) for m in msgs]
