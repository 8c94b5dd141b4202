"""GPU parity tests of the small-ring kernels (concrete_amd/csrc/pbs_small.hip: N = 512, k = 3 and
N = 256, k = 5 / 6; pbs512k4.hip: N = 512, k = 4; l = 1) — the optimizer's 1- to 3-bit rows
(v0_last_128: opt3 n = 722 logB = 18, opt1 n = 592 logB = 15, k = 6 n = 596 logB = 18, k = 4 n = 731
logB = 23; bench.py --config opt3 / opt1) — vs the CPU oracle.

Bit-exact u64 equality with the oracle's pure-integer Karatsuba product on the same keys and
inputs, the measured rounding residual below the scheme's certified bound
(oracle/pyoracle.py:gpu_small_error_bound, itself < 1/2), decrypt(out) == LUT[m], the device key
layout against numpy transforms, both digit forms at N = 512 (one sub-digit at logB <= 15, two
above), ragged batches (four ciphertexts per workgroup; at k = 5 the second wave of each
ciphertext carries two empty polynomial slots), index arrays and mapped LUTs, edge inputs.
"""
from dataclasses import replace

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

# shape -> (message bits, optimizer row parameters): opt3, opt1, the k = 6 row of v0_last_128 at
# 1 bit, log norm2 2 (n = 596, br 1/18) and the k = 4 row at 3 bits, log norm2 3 (n = 731, br 1/23)
SHAPES = {"N512_k3": (3, None), "N256_k5": (1, None),
          "N256_k6": (1, dict(n=596, k=6, N=256, level=1, base_log=18, ks_level=3, ks_base_log=4)),
          "N512_k4": (3, dict(n=731, k=4, N=512, level=1, base_log=23, ks_level=3, ks_base_log=4))}


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a visible MI355X"
    return torch


@pytest.fixture(scope="module")
def B():
    from concrete_amd import backend
    return backend


class Setup:
    def __init__(self, B, oracle, torch, p, seed):
        self.p = p
        self.op = oracle.Params(n=p.n, k=p.k, N=p.N, l=p.level, logB=p.base_log)
        self.lwe_sk = B.binary_key(p.n, seed)
        self.glwe_sk = B.binary_key(p.big_n, seed + 1)
        self.bsk = B.bsk_generate(p, self.lwe_sk, self.glwe_sk, seed + 2)
        self.fbsk = B.convert_bsk(p, self.bsk, "cuda:0")
        torch.cuda.synchronize()


_cache = {}


def small_setup(B, oracle, torch, shape, n=None, base_log=None, seed=9000):
    key = (shape, n, base_log, seed)
    if key not in _cache:
        bits, explicit = SHAPES[shape]
        p = B.PbsParams(**explicit) if explicit else B.OPTIMIZER_SETS[bits]
        p = replace(p, n=n if n is not None else p.n, base_log=base_log if base_log is not None else p.base_log)
        _cache[key] = Setup(B, oracle, torch, p, seed)
    return _cache[key]


def encrypt(B, S, msgs, width, seed, std=None):
    std = B.secure_std(1, S.p.n) if std is None else std
    return B.lwe_encrypt(S.lwe_sk, [B.encode(m, width) for m in msgs], S.p.n, std, seed)


def lut_acc(B, S, table, width):
    return B.trivial_glwe(S.p, B.expand_lut(np.array(table, dtype=np.uint64), S.p.N, width))


def run_gpu(B, S, cts, luts, torch, lut_idx=None, in_idx=None, out_idx=None, resid=False):
    dev = "cuda:0"
    args = {}
    n_s = cts.shape[0] if in_idx is None else len(in_idx)
    for name, a in (("lut_idx", lut_idx), ("in_idx", in_idx), ("out_idx", out_idx)):
        if a is not None:
            args[name] = B.to_device(np.asarray(a, dtype=np.uint64), dev)
    out = torch.zeros((n_s, S.p.lwe_out_size), dtype=torch.int64, device=dev)
    r = torch.zeros(1, dtype=torch.int64, device=dev) if resid else None
    B.pbs(S.p, S.fbsk, B.to_device(cts, dev), B.to_device(np.atleast_2d(luts), dev), out=out, num_samples=n_s,
          resid=r, **args)
    torch.cuda.synchronize()
    res = B.to_host(out)
    if resid:
        return res, float(np.array([r.item()], dtype=np.int64).view(np.float64)[0])
    return res


def run_oracle(oracle, S, cts, luts, lut_idx=None, in_idx=None, out_idx=None):
    out, _ = oracle.pbs_batch(S.op, cts, np.atleast_2d(luts), bsk=S.bsk, mode=oracle.MODE_KARATSUBA,
                              lut_idx=lut_idx, in_idx=in_idx, out_idx=out_idx)
    return out


def bound(B, oracle, S):
    return oracle.gpu_small_error_bound(B.to_host(S.fbsk).view(np.float64), S.p.N, S.p.k, S.p.base_log, S.p.level)


def signed_limb(x, limb, limbs=4):
    rem = x.astype(np.uint64).copy()
    w = 64 // limbs
    val = None
    for _ in range(limb + 1):
        vv = (rem & np.uint64((1 << w) - 1)).astype(np.int64)
        sgn = np.where(vv >= (1 << (w - 1)), vv - (1 << w), vv)
        val = sgn
        rem = (rem - sgn.astype(np.uint64)) >> np.uint64(w)
    return val.astype(np.float64)


@pytest.mark.parametrize("shape", list(SHAPES))
def test_key_format_and_layout(B, oracle, torch_cuda, shape):
    """Device key [n][limb][col][row][slot][lane] == the 16-bit limb of key polynomial (row, col),
    folded (g_t + i g_{t+N/2}), twisted by zeta_2N^t and transformed (N/2 points), at frequency
    fft512_freq(lane, slot), divided by 512 P (P = 1024 / N).  (numpy's FFT is not correctly
    rounded: tolerance 1e-13.)"""
    S = small_setup(B, oracle, torch_cuda, shape, n=6)
    p = S.p
    N, K1, M, P = p.N, p.k + 1, p.N // 2, 1024 // p.N
    assert B.bsk_format(p) == (5, 4, 16)
    assert B.fourier_bsk_bytes(p) == p.n * 4 * K1 * K1 * M * 16
    got = B.to_host(S.fbsk).view(np.float64).reshape(p.n, 4, K1, K1, M // 64, 64, 2)
    bsk = S.bsk.reshape(p.n, 1, K1, K1, N)
    lane = np.arange(64)
    slot = np.arange(M // 64)
    K = (lane[None, :] >> 3) + 8 * (lane[None, :] & 7) + 64 * slot[:, None]
    tw = np.exp(1j * np.pi * np.arange(M) / N)
    worst = 0.0
    for i in (0, p.n - 1):
        for li in range(4):
            for col in range(K1):
                for row in range(K1):
                    lv = signed_limb(bsk[i, 0, row, col], li)
                    ref = np.fft.fft((lv[:M] + 1j * lv[M:]) * tw)[K] / (512.0 * P)
                    gg = got[i, li, col, row]
                    worst = max(worst, np.max(np.abs(gg[..., 0] + 1j * gg[..., 1] - ref)) / np.max(np.abs(ref)))
    assert worst < 1e-13, worst


@pytest.mark.parametrize("batch", [1, 3, 4, 9])
@pytest.mark.parametrize("shape", list(SHAPES))
def test_bit_exact_small(B, oracle, torch_cuda, shape, batch):
    """Ragged batches: 1, 3 and 9 leave ciphertext slots of the last workgroup empty."""
    S = small_setup(B, oracle, torch_cuda, shape, n=14)
    width = 3
    rng = np.random.RandomState(batch)
    table = rng.randint(0, 8, size=8)
    msgs = rng.randint(0, 8, size=batch)
    cts = encrypt(B, S, msgs, width, 10 + batch, std=2.0 ** -30)
    acc = lut_acc(B, S, table, width)
    got, resid = run_gpu(B, S, cts, acc, torch_cuda, resid=True)
    assert np.array_equal(got, run_oracle(oracle, S, cts, acc))
    assert resid < bound(B, oracle, S) < 0.5
    dec = B.lwe_decrypt(S.glwe_sk, got, S.p.big_n)
    assert [B.decode(d, width) for d in dec] == [int(table[m]) for m in msgs]


@pytest.mark.parametrize("shape,logB", [("N512_k3", 6), ("N512_k3", 15), ("N512_k3", 16), ("N512_k3", 24),
                                        ("N256_k5", 4), ("N256_k5", 12), ("N256_k5", 16), ("N256_k5", 24),
                                        ("N256_k6", 15), ("N256_k6", 24),
                                        ("N512_k4", 4), ("N512_k4", 15), ("N512_k4", 16), ("N512_k4", 24)])
def test_digit_forms(B, oracle, torch_cuda, shape, logB):
    """One sub-digit up to logB = 15, the split d = d_lo + 2^16 d_hi from 16 (|d_hi| = 1 at the tie)
    to the largest accepted 24, at both ring sizes."""
    S = small_setup(B, oracle, torch_cuda, shape, n=10, base_log=logB, seed=9100 + logB)
    width = 2
    rng = np.random.RandomState(logB)
    msgs = rng.randint(0, 4, size=6)
    cts = encrypt(B, S, msgs, width, 50 + logB, std=2.0 ** -30)
    acc = lut_acc(B, S, rng.randint(0, 4, size=4), width)
    got, resid = run_gpu(B, S, cts, acc, torch_cuda, resid=True)
    assert np.array_equal(got, run_oracle(oracle, S, cts, acc))
    assert resid < bound(B, oracle, S) < 0.5


def test_n256_wide_digits_run_on_the_general_path(B, oracle, torch_cuda):
    """N = 256, k = 5 past the kernel's gate (logB = 25): through a keyset (memref route) the call
    runs on the general path's companion key, built from the keyset's standard key; bit-exact."""
    from concrete_amd import runtime as R
    p = replace(B.OPTIMIZER_SETS[1], n=8, base_log=25)
    assert B.pbs_supported(p)
    lwe_sk = B.binary_key(p.n, 9300)
    glwe_sk = B.binary_key(p.big_n, 9301)
    bsk = B.bsk_generate(p, lwe_sk, glwe_sk, 9302)
    width = 2
    rng = np.random.RandomState(25)
    table = rng.randint(0, 4, size=4).astype(np.uint64)
    tlu = B.expand_lut(table, p.N, width)
    msgs = rng.randint(0, 4, size=5)
    cts = B.lwe_encrypt(lwe_sk, [B.encode(m, width) for m in msgs], p.n, 2.0 ** -30, 77)
    op = oracle.Params(n=p.n, k=p.k, N=p.N, l=p.level, logB=p.base_log)
    ref, _ = oracle.pbs_batch(op, cts, B.trivial_glwe(p, tlu)[None, :], bsk=bsk, mode=oracle.MODE_KARATSUBA)
    ks = R.Keyset([0])
    try:
        ks.add_bsk(0, bsk, p)
        got = R.batched_bootstrap(ks, p, cts, tlu)
    finally:
        ks.close()
    assert np.array_equal(got, ref)


@pytest.mark.parametrize("shape", list(SHAPES))
def test_index_arrays_and_mapped_luts(B, oracle, torch_cuda, shape):
    S = small_setup(B, oracle, torch_cuda, shape, n=14)
    width = 2
    nb = 7
    rng = np.random.RandomState(9)
    msgs = rng.randint(0, 4, size=nb)
    cts = encrypt(B, S, msgs, width, 41, std=2.0 ** -30)
    luts = np.stack([lut_acc(B, S, rng.randint(0, 4, size=4), width) for _ in range(nb)])
    lut_idx = rng.permutation(nb).astype(np.uint64)
    in_idx = rng.permutation(nb).astype(np.uint64)
    out_idx = rng.permutation(nb).astype(np.uint64)
    got = run_gpu(B, S, cts, luts, torch_cuda, lut_idx=lut_idx, in_idx=in_idx, out_idx=out_idx)
    ref = run_oracle(oracle, S, cts, luts, lut_idx=lut_idx, in_idx=in_idx, out_idx=out_idx)
    assert np.array_equal(got, ref)


@pytest.mark.parametrize("shape", list(SHAPES))
def test_edge_inputs(B, oracle, torch_cuda, shape):
    S = small_setup(B, oracle, torch_cuda, shape, n=14)
    p = S.p
    width = 2
    rng = np.random.RandomState(5)
    cts = encrypt(B, S, rng.randint(0, 4, size=8), width, 31, std=2.0 ** -30)
    cts[0, : p.n // 2] = 0
    cts[1, :] = 0
    cts[2, :] = np.uint64(0xFFFFFFFFFFFFFFFF)
    cts[3, : p.n] = np.uint64(1)
    cts[4, : p.n] = np.uint64((1 << 54) - 1)
    cts[5, p.n] = np.uint64(0xFFFFFFFFFFFFFFFF - 5)
    cts[6, : p.n] = np.uint64(1 << 63)
    cts[7, : p.n] = np.uint64(3 << 53)
    acc = lut_acc(B, S, [3, 1, 0, 2], width)
    got = run_gpu(B, S, cts, acc, torch_cuda)
    assert np.array_equal(got, run_oracle(oracle, S, cts, acc))


@pytest.mark.parametrize("shape", list(SHAPES))
def test_full_row_bit_exact_and_bound(B, oracle, torch_cuda, shape):
    """The full optimizer row (opt3: n = 722; opt1: n = 592; k = 6: n = 596; k = 4: n = 731): 512 samples decrypted, 3 bit-exact
    vs the exact oracle, the measured residual under the certified bound (< 1/2)."""
    S = small_setup(B, oracle, torch_cuda, shape)
    width = SHAPES[shape][0]
    rng = np.random.RandomState(3)
    table = rng.randint(0, 1 << width, size=1 << width)
    nb = 512
    msgs = rng.randint(0, 1 << width, size=nb)
    cts = encrypt(B, S, msgs, width, 77)
    acc = lut_acc(B, S, table, width)
    got, resid = run_gpu(B, S, cts, acc, torch_cuda, resid=True)
    b = bound(B, oracle, S)
    assert resid < b < 0.5, (resid, b)
    dec = B.lwe_decrypt(S.glwe_sk, got, S.p.big_n)
    assert [B.decode(d, width) for d in dec] == [int(table[m]) for m in msgs]
    pick = np.array([0, 1, nb - 1])
    assert np.array_equal(got[pick], run_oracle(oracle, S, cts[pick], acc))


@pytest.mark.parametrize("n", [1, 2, 3])
@pytest.mark.parametrize("shape", list(SHAPES))
def test_tiny_n(B, oracle, torch_cuda, shape, n):
    """Blind rotations of 1-3 steps: the key ring's prologue (DIST groups in flight) and its tail
    meet within one or two steps."""
    S = small_setup(B, oracle, torch_cuda, shape, n=n, seed=9400 + n)
    width = 2
    rng = np.random.RandomState(n)
    msgs = rng.randint(0, 4, size=5)
    cts = encrypt(B, S, msgs, width, 60 + n, std=2.0 ** -30)
    acc = lut_acc(B, S, rng.randint(0, 4, size=4), width)
    got = run_gpu(B, S, cts, acc, torch_cuda)
    assert np.array_equal(got, run_oracle(oracle, S, cts, acc))


# ---- N = 512, k = 4 at l = 3 .. 5 (pbs512k4.hip's levels: the rows at br 3/12, 4/9, 5/8) ----------
K4_LEVEL_ROWS = {2: (16, 700), 3: (12, 700), 4: (9, 702), 5: (8, 689)}  # level -> (logB, a 3-bit row's n)


def limb13(x, limb):
    """Balanced limb of u64 values on the 5-limb grid (13, 13, 13, 13, 12 bits; bsk.hip limb_value)."""
    rem = x.astype(np.uint64).copy()
    val = None
    for t in range(limb + 1):
        w = 13 if t < 4 else 12
        vv = (rem & np.uint64((1 << w) - 1)).astype(np.int64)
        val = np.where(vv >= (1 << (w - 1)), vv - (1 << w), vv)
        rem = (rem - val.astype(np.uint64)) >> np.uint64(w)
    return val.astype(np.float64)


def k4_level_setup(B, oracle, torch, level, n, seed):
    key = ("k4l", level, n, seed)
    if key not in _cache:
        logB = K4_LEVEL_ROWS[level][0]
        p = B.PbsParams(n=n, k=4, N=512, level=level, base_log=logB, ks_level=3, ks_base_log=4)
        _cache[key] = Setup(B, oracle, torch, p, seed)
    return _cache[key]


@pytest.mark.parametrize("level", [2, 3, 4, 5])
def test_k4_levels_key_layout(B, oracle, torch_cuda, level):
    """[n][limb][col][q][row][slot][lane] (l = 2, five 13-bit limbs) or level-major
    [n][q][limb][col][row][slot][lane] (l >= 3): level v = l - 1 - q of key polynomial (row, col)."""
    S = k4_level_setup(B, oracle, torch_cuda, level, 3, 9600 + level)
    p = S.p
    K1, M, N = 5, 256, 512
    L = 5 if level == 2 else 4
    assert B.bsk_format(p) == ((5, 5, 13) if level == 2 else (5, 4, 16))
    assert B.fourier_bsk_bytes(p) == p.n * level * L * 25 * M * 16
    got = B.to_host(S.fbsk).view(np.float64)
    if level >= 3:  # the one-level-at-a-time kernel's level-major key, [n][q][limb][col][row]
        got = got.reshape(p.n, level, L, K1, K1, 4, 64, 2).transpose(0, 2, 3, 1, 4, 5, 6, 7)
    else:
        got = got.reshape(p.n, L, K1, level, K1, 4, 64, 2)
    bsk = S.bsk.reshape(p.n, level, K1, K1, N)
    lane = np.arange(64)
    K = (lane[None, :] >> 3) + 8 * (lane[None, :] & 7) + 64 * np.arange(4)[:, None]
    tw = np.exp(1j * np.pi * np.arange(M) / N)
    worst = 0.0
    for i in (0, p.n - 1):
        for li in (0, L - 1):
            for col in (0, 4):
                for q in range(level):
                    for row in (0, 3):
                        src = bsk[i, level - 1 - q, row, col]
                        lv = limb13(src, li) if L == 5 else signed_limb(src, li)
                        ref = np.fft.fft((lv[:M] + 1j * lv[M:]) * tw)[K] / 1024.0
                        gg = got[i, li, col, q, row]
                        worst = max(worst, np.max(np.abs(gg[..., 0] + 1j * gg[..., 1] - ref)) / np.max(np.abs(ref)))
    assert worst < 1e-13, worst


@pytest.mark.parametrize("n", [1, 2, 9])
@pytest.mark.parametrize("level", [2, 3, 4, 5])
def test_k4_levels_bit_exact(B, oracle, torch_cuda, level, n):
    """Bit-exact vs the exact oracle over ring prologues / tails (n = 1, 2) and a longer rotation, odd
    batch (the last workgroup's second ciphertext empty), residual under the certified bound."""
    S = k4_level_setup(B, oracle, torch_cuda, level, n, 9700 + 10 * level + n)
    width = 2
    rng = np.random.RandomState(level * 10 + n)
    msgs = rng.randint(0, 4, size=5)
    cts = encrypt(B, S, msgs, width, 80 + n, std=2.0 ** -30)
    acc = lut_acc(B, S, rng.randint(0, 4, size=4), width)
    got, resid = run_gpu(B, S, cts, acc, torch_cuda, resid=True)
    assert np.array_equal(got, run_oracle(oracle, S, cts, acc))
    assert resid < bound(B, oracle, S) < 0.5


@pytest.mark.parametrize("level", [2, 3, 5])
def test_k4_levels_full_row(B, oracle, torch_cuda, level):
    """The full 3-bit rows (br 2/16 n = 700, br 3/12 n = 700, br 5/8 n = 689): 256 samples decrypted, 2 bit-exact, residual
    under the bound."""
    S = k4_level_setup(B, oracle, torch_cuda, level, K4_LEVEL_ROWS[level][1], 9800 + level)
    width = 3
    rng = np.random.RandomState(level)
    table = rng.randint(0, 8, size=8)
    msgs = rng.randint(0, 8, size=256)
    cts = encrypt(B, S, msgs, width, 90 + level)
    acc = lut_acc(B, S, table, width)
    got, resid = run_gpu(B, S, cts, acc, torch_cuda, resid=True)
    b = bound(B, oracle, S)
    assert resid < b < 0.5, (resid, b)
    dec = B.lwe_decrypt(S.glwe_sk, got, S.p.big_n)
    assert [B.decode(d, width) for d in dec] == [int(table[m]) for m in msgs]
    assert np.array_equal(got[:2], run_oracle(oracle, S, cts[:2], acc))


# ---- pbs_small.hip at l = 2, 3 (whole digits; the rows at br 2/10, 2/12, 3/9) ---------------------
SM_LEVEL_ROWS = {  # label -> (k, N, l, logB, an optimizer row's n, its message bits)
    "k5_N256_l2": (5, 256, 2, 10, 594, 1), "k6_N256_l2": (6, 256, 2, 12, 614, 1),
    "k6_N256_l3": (6, 256, 3, 9, 601, 1), "k3_N512_l2": (3, 512, 2, 12, 739, 3),
    "k3_N512_l3": (3, 512, 3, 9, 700, 3)}


def sm_level_setup(B, oracle, torch, label, n, seed):
    key = ("sml", label, n, seed)
    if key not in _cache:
        k, N, level, logB = SM_LEVEL_ROWS[label][:4]
        p = B.PbsParams(n=n, k=k, N=N, level=level, base_log=logB, ks_level=3, ks_base_log=4)
        _cache[key] = Setup(B, oracle, torch, p, seed)
    return _cache[key]


@pytest.mark.parametrize("label", ["k5_N256_l2", "k3_N512_l3"])
def test_small_levels_key_layout(B, oracle, torch_cuda, label):
    """[n][limb][cg][q][c2][row][slot][lane] (col = cg GC + c2; GC = 2 at N = 256, k = 5): level
    v = l - 1 - q of key polynomial (row, col)."""
    S = sm_level_setup(B, oracle, torch_cuda, label, 3, 9900)
    p = S.p
    N, K1, M, P, level = p.N, p.k + 1, p.N // 2, 1024 // p.N, p.level
    GC = 2 if (N == 256 and K1 % 2 == 0) else 1
    assert B.bsk_format(p) == (5, 4, 16)
    got = B.to_host(S.fbsk).view(np.float64).reshape(p.n, 4, K1 // GC, level, GC, K1, M // 64, 64, 2)
    bsk = S.bsk.reshape(p.n, level, K1, K1, N)
    lane = np.arange(64)
    K = (lane[None, :] >> 3) + 8 * (lane[None, :] & 7) + 64 * np.arange(M // 64)[:, None]
    tw = np.exp(1j * np.pi * np.arange(M) / N)
    worst = 0.0
    for i in (0, p.n - 1):
        for li in (0, 3):
            for col in range(K1):
                for q in range(level):
                    for row in (0, K1 - 1):
                        lv = signed_limb(bsk[i, level - 1 - q, row, col], li)
                        ref = np.fft.fft((lv[:M] + 1j * lv[M:]) * tw)[K] / (512.0 * P)
                        gg = got[i, li, col // GC, q, col % GC, row]
                        worst = max(worst, np.max(np.abs(gg[..., 0] + 1j * gg[..., 1] - ref)) / np.max(np.abs(ref)))
    assert worst < 1e-13, worst


@pytest.mark.parametrize("n", [1, 2, 9])
@pytest.mark.parametrize("label", list(SM_LEVEL_ROWS))
def test_small_levels_bit_exact(B, oracle, torch_cuda, label, n):
    """Bit-exact vs the exact oracle over ring prologues / tails and a longer rotation, a ragged batch
    of 5 (four ciphertexts per workgroup), residual under the certified bound."""
    S = sm_level_setup(B, oracle, torch_cuda, label, n, 9910 + n)
    width = 2
    rng = np.random.RandomState(n)
    msgs = rng.randint(0, 4, size=5)
    cts = encrypt(B, S, msgs, width, 85 + n, std=2.0 ** -30)
    acc = lut_acc(B, S, rng.randint(0, 4, size=4), width)
    got, resid = run_gpu(B, S, cts, acc, torch_cuda, resid=True)
    assert np.array_equal(got, run_oracle(oracle, S, cts, acc))
    assert resid < bound(B, oracle, S) < 0.5


@pytest.mark.parametrize("label", ["k5_N256_l2", "k6_N256_l3", "k3_N512_l3"])
def test_small_levels_full_row(B, oracle, torch_cuda, label):
    """Full rows: 256 samples decrypted, 2 bit-exact, residual under the bound."""
    S = sm_level_setup(B, oracle, torch_cuda, label, SM_LEVEL_ROWS[label][4], 9950)
    width = SM_LEVEL_ROWS[label][5]
    rng = np.random.RandomState(11)
    table = rng.randint(0, 1 << width, size=1 << width)
    msgs = rng.randint(0, 1 << width, size=256)
    cts = encrypt(B, S, msgs, width, 95)
    acc = lut_acc(B, S, table, width)
    got, resid = run_gpu(B, S, cts, acc, torch_cuda, resid=True)
    b = bound(B, oracle, S)
    assert resid < b < 0.5, (resid, b)
    dec = B.lwe_decrypt(S.glwe_sk, got, S.p.big_n)
    assert [B.decode(d, width) for d in dec] == [int(table[m]) for m in msgs]
    assert np.array_equal(got[:2], run_oracle(oracle, S, cts[:2], acc))


# ---- N = 512, k = 4 at l >= 6 (pbs512k4_many_kernel: one level at a time, level-major key) -----------
K4_MANY_ROWS = {6: (7, 693), 8: (5, 668), 11: (4, 731), 22: (2, 690), 44: (1, 629)}  # l -> (logB, a row's n)


def test_k4_many_levels_key_layout(B, oracle, torch_cuda):
    """[n][q][limb][col][row][slot][lane]: level v = l - 1 - q of key polynomial (row, col)."""
    level, logB = 6, 7
    S = Setup(B, oracle, torch_cuda, B.PbsParams(n=2, k=4, N=512, level=level, base_log=logB), 9980)
    p = S.p
    assert B.bsk_format(p) == (5, 4, 16)
    got = B.to_host(S.fbsk).view(np.float64).reshape(p.n, level, 4, 5, 5, 4, 64, 2)
    bsk = S.bsk.reshape(p.n, level, 5, 5, 512)
    lane = np.arange(64)
    K = (lane[None, :] >> 3) + 8 * (lane[None, :] & 7) + 64 * np.arange(4)[:, None]
    tw = np.exp(1j * np.pi * np.arange(256) / 512)
    worst = 0.0
    for i in (0, 1):
        for q in (0, 2, level - 1):
            for li in (0, 3):
                for col in (0, 4):
                    for row in (1, 4):
                        lv = signed_limb(bsk[i, level - 1 - q, row, col], li)
                        ref = np.fft.fft((lv[:256] + 1j * lv[256:]) * tw)[K] / 1024.0
                        gg = got[i, q, li, col, row]
                        worst = max(worst, np.max(np.abs(gg[..., 0] + 1j * gg[..., 1] - ref)) / np.max(np.abs(ref)))
    assert worst < 1e-13, worst


@pytest.mark.parametrize("n", [1, 2, 5])
@pytest.mark.parametrize("level", list(K4_MANY_ROWS))
def test_k4_many_levels_bit_exact(B, oracle, torch_cuda, level, n):
    """Bit-exact vs the exact oracle at 6 .. 44 levels (ring prologue and tail, a 5-step rotation), odd
    batch, residual under the certified bound."""
    logB = K4_MANY_ROWS[level][0]
    S = Setup(B, oracle, torch_cuda, B.PbsParams(n=n, k=4, N=512, level=level, base_log=logB), 9990 + level + n)
    width = 2
    rng = np.random.RandomState(level + n)
    msgs = rng.randint(0, 4, size=5)
    cts = encrypt(B, S, msgs, width, 20 + n, std=2.0 ** -30)
    acc = lut_acc(B, S, rng.randint(0, 4, size=4), width)
    got, resid = run_gpu(B, S, cts, acc, torch_cuda, resid=True)
    assert np.array_equal(got, run_oracle(oracle, S, cts, acc))
    assert resid < bound(B, oracle, S) < 0.5


@pytest.mark.parametrize("level", [6, 22])
def test_k4_many_levels_full_row(B, oracle, torch_cuda, level):
    """Full rows (br 6/7 n = 693, br 22/2 n = 690): 128 samples decrypted, 1 bit-exact, residual
    under the bound."""
    logB, n = K4_MANY_ROWS[level]
    S = Setup(B, oracle, torch_cuda, B.PbsParams(n=n, k=4, N=512, level=level, base_log=logB), 9970 + level)
    width = 2
    rng = np.random.RandomState(level)
    table = rng.randint(0, 4, size=4)
    msgs = rng.randint(0, 4, size=128)
    cts = encrypt(B, S, msgs, width, 40 + level)
    acc = lut_acc(B, S, table, width)
    got, resid = run_gpu(B, S, cts, acc, torch_cuda, resid=True)
    b = bound(B, oracle, S)
    assert resid < b < 0.5, (resid, b)
    dec = B.lwe_decrypt(S.glwe_sk, got, S.p.big_n)
    assert [B.decode(d, width) for d in dec] == [int(table[m]) for m in msgs]
    assert np.array_equal(got[:1], run_oracle(oracle, S, cts[:1], acc))
