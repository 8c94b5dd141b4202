"""GPU parity tests of the k = 2, N = 1024, l = 1 / 2 path (the optimizer's 4-bit rows, v0_last_128:
n = 801, logB = 23, bench.py --config opt4; and n = 742-754, l = 2, logB = 15 at log norm2 7-13)
— concrete_amd/csrc/pbs1024k2.hip vs the CPU oracle.

Bit-exact u64 equality with the oracle's pure-integer Karatsuba product on the same keys and
inputs, the measured rounding residual below the GPU scheme's certified bound
(oracle/pyoracle.py:gpu1024k2_error_bound, itself < 1/2), decrypt(out) == LUT[m], the device key
layout against numpy transforms, the digit split at its edges, odd batches (a workgroup holds two
ciphertexts) and the runtime's index-array semantics.
"""
from dataclasses import replace

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


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


@pytest.fixture(scope="module")
def opt4(B, oracle, torch_cuda):
    return Setup(B, oracle, torch_cuda, B.OPTIMIZER_SETS[4], 8000)


@pytest.fixture(scope="module")
def small(B, oracle, torch_cuda):
    return Setup(B, oracle, torch_cuda, replace(B.OPTIMIZER_SETS[4], n=14), 8100)


def encrypt(B, S, msgs, width, seed, std=None):
    std = B.secure_std(1, S.p.n) if std is None else std
    return B.lwe_encrypt(S.lwe_sk, [B.encode(m, width) for m in msgs], S.p.n, std, seed)


def lut_acc(B, S, table, width):
    return B.trivial_glwe(S.p, B.expand_lut(np.array(table, dtype=np.uint64), S.p.N, width))


def run_gpu(B, S, cts, luts, torch, lut_idx=None, in_idx=None, out_idx=None, out_rows=None, resid=False):
    dev = "cuda:0"
    args = {}
    n_s = cts.shape[0] if in_idx is None else len(in_idx)
    for name, a in (("lut_idx", lut_idx), ("in_idx", in_idx), ("out_idx", out_idx)):
        if a is not None:
            args[name] = B.to_device(np.asarray(a, dtype=np.uint64), dev)
    out = torch.zeros(((out_rows or n_s), S.p.lwe_out_size), dtype=torch.int64, device=dev)
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


def signed_limb(x, limb, limbs=4):
    """Balanced signed 16-bit limb of u64 values (the device converter's rule)."""
    rem = x.astype(np.uint64).copy()
    w = 64 // limbs
    val = None
    for _ in range(limb + 1):
        vv = (rem & np.uint64((1 << w) - 1)).astype(np.int64)
        sgn = np.where(vv >= (1 << (w - 1)), vv - (1 << w), vv)
        val = sgn
        rem = (rem - sgn.astype(np.uint64)) >> np.uint64(w)
    return val.astype(np.float64)


def test_key_format(B, small):
    assert B.bsk_format(small.p) == (4, 4, 16)
    assert B.fourier_bsk_bytes(small.p) == small.p.n * 4 * 9 * 512 * 16


def test_fourier_key_layout(B, small, torch_cuda):
    """Device key [n][limb][col][row][slot][lane] == the 16-bit limb of key polynomial (row, col),
    folded (g_t + i g_{t+512}), twisted by zeta^t (zeta = e^{i pi/1024}) and transformed, at
    frequency fft512_freq(lane, slot), divided by 512.  (numpy's FFT is not correctly rounded:
    tolerance 1e-13.)"""
    p = small.p
    got = B.to_host(small.fbsk).view(np.float64).reshape(p.n, 4, 3, 3, 8, 64, 2)
    bsk = small.bsk.reshape(p.n, 1, 3, 3, 1024)
    lane = np.arange(64)
    slot = np.arange(8)
    K = (lane[None, :] >> 3) + 8 * (lane[None, :] & 7) + 64 * slot[:, None]
    tw = np.exp(1j * np.pi * np.arange(512) / 1024.0)
    worst = 0.0
    for i in (0, p.n - 1):
        for li in range(4):
            for col in range(3):
                for row in range(3):
                    lv = signed_limb(bsk[i, 0, row, col], li)
                    ref = np.fft.fft((lv[:512] + 1j * lv[512:]) * tw)[K] / 512.0
                    gg = got[i, li, col, row]
                    worst = max(worst, np.max(np.abs(gg[..., 0] + 1j * gg[..., 1] - ref)) / np.max(np.abs(ref)))
    assert worst < 1e-13, worst


@pytest.mark.parametrize("batch", [1, 2, 5, 8])
def test_bit_exact_small(B, oracle, small, torch_cuda, batch):
    """Odd batches leave the second ciphertext of the last workgroup empty."""
    width = 4
    rng = np.random.RandomState(batch)
    table = rng.randint(0, 16, size=16)
    msgs = rng.randint(0, 16, size=batch)
    cts = encrypt(B, small, msgs, width, 10 + batch, std=2.0 ** -30)
    acc = lut_acc(B, small, table, width)
    got, resid = run_gpu(B, small, cts, acc, torch_cuda, resid=True)
    assert np.array_equal(got, run_oracle(oracle, small, cts, acc))
    assert resid < oracle.gpu1024k2_error_bound(B.to_host(small.fbsk).view(np.float64), small.p.base_log) < 0.5
    dec = B.lwe_decrypt(small.glwe_sk, got, small.p.big_n)
    assert [B.decode(d, width) for d in dec] == [int(table[m]) for m in msgs]


@pytest.mark.parametrize("logB", [8, 16, 17, 24])
def test_other_base_logs(B, oracle, torch_cuda, logB):
    """The digit split d = d_lo + 2^16 d_hi at its edges: d_hi == 0 (logB <= 16), |d_hi| <= 2
    (17) and the largest accepted digit (24, |d_hi| <= 129); bit-exact, residual under the bound."""
    S = Setup(B, oracle, torch_cuda, replace(B.OPTIMIZER_SETS[4], n=10, base_log=logB), 8200 + logB)
    width = 3
    rng = np.random.RandomState(logB)
    msgs = rng.randint(0, 8, size=6)
    cts = encrypt(B, S, msgs, width, 50 + logB, std=2.0 ** -30)
    acc = lut_acc(B, S, rng.randint(0, 8, size=8), width)
    got, resid = run_gpu(B, S, cts, acc, torch_cuda, resid=True)
    assert np.array_equal(got, run_oracle(oracle, S, cts, acc))
    assert resid < oracle.gpu1024k2_error_bound(B.to_host(S.fbsk).view(np.float64), logB) < 0.5


def test_index_arrays_and_mapped_luts(B, oracle, small, torch_cuda):
    width = 3
    nb = 7
    rng = np.random.RandomState(9)
    msgs = rng.randint(0, 8, size=nb)
    cts = encrypt(B, small, msgs, width, 41, std=2.0 ** -30)
    luts = np.stack([lut_acc(B, small, rng.randint(0, 8, size=8), width) for _ in range(nb)])
    lut_idx = rng.permutation(nb).astype(np.uint64)
    in_idx = rng.permutation(nb).astype(np.uint64)
    out_idx = rng.permutation(nb).astype(np.uint64)
    got = run_gpu(B, small, cts, luts, torch_cuda, lut_idx=lut_idx, in_idx=in_idx, out_idx=out_idx)
    ref = run_oracle(oracle, small, cts, luts, lut_idx=lut_idx, in_idx=in_idx, out_idx=out_idx)
    assert np.array_equal(got, ref)


def test_edge_inputs(B, oracle, small, torch_cuda):
    p = small.p
    width = 3
    rng = np.random.RandomState(5)
    cts = encrypt(B, small, rng.randint(0, 8, size=8), width, 31, std=2.0 ** -30)
    cts[0, : p.n // 2] = 0
    cts[1, :] = 0
    cts[2, :] = np.uint64(0xFFFFFFFFFFFFFFFF)
    cts[3, : p.n] = np.uint64(1)
    cts[4, : p.n] = np.uint64((1 << 53) - 1)
    cts[5, p.n] = np.uint64(0xFFFFFFFFFFFFFFFF - 5)
    cts[6, : p.n] = np.uint64(1 << 63)
    cts[7, : p.n] = np.uint64(3 << 52)                  # odd modulus switch
    acc = lut_acc(B, small, [3, 1, 0, 2, 7, 5, 4, 6], width)
    got = run_gpu(B, small, cts, acc, torch_cuda)
    assert np.array_equal(got, run_oracle(oracle, small, cts, acc))


def test_opt4_full_bit_exact_and_bound(B, oracle, opt4, torch_cuda):
    """The full 4-bit row (n = 801): bit-exact vs the exact oracle on 4 samples, the measured
    residual under the certified bound (< 1/2), every sample of a 512-batch decrypts to LUT[m]."""
    width = 4
    rng = np.random.RandomState(3)
    table = rng.randint(0, 16, size=16)
    nb = 512
    msgs = rng.randint(0, 16, size=nb)
    cts = encrypt(B, opt4, msgs, width, 77)
    acc = lut_acc(B, opt4, table, width)
    got, resid = run_gpu(B, opt4, cts, acc, torch_cuda, resid=True)
    bound = oracle.gpu1024k2_error_bound(B.to_host(opt4.fbsk).view(np.float64), opt4.p.base_log)
    assert resid < bound < 0.5, (resid, bound)
    dec = B.lwe_decrypt(opt4.glwe_sk, got, opt4.p.big_n)
    assert [B.decode(d, width) for d in dec] == [int(table[m]) for m in msgs]
    pick = np.array([0, 1, 2, nb - 1])
    assert np.array_equal(got[pick], run_oracle(oracle, opt4, cts[pick], acc))


@pytest.mark.parametrize("level", [1, 2, 3])
@pytest.mark.parametrize("n", [1, 2, 3])
def test_tiny_n(B, oracle, torch_cuda, n, level):
    """Blind rotations of 1-3 steps: the key ring's prologue and tail (the last step issues no
    further groups and waits for fewer in flight) meet within one or two steps."""
    p = replace(B.OPTIMIZER_SETS[4], n=n, level=level, base_log={1: 23, 2: 15, 3: 12}[level])
    S = Setup(B, oracle, torch_cuda, p, 8400 + 10 * level + n)
    width = 3
    rng = np.random.RandomState(n)
    msgs = rng.randint(0, 8, size=5)
    cts = encrypt(B, S, msgs, width, 60 + n, std=2.0 ** -30)
    acc = lut_acc(B, S, rng.randint(0, 8, size=8), width)
    got = run_gpu(B, S, cts, acc, torch_cuda)
    assert np.array_equal(got, run_oracle(oracle, S, cts, acc))


# ---- l = 2 (the rows at log norm2 7-13: br 2/15, n = 742-754) ------------------------------
def test_two_level_key_layout(B, oracle, torch_cuda):
    """Device key [n][limb][col][q][row][slot][lane]: level v = 1 - q of key polynomial (row, col)."""
    S = Setup(B, oracle, torch_cuda, replace(B.OPTIMIZER_SETS[4], n=4, level=2, base_log=15), 8500)
    p = S.p
    assert B.bsk_format(p) == (4, 4, 16)
    assert B.fourier_bsk_bytes(p) == p.n * 2 * 4 * 9 * 512 * 16
    got = B.to_host(S.fbsk).view(np.float64).reshape(p.n, 4, 3, 2, 3, 8, 64, 2)
    bsk = S.bsk.reshape(p.n, 2, 3, 3, 1024)
    lane = np.arange(64)
    slot = np.arange(8)
    K = (lane[None, :] >> 3) + 8 * (lane[None, :] & 7) + 64 * slot[:, None]
    tw = np.exp(1j * np.pi * np.arange(512) / 1024.0)
    worst = 0.0
    for i in (0, p.n - 1):
        for li in range(4):
            for col in range(3):
                for q in range(2):
                    for row in range(3):
                        lv = signed_limb(bsk[i, 1 - q, row, col], li)
                        ref = np.fft.fft((lv[:512] + 1j * lv[512:]) * tw)[K] / 512.0
                        gg = got[i, li, col, q, row]
                        worst = max(worst, np.max(np.abs(gg[..., 0] + 1j * gg[..., 1] - ref)) / np.max(np.abs(ref)))
    assert worst < 1e-13, worst


@pytest.mark.parametrize("logB,batch", [(15, 5), (8, 3), (1, 2)])
def test_two_levels_bit_exact(B, oracle, torch_cuda, logB, batch):
    S = Setup(B, oracle, torch_cuda, replace(B.OPTIMIZER_SETS[4], n=10, level=2, base_log=logB), 8600 + logB)
    width = 3
    rng = np.random.RandomState(logB)
    msgs = rng.randint(0, 8, size=batch)
    cts = encrypt(B, S, msgs, width, 70 + logB, std=2.0 ** -30)
    acc = lut_acc(B, S, rng.randint(0, 8, size=8), width)
    got, resid = run_gpu(B, S, cts, acc, torch_cuda, resid=True)
    assert np.array_equal(got, run_oracle(oracle, S, cts, acc))
    assert resid < oracle.gpu1024k2_error_bound(B.to_host(S.fbsk).view(np.float64), logB, 2) < 0.5


def test_two_levels_full_row(B, oracle, torch_cuda):
    """v0_last_128's 4-bit row at log norm2 7 (k = 2, N = 1024, n = 742, br 2/15): 256 samples
    decrypted, 2 bit-exact vs the exact oracle, residual under the certified bound."""
    S = Setup(B, oracle, torch_cuda, B.PbsParams(n=742, k=2, N=1024, level=2, base_log=15, ks_level=3,
                                                ks_base_log=4), 8700)
    width = 4
    rng = np.random.RandomState(7)
    table = rng.randint(0, 16, size=16)
    msgs = rng.randint(0, 16, size=256)
    cts = encrypt(B, S, msgs, width, 99)
    acc = lut_acc(B, S, table, width)
    got, resid = run_gpu(B, S, cts, acc, torch_cuda, resid=True)
    bound = oracle.gpu1024k2_error_bound(B.to_host(S.fbsk).view(np.float64), 15, 2)
    assert resid < bound < 0.5, (resid, bound)
    dec = B.lwe_decrypt(S.glwe_sk, got, S.p.big_n)
    assert [B.decode(d, width) for d in dec] == [int(table[m]) for m in msgs]
    assert np.array_equal(got[:2], run_oracle(oracle, S, cts[:2], acc))


# ---- l = 3 (the rows at log norm2 14-17: br 3/12, n = 742-769) -------------------------------------
@pytest.mark.parametrize("logB,batch", [(12, 5), (5, 2)])
def test_three_levels_bit_exact(B, oracle, torch_cuda, logB, batch):
    S = Setup(B, oracle, torch_cuda, replace(B.OPTIMIZER_SETS[4], n=10, level=3, base_log=logB), 8800 + logB)
    width = 3
    rng = np.random.RandomState(logB)
    msgs = rng.randint(0, 8, size=batch)
    cts = encrypt(B, S, msgs, width, 75 + logB, std=2.0 ** -30)
    acc = lut_acc(B, S, rng.randint(0, 8, size=8), width)
    got, resid = run_gpu(B, S, cts, acc, torch_cuda, resid=True)
    assert np.array_equal(got, run_oracle(oracle, S, cts, acc))
    assert resid < oracle.gpu1024k2_error_bound(B.to_host(S.fbsk).view(np.float64), logB, 3) < 0.5


def test_three_levels_full_row(B, oracle, torch_cuda):
    """The 4-bit row at log norm2 14 (n = 742, br 3/12): 256 samples decrypted, 2 bit-exact, residual
    under the bound."""
    S = Setup(B, oracle, torch_cuda, B.PbsParams(n=742, k=2, N=1024, level=3, base_log=12, ks_level=3,
                                                ks_base_log=4), 8900)
    width = 4
    rng = np.random.RandomState(14)
    table = rng.randint(0, 16, size=16)
    msgs = rng.randint(0, 16, size=256)
    cts = encrypt(B, S, msgs, width, 98)
    acc = lut_acc(B, S, table, width)
    got, resid = run_gpu(B, S, cts, acc, torch_cuda, resid=True)
    bound = oracle.gpu1024k2_error_bound(B.to_host(S.fbsk).view(np.float64), 12, 3)
    assert resid < bound < 0.5, (resid, bound)
    dec = B.lwe_decrypt(S.glwe_sk, got, S.p.big_n)
    assert [B.decode(d, width) for d in dec] == [int(table[m]) for m in msgs]
    assert np.array_equal(got[:2], run_oracle(oracle, S, cts[:2], acc))


# ---- l >= 4 (pbs1024k2_many_kernel: one level at a time, level-major key; br 4/9 .. 44/1) ---------
K2_MANY_ROWS = {4: (9, 731), 5: (8, 722), 8: (5, 743), 15: (3, 754), 44: (1, 727)}  # l -> (logB, a row's n)


def test_many_levels_key_layout(B, oracle, torch_cuda):
    """[n][q][limb][col][row][slot][lane]: level v = l - 1 - q of key polynomial (row, col)."""
    level, logB = 4, 9
    S = Setup(B, oracle, torch_cuda, B.PbsParams(n=2, k=2, N=1024, level=level, base_log=logB), 8950)
    p = S.p
    assert B.bsk_format(p) == (4, 4, 16)
    got = B.to_host(S.fbsk).view(np.float64).reshape(p.n, level, 4, 3, 3, 8, 64, 2)
    bsk = S.bsk.reshape(p.n, level, 3, 3, 1024)
    lane = np.arange(64)
    K = (lane[None, :] >> 3) + 8 * (lane[None, :] & 7) + 64 * np.arange(8)[:, None]
    tw = np.exp(1j * np.pi * np.arange(512) / 1024.0)
    worst = 0.0
    for i in (0, 1):
        for q in range(level):
            for li in (0, 3):
                for col in (0, 2):
                    for row in (0, 2):
                        lv = signed_limb(bsk[i, level - 1 - q, row, col], li)
                        ref = np.fft.fft((lv[:512] + 1j * lv[512:]) * tw)[K] / 512.0
                        gg = got[i, q, li, col, row]
                        worst = max(worst, np.max(np.abs(gg[..., 0] + 1j * gg[..., 1] - ref)) / np.max(np.abs(ref)))
    assert worst < 1e-13, worst


@pytest.mark.parametrize("n", [1, 2, 5])
@pytest.mark.parametrize("level", list(K2_MANY_ROWS))
def test_many_levels_bit_exact(B, oracle, torch_cuda, level, n):
    logB = K2_MANY_ROWS[level][0]
    S = Setup(B, oracle, torch_cuda, B.PbsParams(n=n, k=2, N=1024, level=level, base_log=logB), 8960 + level + n)
    width = 3
    rng = np.random.RandomState(level + n)
    msgs = rng.randint(0, 8, size=5)
    cts = encrypt(B, S, msgs, width, 30 + n, std=2.0 ** -30)
    acc = lut_acc(B, S, rng.randint(0, 8, size=8), width)
    got, resid = run_gpu(B, S, cts, acc, torch_cuda, resid=True)
    assert np.array_equal(got, run_oracle(oracle, S, cts, acc))
    assert resid < oracle.gpu1024k2_error_bound(B.to_host(S.fbsk).view(np.float64), logB, level) < 0.5


@pytest.mark.parametrize("level", [4, 15])
def test_many_levels_full_row(B, oracle, torch_cuda, level):
    """The 4-bit rows at br 4/9 (n = 731) and 15/3 (n = 754): 128 samples decrypted, 1 bit-exact,
    residual under the bound."""
    logB, n = K2_MANY_ROWS[level]
    S = Setup(B, oracle, torch_cuda, B.PbsParams(n=n, k=2, N=1024, level=level, base_log=logB), 8970 + level)
    width = 4
    rng = np.random.RandomState(level)
    table = rng.randint(0, 16, size=16)
    msgs = rng.randint(0, 16, size=128)
    cts = encrypt(B, S, msgs, width, 50 + level)
    acc = lut_acc(B, S, table, width)
    got, resid = run_gpu(B, S, cts, acc, torch_cuda, resid=True)
    bound = oracle.gpu1024k2_error_bound(B.to_host(S.fbsk).view(np.float64), logB, level)
    assert resid < bound < 0.5, (resid, bound)
    dec = B.lwe_decrypt(S.glwe_sk, got, S.p.big_n)
    assert [B.decode(d, width) for d in dec] == [int(table[m]) for m in msgs]
    assert np.array_equal(got[:1], run_oracle(oracle, S, cts[:1], acc))
