"""GPU parity tests of the N = 2048 path (BASELINE.json configs[3], cfg4: n = 742, l = 1,
logB = 23) — concrete_amd/csrc/pbs2048.hip vs the CPU oracle.

Bit-exact u64 equality with the oracle's exact product (its certified 8-limb FFT path), the
GPU scheme's own certified rounding bound checked against the measured residual, decrypt-level
checks on the reference generators' cleartext vectors (p <= 5: cfg4's PBS output noise is
~2e-5), and the runtime's index-array semantics.
"""
import json
import math
import os
from dataclasses import replace

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "reference_lut_fixtures.json")


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
    def __init__(self, B, oracle, torch, p, seed, oracle_key=True):
        self.p = p
        self.op = oracle.Params(n=p.n, k=p.k, N=p.N, l=p.level, logB=p.base_log, ks_l=p.ks_level,
                                ks_logB=p.ks_base_log, limbs=oracle.limbs_for(p.N))
        self.lwe_sk = B.binary_key(p.n, seed)
        self.glwe_sk = B.binary_key(p.big_n, seed + 1)
        self.bsk = B.bsk_generate(p, self.lwe_sk, self.glwe_sk, seed + 2)
        self.fbsk_cpu = oracle.bsk_to_fourier(self.op, self.bsk) if oracle_key else None
        self.fbsk = B.convert_bsk(p, self.bsk, "cuda:0")
        torch.cuda.synchronize()


@pytest.fixture(scope="module")
def cfg4(B, oracle, torch_cuda):
    return Setup(B, oracle, torch_cuda, B.CFG4, 4000)


@pytest.fixture(scope="module")
def small4(B, oracle, torch_cuda):
    return Setup(B, oracle, torch_cuda, replace(B.CFG4, n=20), 5000)


def encrypt(B, S, msgs, width, seed, std=None):
    std = B.secure_std(1, S.p.n) if std is None else std
    return B.lwe_encrypt(S.lwe_sk, [B.encode(m, width) for m in msgs], S.p.n, std, seed)


def lut_acc(B, S, table, width, signed=False):
    return B.trivial_glwe(S.p, B.expand_lut(np.array(table, dtype=np.uint64), S.p.N, width, signed))


def run_gpu(B, S, cts, luts, torch, lut_idx=None, in_idx=None, out_idx=None, out_rows=None, resid=False):
    dev = "cuda:0"
    d_in = B.to_device(cts, dev)
    d_luts = B.to_device(np.atleast_2d(luts), dev)
    args = {}
    n_s = cts.shape[0] if in_idx is None else len(in_idx)
    for name, a in (("lut_idx", lut_idx), ("in_idx", in_idx), ("out_idx", out_idx)):
        if a is not None:
            args[name] = B.to_device(np.asarray(a, dtype=np.uint64), dev)
    out = torch.zeros(((out_rows or n_s), S.p.lwe_out_size), dtype=torch.int64, device=dev)
    r = torch.zeros(1, dtype=torch.int64, device=dev) if resid else None
    B.pbs(S.p, S.fbsk, d_in, d_luts, out=out, num_samples=n_s, resid=r, **args)
    torch.cuda.synchronize()
    res = B.to_host(out)
    if resid:
        return res, float(np.array([r.item()], dtype=np.int64).view(np.float64)[0])
    return res


def run_oracle(oracle, S, cts, luts, lut_idx=None, in_idx=None, out_idx=None):
    out, _ = oracle.pbs_batch(S.op, cts, np.atleast_2d(luts), fbsk=S.fbsk_cpu, lut_idx=lut_idx, in_idx=in_idx,
                              out_idx=out_idx)
    return out


def signed_limb(x, limb, limbs=4):
    """Balanced signed limb of u64 values (16-bit limbs; same rule as the device converter)."""
    rem = x.astype(np.uint64).copy()
    w = 64 // limbs
    val = None
    for _ in range(limb + 1):
        vv = (rem & np.uint64((1 << w) - 1)).astype(np.int64)
        sgn = np.where(vv >= (1 << (w - 1)), vv - (1 << w), vv)
        val = sgn
        rem = (rem - sgn.astype(np.uint64)) >> np.uint64(w)
    return val.astype(np.float64)


def test_fourier_key_2048_layout(B, small4, torch_cuda):
    """Device key [n][limb][col][row][+-][slot][lane] == the N = 2048 key polynomial's 16-bit limb
    evaluated at +-s_k, s_k = exp(i pi (1 - 4k) / 2048), k = fft512_freq(lane, slot), divided by
    1024: (G_e(alpha_k) +- s_k G_o(alpha_k)) / 1024 with G_e / G_o the numpy transforms of the parity
    halves (folded, twisted by zeta^t, zeta = e^{i pi/1024}).  (numpy's FFT is not correctly
    rounded: tolerance 1e-13.)"""
    p = small4.p
    got = B.to_host(small4.fbsk).view(np.float64).reshape(p.n, 4, 2, 2, 2, 8, 64, 2)
    bsk = small4.bsk.reshape(p.n, 1, 2, 2, 2048)
    lane = np.arange(64)
    slot = np.arange(8)
    K = (lane[None, :] >> 3) + 8 * (lane[None, :] & 7) + 64 * slot[:, None]
    t = np.arange(512)
    tw = np.exp(1j * np.pi * t / 1024.0)
    sroot = np.exp(1j * np.pi * (1.0 - 4.0 * K) / 2048.0)
    worst = 0.0
    for i in (0, p.n - 1):
        for li in range(4):
            for col in range(2):
                for row in range(2):
                    spec = []
                    for par in range(2):
                        lv = signed_limb(bsk[i, 0, row, col, par::2], li)
                        z = (lv[:512] + 1j * lv[512:]) * tw
                        spec.append(np.fft.fft(z)[K])
                    for pm, sign in ((0, 1.0), (1, -1.0)):
                        ref = (spec[0] + sign * sroot * spec[1]) / 1024.0
                        gg = got[i, li, col, row, pm]
                        err = np.max(np.abs(gg[..., 0] + 1j * gg[..., 1] - ref))
                        worst = max(worst, err / np.max(np.abs(ref)))
    assert worst < 1e-13, worst


@pytest.mark.parametrize("batch", [1, 3, 8])
def test_pbs2048_bit_exact_small(B, oracle, small4, torch_cuda, batch):
    width = 4
    rng = np.random.RandomState(batch)
    table = rng.randint(0, 16, size=16)
    msgs = rng.randint(0, 16, size=batch)
    cts = encrypt(B, small4, msgs, width, 10 + batch, std=2.0 ** -30)
    acc = lut_acc(B, small4, table, width)
    got = run_gpu(B, small4, cts, acc, torch_cuda)
    ref = run_oracle(oracle, small4, cts, acc)
    assert np.array_equal(got, ref)
    dec = B.lwe_decrypt(small4.glwe_sk, got, small4.p.big_n)
    assert [B.decode(d, width) for d in dec] == [int(table[m]) for m in msgs]


@pytest.mark.parametrize("logB", [8, 16, 17, 24])
def test_pbs2048_other_base_logs(B, oracle, torch_cuda, logB):
    """The digit split d = d_lo + 2^16 d_hi at its edges: d_hi == 0 (logB <= 16), |d_hi| <= 2
    (17) and the largest accepted digit (24, |d_hi| <= 129); bit-exact, residual under the bound."""
    S = Setup(B, oracle, torch_cuda, replace(B.CFG4, n=12, base_log=logB), 6000 + logB)
    width = 3
    rng = np.random.RandomState(logB)
    msgs = rng.randint(0, 8, size=6)
    cts = encrypt(B, S, msgs, width, 50 + logB, std=2.0 ** -30)
    acc = lut_acc(B, S, rng.randint(0, 8, size=8), width)
    got, resid = run_gpu(B, S, cts, acc, torch_cuda, resid=True)
    assert np.array_equal(got, run_oracle(oracle, S, cts, acc))
    assert resid < oracle.gpu2048_error_bound(B.to_host(S.fbsk).view(np.float64), logB) < 0.5


def test_pbs2048_cfg4_bit_exact_and_bound(B, oracle, cfg4, torch_cuda):
    """Full cfg4 (n = 742): bit-exact vs the oracle; the measured rounding residual stays below
    the GPU scheme's certified bound, itself < 1/2."""
    width = 5
    rng = np.random.RandomState(3)
    table = rng.randint(0, 32, size=32)
    msgs = rng.randint(0, 32, size=16)
    cts = encrypt(B, cfg4, msgs, width, 77)
    acc = lut_acc(B, cfg4, table, width)
    got, resid = run_gpu(B, cfg4, cts, acc, torch_cuda, resid=True)
    ref = run_oracle(oracle, cfg4, cts, acc)
    assert np.array_equal(got, ref)
    bound = oracle.gpu2048_error_bound(B.to_host(cfg4.fbsk).view(np.float64), cfg4.p.base_log)
    assert resid < bound < 0.5, (resid, bound)
    dec = B.lwe_decrypt(cfg4.glwe_sk, got, cfg4.p.big_n)
    assert [B.decode(d, width) for d in dec] == [int(table[m]) for m in msgs]


def test_pbs2048_edge_inputs(B, oracle, small4, torch_cuda):
    p = small4.p
    width = 3
    rng = np.random.RandomState(5)
    cts = encrypt(B, small4, rng.randint(0, 8, size=8), width, 31, std=2.0 ** -30)
    cts[0, : p.n // 2] = 0
    cts[1, :] = 0
    cts[2, :] = np.uint64(0xFFFFFFFFFFFFFFFF)
    cts[3, : p.n] = np.uint64(1)
    cts[4, : p.n] = np.uint64((1 << 52) - 1)
    cts[5, p.n] = np.uint64(0xFFFFFFFFFFFFFFFF - 5)
    cts[6, : p.n] = np.uint64(1 << 63)
    cts[7, : p.n] = np.uint64(3 << 51)                  # odd modulus switch (parities swap)
    acc = lut_acc(B, small4, [3, 1, 0, 2, 7, 5, 4, 6], width)
    got = run_gpu(B, small4, cts, acc, torch_cuda)
    ref = run_oracle(oracle, small4, cts, acc)
    assert np.array_equal(got, ref)


def test_pbs2048_index_arrays_and_mapped_luts(B, oracle, small4, torch_cuda):
    width = 3
    nb = 7
    rng = np.random.RandomState(9)
    msgs = rng.randint(0, 8, size=nb)
    cts = encrypt(B, small4, msgs, width, 41, std=2.0 ** -30)
    tables = [rng.randint(0, 8, size=8) for _ in range(nb)]
    luts = np.stack([lut_acc(B, small4, t, width) for t in tables])
    lut_idx = rng.permutation(nb).astype(np.uint64)
    in_idx = rng.permutation(nb).astype(np.uint64)
    out_idx = rng.permutation(nb).astype(np.uint64)
    got = run_gpu(B, small4, cts, luts, torch_cuda, lut_idx=lut_idx, in_idx=in_idx, out_idx=out_idx)
    ref = run_oracle(oracle, small4, cts, luts, lut_idx=lut_idx, in_idx=in_idx, out_idx=out_idx)
    assert np.array_equal(got, ref)


def test_pbs2048_reference_fixtures_decrypt(B, cfg4, torch_cuda):
    """Reference generators' cleartext vectors up to p = 5 (signed and unsigned variants)."""
    fx = json.load(open(GOLDEN))
    cases = [c for c in fx["apply_lookup_table"] + fx["linalg_apply_lookup_table"]
             if len(c["lut"]) <= 32 and not c["description"].endswith("_2layer")]
    assert cases
    for ci, c in enumerate(cases):
        width = int(math.log2(len(c["lut"])))
        xs = [int(x) & ((1 << 64) - 1) for x in c["input"]]
        cts = encrypt(B, cfg4, xs, width, 700 + ci)
        if c["input_signed"]:
            cts[:, cfg4.p.n] += B.encode(1 << (width - 1), width)
        table = np.array(c["lut"], dtype=np.int64).view(np.uint64)
        acc = lut_acc(B, cfg4, table, width, c["input_signed"])
        got = run_gpu(B, cfg4, cts, acc, torch_cuda)
        dec = B.lwe_decrypt(cfg4.glwe_sk, got, cfg4.p.big_n)
        assert [B.decode(d, width, c["output_signed"]) for d in dec] == c["expected"], c["description"]


def test_pbs2048_batch_properties(B, oracle, cfg4, torch_cuda):
    """cfg4 at B = 1024 (configs[3]): every sample decrypts to LUT[m]; 8 random rows bit-exact."""
    width = 5
    nb = 1024
    rng = np.random.RandomState(12)
    table = rng.randint(0, 32, size=32)
    msgs = rng.randint(0, 32, size=nb)
    cts = encrypt(B, cfg4, msgs, width, 4321)
    acc = lut_acc(B, cfg4, table, width)
    got = run_gpu(B, cfg4, cts, acc, torch_cuda)
    dec = B.lwe_decrypt(cfg4.glwe_sk, got, cfg4.p.big_n)
    assert all(B.decode(d, width) == table[m] for d, m in zip(dec, msgs))
    pick = rng.choice(nb, size=8, replace=False)
    ref = run_oracle(oracle, cfg4, cts[pick], acc)
    assert np.array_equal(got[pick], ref)


# ---- l = 2 .. 4 (whole digits; the optimizer's 5-bit rows at br 2/15, 3/11, 4/9) -----------------
LEVEL_ROWS = {2: (15, 783), 3: (11, 784), 4: (9, 761)}  # level -> (logB, an optimizer row's n)


def test_fourier_key_2048_levels_layout(B, torch_cuda, oracle):
    """[n][limb][col][q][row][+-][slot][lane]: level v = l - 1 - q of key polynomial (row, col)."""
    level = 3
    S = Setup(B, oracle, torch_cuda, replace(B.CFG4, n=2, level=level, base_log=11), 6500)
    p = S.p
    assert B.bsk_format(p) == (2, 4, 16)
    assert B.fourier_bsk_bytes(p) == p.n * level * 4 * 4 * 2 * 512 * 16
    got = B.to_host(S.fbsk).view(np.float64).reshape(p.n, 4, 2, level, 2, 2, 8, 64, 2)
    bsk = S.bsk.reshape(p.n, level, 2, 2, 2048)
    lane = np.arange(64)
    K = (lane[None, :] >> 3) + 8 * (lane[None, :] & 7) + 64 * np.arange(8)[:, None]
    tw = np.exp(1j * np.pi * np.arange(512) / 1024.0)
    sroot = np.exp(1j * np.pi * (1.0 - 4.0 * K) / 2048.0)
    worst = 0.0
    for i in (0, p.n - 1):
        for li in (0, 3):
            for col in range(2):
                for q in range(level):
                    for row in range(2):
                        spec = []
                        for par in range(2):
                            lv = signed_limb(bsk[i, level - 1 - q, row, col, par::2], li)
                            spec.append(np.fft.fft((lv[:512] + 1j * lv[512:]) * tw)[K])
                        for pm, sign in ((0, 1.0), (1, -1.0)):
                            ref = (spec[0] + sign * sroot * spec[1]) / 1024.0
                            gg = got[i, li, col, q, row, pm]
                            worst = max(worst, np.max(np.abs(gg[..., 0] + 1j * gg[..., 1] - ref)) / np.max(np.abs(ref)))
    assert worst < 1e-13, worst


@pytest.mark.parametrize("n", [1, 2, 9])
@pytest.mark.parametrize("level", [2, 3, 4])
def test_pbs2048_levels_bit_exact(B, oracle, torch_cuda, level, n):
    """Bit-exact vs the exact oracle at each level count over ring prologues / tails (n = 1, 2) and a
    longer rotation, an odd batch, residual under the certified bound."""
    logB = LEVEL_ROWS[level][0]
    S = Setup(B, oracle, torch_cuda, replace(B.CFG4, n=n, level=level, base_log=logB), 6600 + 10 * level + n)
    width = 3
    rng = np.random.RandomState(level * 10 + n)
    msgs = rng.randint(0, 8, size=5)
    cts = encrypt(B, S, msgs, width, 70 + n, std=2.0 ** -30)
    acc = lut_acc(B, S, rng.randint(0, 8, size=8), width)
    got, resid = run_gpu(B, S, cts, acc, torch_cuda, resid=True)
    assert np.array_equal(got, run_oracle(oracle, S, cts, acc))
    assert resid < oracle.gpu2048_error_bound(B.to_host(S.fbsk).view(np.float64), logB, level) < 0.5


@pytest.mark.parametrize("level", [2, 4])
def test_pbs2048_levels_full_row(B, oracle, torch_cuda, level):
    """The 5-bit rows at br 2/15 (n = 783) and 4/9 (n = 761): 256 samples decrypted, 2 bit-exact,
    residual under the bound."""
    logB, n = LEVEL_ROWS[level]
    S = Setup(B, oracle, torch_cuda, replace(B.CFG4, n=n, level=level, base_log=logB), 6700 + level)
    width = 5
    rng = np.random.RandomState(level)
    table = rng.randint(0, 32, size=32)
    msgs = rng.randint(0, 32, size=256)
    cts = encrypt(B, S, msgs, width, 90 + level)
    acc = lut_acc(B, S, table, width)
    got, resid = run_gpu(B, S, cts, acc, torch_cuda, resid=True)
    bound = oracle.gpu2048_error_bound(B.to_host(S.fbsk).view(np.float64), logB, level)
    assert resid < bound < 0.5, (resid, bound)
    dec = B.lwe_decrypt(S.glwe_sk, got, S.p.big_n)
    assert [B.decode(d, width) for d in dec] == [int(table[m]) for m in msgs]
    assert np.array_equal(got[:2], run_oracle(oracle, S, cts[:2], acc))
