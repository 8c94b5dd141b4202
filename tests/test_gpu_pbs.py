"""GPU parity tests: libconcrete_hip.so (HIP kernels on cuda:0) vs the CPU oracle.

Bit-exact u64 equality of every output word (integer/torus work: no tolerance), plus
decrypt-level checks against the reference generators' cleartext vectors and
size-independent properties at the metric's batch size.
"""
import ctypes as C
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


def oparams(oracle, p):
    return oracle.Params(n=p.n, k=p.k, N=p.N, l=p.level, logB=p.base_log, ks_l=p.ks_level, ks_logB=p.ks_base_log)


class Setup:
    def __init__(self, B, oracle, torch, p, seed):
        self.p = p
        self.op = oparams(oracle, p)
        self.lwe_sk = B.binary_key(p.n, seed)
        self.glwe_sk = B.binary_key(p.big_n, seed + 1)
        self.bsk = B.bsk_generate(p, self.lwe_sk, self.glwe_sk, seed + 2)
        self.fbsk_cpu = oracle.bsk_to_fourier(self.op, self.bsk)
        self.fbsk = B.convert_bsk(p, self.bsk, "cuda:0")
        torch.cuda.synchronize()


@pytest.fixture(scope="module")
def cfg2(B, oracle, torch_cuda):
    return Setup(B, oracle, torch_cuda, B.CFG2, 1000)


@pytest.fixture(scope="module")
def small(B, oracle, torch_cuda):
    return Setup(B, oracle, torch_cuda, replace(B.CFG2, n=24), 2000)


def encrypt(B, S, msgs, width, seed, std=None):
    std = B.secure_std(1, S.p.n) if std is None else std
    return B.lwe_encrypt(S.lwe_sk, [B.encode(m, width) for m in msgs], S.p.n, std, seed)


def lut_acc(B, S, table, width):
    return B.trivial_glwe(S.p, B.expand_lut(np.array(table, dtype=np.uint64), S.p.N, width))


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
    out, resid = oracle.pbs_batch(S.op, cts, np.atleast_2d(luts), fbsk=S.fbsk_cpu, lut_idx=lut_idx, in_idx=in_idx,
                                  out_idx=out_idx)
    return out


def test_fourier_key_matches_oracle_transform(B, small, torch_cuda):
    """Device conversion (double-double FFT) == oracle extended-precision transform, reordered
    into the kernel's layout [n][limb][co][ro][q][slot][lane]: slots 0..3 of group (limb, co,
    ro) hold column co / row ro, slots 4..7 column 1 - co / row 1 - ro; both transforms are
    within ~1 ulp of the exact spectrum."""
    p = small.p
    L = p.level
    g = B.to_host(small.fbsk).view(np.float64).reshape(p.n, 3, 2, 2, L, 8, 64, 2)
    o = small.fbsk_cpu.reshape(p.n, L, p.k + 1, p.k + 1, 3, 2, 512)
    lane = np.arange(64)
    slot = np.arange(8)
    K = (lane[None, :] >> 3) + 8 * (lane[None, :] & 7) + 64 * slot[:, None]  # (8, 64)
    maxrel = 0.0
    for v in range(L):
        q = L - 1 - v
        for li in range(3):
            for co in range(2):
                for ro in range(2):
                    for s0, (row, col) in ((slice(0, 4), (ro, co)), (slice(4, 8), (1 - ro, 1 - co))):
                        ref_re = o[:, v, row, col, li, 0][:, K[s0]]
                        ref_im = o[:, v, row, col, li, 1][:, K[s0]]
                        got = g[:, li, co, ro, q, s0]
                        scale = np.max(np.abs(o[:, v, row, col, li]))
                        err = max(np.max(np.abs(got[..., 0] - ref_re)), np.max(np.abs(got[..., 1] - ref_im)))
                        maxrel = max(maxrel, err / scale)
    assert maxrel < 4e-16, maxrel


@pytest.mark.parametrize("batch", [1, 3, 4, 5, 64])
def test_pbs_bit_exact_small(B, oracle, small, torch_cuda, batch):
    width = 3
    rng = np.random.RandomState(batch)
    table = rng.randint(0, 8, size=8)
    msgs = rng.randint(0, 8, size=batch)
    cts = encrypt(B, small, msgs, width, 10 + batch, std=2.0 ** -25)
    acc = lut_acc(B, small, table, width)
    got = run_gpu(B, small, cts, acc, torch_cuda)
    ref = run_oracle(oracle, small, cts, acc)
    assert np.array_equal(got, ref)
    dec = B.lwe_decrypt(small.glwe_sk, got, small.p.big_n)
    assert [B.decode(d, width) for d in dec] == [int(table[m]) for m in msgs]


def test_pbs_bit_exact_cfg2(B, oracle, cfg2, torch_cuda):
    width = 3
    rng = np.random.RandomState(7)
    table = rng.randint(0, 8, size=8)
    msgs = rng.randint(0, 8, size=64)
    cts = encrypt(B, cfg2, msgs, width, 77)
    acc = lut_acc(B, cfg2, table, width)
    got, resid = run_gpu(B, cfg2, cts, acc, torch_cuda, resid=True)
    ref = run_oracle(oracle, cfg2, cts, acc)
    assert np.array_equal(got, ref)
    bound = oracle.fft_error_bound(cfg2.op, cfg2.fbsk_cpu)
    assert resid < bound < 0.5, (resid, bound)
    dec = B.lwe_decrypt(cfg2.glwe_sk, got, cfg2.p.big_n)
    assert [B.decode(d, width) for d in dec] == [int(table[m]) for m in msgs]


@pytest.mark.parametrize("level,base_log", [(1, 11), (1, 5), (2, 10), (2, 6), (3, 9), (3, 3)])
def test_pbs_bit_exact_other_decompositions(B, oracle, torch_cuda, level, base_log):
    """The L = 1 / 2 / 3 kernel instantiations across the exact range of the gate
    ((k+1) l 2^logB <= 4096, pbs.hpp pbs1024_exact), each against the oracle bit for bit."""
    p = replace(B.CFG2, n=16, level=level, base_log=base_log)
    assert B.pbs_supported(p)
    S = Setup(B, oracle, torch_cuda, p, 3000 + 10 * level + base_log)
    width = 2
    rng = np.random.RandomState(base_log)
    table = rng.randint(0, 4, size=4)
    msgs = rng.randint(0, 4, size=40)
    cts = encrypt(B, S, msgs, width, 41, std=2.0 ** -25)
    acc = lut_acc(B, S, table, width)
    got, resid = run_gpu(B, S, cts, acc, torch_cuda, resid=True)
    assert np.array_equal(got, run_oracle(oracle, S, cts, acc))
    bound = oracle.fft_error_bound(S.op, S.fbsk_cpu)
    assert resid < bound < 0.5, (resid, bound)
    if level * base_log >= 15:  # coarser decompositions do not decrypt (approximation noise)
        dec = B.lwe_decrypt(S.glwe_sk, got, p.big_n)
        assert [B.decode(d, width) for d in dec] == [int(table[m]) for m in msgs]


def test_pbs_edge_inputs(B, oracle, small, torch_cuda):
    """Zero mask elements (tfhe skip rule), mask elements whose modulus switch is 0 or 2N-1,
    body near 2^64 (modulus switch wraps to 2N), all-zero and all-ones ciphertexts."""
    p = small.p
    width = 2
    rng = np.random.RandomState(5)
    cts = encrypt(B, small, rng.randint(0, 4, size=8), width, 31, std=2.0 ** -25)
    cts[0, : p.n // 2] = 0
    cts[1, :] = 0
    cts[2, :] = np.uint64(0xFFFFFFFFFFFFFFFF)
    cts[3, : p.n] = np.uint64(1)                         # ms(1) == 0 but a_i != 0
    cts[4, : p.n] = np.uint64((1 << 53) - 1)             # just below a modswitch rounding boundary
    cts[5, p.n] = np.uint64(0xFFFFFFFFFFFFFFFF - 5)      # body rounds up to 2N
    cts[6, : p.n] = np.uint64(1 << 63)                   # ms = N (negation)
    acc = lut_acc(B, small, [3, 1, 0, 2], width)
    got = run_gpu(B, small, cts, acc, torch_cuda)
    ref = run_oracle(oracle, small, cts, acc)
    assert np.array_equal(got, ref)


def test_pbs_index_arrays_and_mapped_luts(B, oracle, small, torch_cuda):
    """Runtime index-array semantics (GPUDFG.cpp:1149-1205): permuted inputs/outputs and one
    LUT per sample (memref_batched_mapped_bootstrap_lwe_cuda_u64, wrappers.cpp:317-325)."""
    width = 3
    nb = 12
    rng = np.random.RandomState(9)
    msgs = rng.randint(0, 8, size=nb)
    cts = encrypt(B, small, msgs, width, 41, std=2.0 ** -25)
    tables = [rng.randint(0, 8, size=8) for _ in range(nb)]
    luts = np.stack([lut_acc(B, small, t, width) for t in tables])
    lut_idx = rng.permutation(nb).astype(np.uint64)
    in_idx = rng.permutation(nb).astype(np.uint64)
    out_idx = rng.permutation(nb).astype(np.uint64)
    got = run_gpu(B, small, cts, luts, torch_cuda, lut_idx=lut_idx, in_idx=in_idx, out_idx=out_idx)
    ref = run_oracle(oracle, small, cts, luts, lut_idx=lut_idx, in_idx=in_idx, out_idx=out_idx)
    assert np.array_equal(got, ref)
    dec = B.lwe_decrypt(small.glwe_sk, got, small.p.big_n)
    for s in range(nb):
        assert B.decode(dec[out_idx[s]], width) == int(tables[lut_idx[s]][msgs[in_idx[s]]])


def test_reference_fixtures_decrypt(B, cfg2, torch_cuda):
    """Cleartext vectors of the reference generators (p <= 3: cfg2's PBS output noise, sigma ~5.5e-3,
    leaves 5.7 sigma to the p = 3 decoding boundary but only 2.8 at p = 4), incl. the
    signed/unsigned variants: a signed input first gets the 2^(p-1) offset added to its body and
    the LUT is expanded half-rotated (FHEToTFHEScalar.cpp:373-413, wrappers.cpp:409-421)."""
    fx = json.load(open(GOLDEN))
    cases = [c for c in fx["apply_lookup_table"] + fx["linalg_apply_lookup_table"]
             if len(c["lut"]) <= 8 and not c["description"].endswith("_2layer")]
    assert len(cases) >= 30
    kinds = set()
    for ci, c in enumerate(cases):
        width = int(math.log2(len(c["lut"])))
        xs = [int(x) & ((1 << 64) - 1) for x in c["input"]]
        cts = encrypt(B, cfg2, xs, width, 500 + ci)
        if c["input_signed"]:
            cts[:, cfg2.p.n] += B.encode(1 << (width - 1), width)
        table = np.array(c["lut"], dtype=np.int64).view(np.uint64)
        acc = B.trivial_glwe(cfg2.p, B.expand_lut(table, cfg2.p.N, width, c["input_signed"]))
        got = run_gpu(B, cfg2, cts, acc, torch_cuda)
        dec = B.lwe_decrypt(cfg2.glwe_sk, got, cfg2.p.big_n)
        assert [B.decode(d, width, c["output_signed"]) for d in dec] == c["expected"], c["description"]
        kinds.add((c["input_signed"], c["output_signed"]))
    assert len(kinds) == 4


def test_metric_batch_properties(B, oracle, cfg2, torch_cuda):
    """B = 4096 (the metric's batch): every sample decrypts to LUT[m]; 16 random rows bit-exact."""
    width = 3
    nb = 4096
    rng = np.random.RandomState(11)
    table = rng.randint(0, 8, size=8)
    msgs = rng.randint(0, 8, size=nb)
    cts = encrypt(B, cfg2, msgs, width, 1234)
    acc = lut_acc(B, cfg2, table, width)
    got = run_gpu(B, cfg2, cts, acc, torch_cuda)
    dec = B.lwe_decrypt(cfg2.glwe_sk, got, cfg2.p.big_n)
    assert all(B.decode(d, width) == table[m] for d, m in zip(dec, msgs))
    pick = rng.choice(nb, size=16, replace=False)
    ref = run_oracle(oracle, cfg2, cts[pick], acc)
    assert np.array_equal(got[pick], ref)


def test_legacy_abi_sequence(B, oracle, small, torch_cuda):
    """Replay of memref_batched_bootstrap_lwe_cuda_u64 (wrappers.cpp:164-256) on the cuda_* ABI:
    stream, H2D, convert (registry), scratch, PBS, cleanup, D2H, drop."""
    from concrete_amd import _native
    L = _native.lib()
    p = small.p
    width = 3
    msgs = np.arange(8)
    cts = encrypt(B, small, msgs, width, 55, std=2.0 ** -25)
    acc = lut_acc(B, small, [7, 6, 5, 4, 3, 2, 1, 0], width)
    nb = len(msgs)
    s = L.cuda_create_stream(0)
    bsk_bytes = p.bsk_len * 8
    d_bsk = L.cuda_malloc_async(bsk_bytes, s, 0)
    L.cuda_convert_lwe_programmable_bootstrap_key_64(s, 0, d_bsk, small.bsk.ctypes.data, p.n, p.k, p.level, p.N)
    assert L.concrete_hip_lookup_bsk(d_bsk)
    d_in = L.cuda_malloc_async(cts.nbytes, s, 0)
    L.cuda_memcpy_async_to_gpu(d_in, cts.ctypes.data, cts.nbytes, s, 0)
    d_out = L.cuda_malloc_async(nb * p.lwe_out_size * 8, s, 0)
    d_acc = L.cuda_malloc_async(acc.nbytes, s, 0)
    L.cuda_memcpy_async_to_gpu(d_acc, acc.ctypes.data, acc.nbytes, s, 0)
    idx = np.arange(nb, dtype=np.uint64)
    zeros = np.zeros(nb, dtype=np.uint64)
    d_idx = L.cuda_malloc_async(idx.nbytes, s, 0)
    d_lidx = L.cuda_malloc_async(idx.nbytes, s, 0)
    L.cuda_memcpy_async_to_gpu(d_idx, idx.ctypes.data, idx.nbytes, s, 0)
    L.cuda_memcpy_async_to_gpu(d_lidx, zeros.ctypes.data, zeros.nbytes, s, 0)
    buf = C.c_void_p()
    L.scratch_cuda_programmable_bootstrap_64(s, 0, C.byref(buf), p.k, p.N, p.level, nb, True)
    L.cuda_programmable_bootstrap_lwe_ciphertext_vector_64(s, 0, d_out, d_idx, d_acc, d_lidx, d_in, d_idx, d_bsk,
                                                          buf, p.n, p.k, p.N, p.base_log, p.level, nb, 1, 1)
    L.cleanup_cuda_programmable_bootstrap(s, 0, C.byref(buf))
    assert not buf.value
    out = np.zeros((nb, p.lwe_out_size), dtype=np.uint64)
    L.cuda_memcpy_async_to_cpu(out.ctypes.data, d_out, out.nbytes, s, 0)
    L.cuda_synchronize_device(0)
    for ptr in (d_in, d_out, d_acc, d_idx, d_lidx):
        L.cuda_drop_async(ptr, s, 0)
    L.cuda_drop(d_bsk, 0)
    assert not L.concrete_hip_lookup_bsk(d_bsk)
    L.cuda_destroy_stream(s, 0)
    ref = run_oracle(oracle, small, cts, acc)
    assert np.array_equal(out, ref)


def test_keyswitch_bit_exact_and_chain(B, oracle, cfg2, torch_cuda):
    """KS (kN -> n) bit-exact vs the oracle, then the KS -> PBS atomic pattern
    (FHEToTFHEScalar.cpp:373-437) on the reference's 2-layer fixtures with p <= 2."""
    p = cfg2.p
    op = cfg2.op
    ksk = B.ksk_generate(p, cfg2.glwe_sk, cfg2.lwe_sk, 4321)
    d_ksk = B.to_device(ksk, "cuda:0")
    fx = json.load(open(GOLDEN))
    cases = [c for c in fx["linalg_apply_lookup_table"] if c["description"].endswith("_2layer") and len(c["lut"]) <= 4]
    assert cases
    for ci, c in enumerate(cases):
        width = int(math.log2(len(c["lut"])))
        xs = c["input"]
        cts = encrypt(B, cfg2, xs, width, 900 + ci)
        acc = lut_acc(B, cfg2, c["lut"], width)
        big = run_gpu(B, cfg2, cts, acc, torch_cuda)            # layer 1: PBS -> kN key
        d_big = B.to_device(big, "cuda:0")
        d_small = B.keyswitch(p, d_ksk, d_big)
        torch_cuda.cuda.synchronize()
        small_cts = B.to_host(d_small)
        assert np.array_equal(small_cts, oracle.keyswitch_batch(op, big, ksk))
        out = run_gpu(B, cfg2, small_cts, acc, torch_cuda)      # layer 2
        dec = B.lwe_decrypt(cfg2.glwe_sk, out, p.big_n)
        assert [B.decode(d, width) for d in dec] == c["expected"], c["description"]


@pytest.mark.parametrize("ks_l,ks_logB", [(4, 3), (7, 3), (3, 4), (4, 4), (6, 6), (2, 10), (2, 11), (1, 20),
                                          (2, 31), (1, 40)])
def test_keyswitch_decompositions(B, oracle, torch_cuda, ks_l, ks_logB):
    """The keyswitch's three product paths (keyswitch.hip), selected by dmax = l 2^(logB-1):
    three 22/21/21-bit key chunks with int32 sums over 16-position blocks when dmax <= 32 ((4,3),
    (7,3), (3,4), and (4,4) at the edge), four 16-bit chunks over 32-position blocks when
    dmax <= 1024 ((6,6), and (2,10) at the edge), the 64-bit products with int64 digits otherwise
    ((2,11), (1,20), and (2,31), (1,40) where a balanced digit can reach +2^31 or beyond); random
    inputs, 37 samples (a partial tile), bit-exact vs the oracle."""
    p = replace(B.CFG2, ks_level=ks_l, ks_base_log=ks_logB)
    glwe_sk = B.binary_key(p.big_n, 8100 + ks_logB)
    lwe_sk = B.binary_key(p.n, 8200 + ks_logB)
    ksk = B.ksk_generate(p, glwe_sk, lwe_sk, 8300 + ks_logB)
    rng = np.random.RandomState(ks_logB)
    cts = rng.randint(0, 2 ** 63, size=(37, p.big_n + 1), dtype=np.int64).astype(np.uint64) * np.uint64(2) + \
        np.uint64(1)
    out = B.keyswitch(p, B.to_device(ksk, "cuda:0"), B.to_device(cts, "cuda:0"))
    torch_cuda.cuda.synchronize()
    op = oracle.Params(n=p.n, k=p.k, N=p.N, l=p.level, logB=p.base_log, ks_l=ks_l, ks_logB=ks_logB)
    assert np.array_equal(B.to_host(out), oracle.keyswitch_batch(op, cts, ksk))


@pytest.mark.parametrize("ks_l,ks_logB,nb", [(4, 3, 64), (4, 3, 300), (7, 3, 129), (3, 4, 200), (5, 3, 96),
                                             (2, 7, 70), (1, 7, 65)])
def test_keyswitch_mfma_path(B, oracle, torch_cuda, ks_l, ks_logB, nb):
    """The int8 matrix-core keyswitch (keyswitch.hip ks_mfma_kernel: 8 balanced key bytes x int8
    digits, int32 sums, taken from 64 samples on when base_log <= 7): bit-exact vs the oracle,
    ragged batches (partial 64-row tiles), n + 1 = 631 output words (partial column tile), the
    widest accepted digits (logB = 7), and permuted in_idx / out_idx."""
    p = replace(B.CFG2, ks_level=ks_l, ks_base_log=ks_logB)
    glwe_sk = B.binary_key(p.big_n, 8400 + ks_logB + ks_l)
    lwe_sk = B.binary_key(p.n, 8500 + ks_logB + ks_l)
    ksk = B.ksk_generate(p, glwe_sk, lwe_sk, 8600 + ks_logB + ks_l)
    rng = np.random.RandomState(nb)
    cts = rng.randint(0, 2 ** 63, size=(nb, p.big_n + 1), dtype=np.int64).astype(np.uint64) * np.uint64(2) + \
        np.uint64(1)
    cts[0] = 0
    cts[1] = np.uint64(0xFFFFFFFFFFFFFFFF)
    dev = "cuda:0"
    d_ksk = B.to_device(ksk, dev)
    op = oracle.Params(n=p.n, k=p.k, N=p.N, l=p.level, logB=p.base_log, ks_l=ks_l, ks_logB=ks_logB)
    ref = oracle.keyswitch_batch(op, cts, ksk)
    out = B.keyswitch(p, d_ksk, B.to_device(cts, dev))
    torch_cuda.cuda.synchronize()
    assert np.array_equal(B.to_host(out), ref)
    in_idx = rng.permutation(nb).astype(np.uint64)
    out_idx = rng.permutation(nb).astype(np.uint64)
    out2 = B.keyswitch(p, d_ksk, B.to_device(cts, dev), in_idx=B.to_device(in_idx, dev),
                       out_idx=B.to_device(out_idx, dev))
    torch_cuda.cuda.synchronize()
    exp = np.zeros_like(ref)
    exp[out_idx.astype(np.int64)] = ref[in_idx.astype(np.int64)]
    assert np.array_equal(B.to_host(out2), exp)


def test_keyswitch_mfma_multi_pass(B, oracle, torch_cuda, monkeypatch):
    """The matrix-core keyswitch in several passes over the batch (the digit matrix of one pass
    is capped; CONCRETE_HIP_KS_CHUNK lowers the cap to 128 rows): 300 samples = 3 passes, with
    and without index arrays, bit-exact vs the oracle."""
    p = B.CFG2
    glwe_sk = B.binary_key(p.big_n, 8701)
    lwe_sk = B.binary_key(p.n, 8702)
    ksk = B.ksk_generate(p, glwe_sk, lwe_sk, 8703)
    rng = np.random.RandomState(8704)
    nb = 300
    cts = rng.randint(0, 2 ** 63, size=(nb, p.big_n + 1), dtype=np.int64).astype(np.uint64) * np.uint64(2) + \
        np.uint64(1)
    dev = "cuda:0"
    d_ksk = B.to_device(ksk, dev)
    op = oracle.Params(n=p.n, k=p.k, N=p.N, l=p.level, logB=p.base_log, ks_l=p.ks_level, ks_logB=p.ks_base_log)
    ref = oracle.keyswitch_batch(op, cts, ksk)
    monkeypatch.setenv("CONCRETE_HIP_KS_CHUNK", "128")
    out = B.keyswitch(p, d_ksk, B.to_device(cts, dev))
    in_idx = rng.permutation(nb).astype(np.uint64)
    out_idx = rng.permutation(nb).astype(np.uint64)
    out2 = B.keyswitch(p, d_ksk, B.to_device(cts, dev), in_idx=B.to_device(in_idx, dev),
                       out_idx=B.to_device(out_idx, dev))
    torch_cuda.cuda.synchronize()
    assert np.array_equal(B.to_host(out), ref)
    exp = np.zeros_like(ref)
    exp[out_idx.astype(np.int64)] = ref[in_idx.astype(np.int64)]
    assert np.array_equal(B.to_host(out2), exp)


def test_configs2_total_batch_65536(B, oracle, cfg2, torch_cuda):
    """BASELINE configs[2]'s whole batch (65,536 PBS) in one launch on one GPU: every sample
    decrypts to LUT[m], 8 random rows bit-exact, outputs of identical inputs identical."""
    width = 3
    nb = 65536
    rng = np.random.RandomState(21)
    table = rng.randint(0, 8, size=8)
    msgs = rng.randint(0, 8, size=nb)
    cts = encrypt(B, cfg2, msgs, width, 2121)
    cts[nb - 1] = cts[0]
    msgs[nb - 1] = msgs[0]
    acc = lut_acc(B, cfg2, table, width)
    got = run_gpu(B, cfg2, cts, acc, torch_cuda)
    dec = B.lwe_decrypt(cfg2.glwe_sk, got, cfg2.p.big_n)
    bad = [s for s, (d, m) in enumerate(zip(dec, msgs)) if B.decode(d, width) != table[m]]
    assert not bad, (len(bad), bad[:8])
    assert np.array_equal(got[0], got[nb - 1])
    pick = rng.choice(nb, size=8, replace=False)
    ref = run_oracle(oracle, cfg2, cts[pick], acc)
    assert np.array_equal(got[pick], ref)


def test_sync_timeout_is_reported(B, oracle, cfg2, torch_cuda):
    """A wave-pair synchronisation that exceeds its spin bound is reported, not silent
    (kernel_util.hpp spin_until_ge): with the bound forced to one poll some sync of a
    512-sample batch gives up, concrete_hip_device_status returns -4 (and clears); with the
    default bound the same batch runs clean and bit-exact."""
    width = 3
    rng = np.random.RandomState(31)
    table = rng.randint(0, 8, size=8)
    msgs = rng.randint(0, 8, size=512)
    cts = encrypt(B, cfg2, msgs, width, 3131)
    acc = lut_acc(B, cfg2, table, width)
    assert B.device_status("cuda:0") == 0
    try:
        B.set_spin_limit(1)
        run_gpu(B, cfg2, cts, acc, torch_cuda)
        assert B.device_status("cuda:0") == -4
        assert "spin bound" in B._native.lib().concrete_hip_last_error().decode()
    finally:
        B.set_spin_limit(0)
    assert B.device_status("cuda:0") == 0  # cleared
    got = run_gpu(B, cfg2, cts[:16], acc, torch_cuda)
    assert B.device_status("cuda:0") == 0
    assert np.array_equal(got, run_oracle(oracle, cfg2, cts[:16], acc))


def test_keyswitch_key_byte_cache_and_fallback(B, oracle, torch_cuda, monkeypatch):
    """the matrix-core keyswitch caches the int8 key bytes of a KSK whose lifetime the
    backend sees (allocated by cuda_malloc_async, as the runtime allocates it), releases them on
    cuda_drop or a rewrite of the buffer, never caches torch-owned memory (its caching allocator
    reuses addresses), and falls back to the scratch-free VALU kernel when operand scratch is
    unavailable (CONCRETE_HIP_KS_SCRATCH_LIMIT forces that).  All bit-exact vs the oracle."""
    from concrete_amd import _native
    L = _native.lib()
    p = B.CFG2
    glwe_sk = B.binary_key(p.big_n, 8801)
    lwe_sk = B.binary_key(p.n, 8802)
    ksk = B.ksk_generate(p, glwe_sk, lwe_sk, 8803)
    ksk2 = B.ksk_generate(p, glwe_sk, lwe_sk, 8804)
    rng = np.random.RandomState(8805)
    nb = 200
    cts = rng.randint(0, 2 ** 63, size=(nb, p.big_n + 1), dtype=np.int64).astype(np.uint64) * np.uint64(2) + \
        np.uint64(1)
    op = oracle.Params(n=p.n, k=p.k, N=p.N, l=p.level, logB=p.base_log, ks_l=p.ks_level, ks_logB=p.ks_base_log)
    ref = oracle.keyswitch_batch(op, cts, ksk)
    ref2 = oracle.keyswitch_batch(op, cts, ksk2)
    d_in = B.to_device(cts, "cuda:0")
    kb = B.RuntimeBuffer(ksk)
    try:
        for _ in range(2):  # built once, then reused
            out = B.keyswitch(p, kb, d_in)
            torch_cuda.cuda.synchronize()
            assert np.array_equal(B.to_host(out), ref)
        kb.write(ksk2)  # cuda_memcpy_async_to_gpu onto the key drops its cached bytes
        out = B.keyswitch(p, kb, d_in)
        torch_cuda.cuda.synchronize()
        assert np.array_equal(B.to_host(out), ref2)
        assert L.concrete_hip_release_device_buffer(kb.data_ptr()) == 1
        assert L.concrete_hip_release_device_buffer(kb.data_ptr()) == 0
    finally:
        kb.free()
    d_ksk = B.to_device(ksk, "cuda:0")
    out = B.keyswitch(p, d_ksk, d_in)
    torch_cuda.cuda.synchronize()
    assert np.array_equal(B.to_host(out), ref)
    assert L.concrete_hip_release_device_buffer(d_ksk.data_ptr()) == 0  # torch memory: not cached
    monkeypatch.setenv("CONCRETE_HIP_KS_SCRATCH_LIMIT", "1")
    out = B.keyswitch(p, d_ksk, d_in)
    torch_cuda.cuda.synchronize()
    assert np.array_equal(B.to_host(out), ref)


@pytest.mark.parametrize("pairs,quad", [(1, -1), (2, -1), (1, 0), (2, 0), (4, -1), (1, 2), (2, 1)])
@pytest.mark.parametrize("level,base_log", [(1, 11), (2, 6), (3, 7)])
def test_pbs_pairs_per_workgroup(B, oracle, torch_cuda, monkeypatch, pairs, quad, level, base_log):
    """The N = 1024 kernel at 1, 2 and 4 ciphertexts per workgroup (the small-batch forms that keep
    every CU busy at <= 2 x CUs ciphertexts, pbs.hip launch_pair; CONCRETE_HIP_PBS_PAIRS forces
    one).  At l = 3 and 1 per workgroup the four-wave kernel runs by default (pbs1024_quad.hip;
    quad -1: the default, 1 / 2: forced with that many ciphertexts per workgroup, 0: the pair
    kernel): ragged batches, permuted index arrays, per-sample LUTs — bit-exact
    vs the oracle with the measured rounding residual below the certified bound."""
    monkeypatch.setenv("CONCRETE_HIP_PBS_PAIRS", str(pairs))
    if quad >= 0:
        monkeypatch.setenv("CONCRETE_HIP_PBS_QUAD", str(quad))
    p = replace(B.CFG2, n=12, level=level, base_log=base_log)
    S = Setup(B, oracle, torch_cuda, p, 5100 + 10 * level + pairs)
    width = 2
    rng = np.random.RandomState(pairs * 100 + level)
    nb = 7
    tables = [rng.randint(0, 4, size=4) for _ in range(nb)]
    msgs = rng.randint(0, 4, size=nb)
    cts = encrypt(B, S, msgs, width, 51 + pairs, std=2.0 ** -25)
    accs = np.stack([lut_acc(B, S, t, width) for t in tables])
    in_idx = rng.permutation(nb).astype(np.uint64)
    out_idx = rng.permutation(nb).astype(np.uint64)
    lut_idx = rng.permutation(nb).astype(np.uint64)
    dev = "cuda:0"
    resid = torch_cuda.zeros(1, dtype=torch_cuda.int64, device=dev)
    out = B.pbs(p, S.fbsk, B.to_device(cts, dev), B.to_device(accs, dev), lut_idx=B.to_device(lut_idx, dev),
                in_idx=B.to_device(in_idx, dev), out_idx=B.to_device(out_idx, dev), resid=resid)
    torch_cuda.cuda.synchronize()
    got = B.to_host(out)
    ref, _ = oracle.pbs_batch(S.op, cts[in_idx.astype(np.int64)], accs, fbsk=S.fbsk_cpu, lut_idx=lut_idx)
    exp = np.zeros_like(ref)
    exp[out_idx.astype(np.int64)] = ref
    assert np.array_equal(got, exp)
    r = float(np.array([int(resid.cpu()[0])], dtype=np.int64).view(np.float64)[0])
    assert r < oracle.fft_error_bound(S.op, S.fbsk_cpu) < 0.5


@pytest.mark.parametrize("n_out,ks_l,ks_logB,nb", [(1024, 4, 3, 37), (1500, 4, 3, 37), (1500, 2, 11, 21),
                                                   (2100, 3, 4, 96), (1024, 4, 3, 80)])
def test_keyswitch_wide_output_rows(B, oracle, torch_cuda, n_out, ks_l, ks_logB, nb):
    """Output LWE dimensions past 1023 (the VALU kernel's 1024-word block, now windows of 1024
    words in blockIdx.z; the matrix-core path from 64 samples): n + 1 = 1025 (a one-word second
    window), 1501, 2101; int32-chunk and 64-bit product forms; bit-exact vs the oracle."""
    p = replace(B.CFG2, n=n_out, ks_level=ks_l, ks_base_log=ks_logB)
    glwe_sk = B.binary_key(p.big_n, 8700 + n_out)
    lwe_sk = B.binary_key(p.n, 8800 + n_out)
    ksk = B.ksk_generate(p, glwe_sk, lwe_sk, 8900 + n_out)
    rng = np.random.RandomState(n_out + nb)
    cts = rng.randint(0, 2 ** 63, size=(nb, p.big_n + 1), dtype=np.int64).astype(np.uint64) * np.uint64(2) + \
        np.uint64(1)
    out = B.keyswitch(p, B.to_device(ksk, "cuda:0"), B.to_device(cts, "cuda:0"))
    torch_cuda.cuda.synchronize()
    op = oracle.Params(n=p.n, k=p.k, N=p.N, l=p.level, logB=p.base_log, ks_l=ks_l, ks_logB=ks_logB)
    assert np.array_equal(B.to_host(out), oracle.keyswitch_batch(op, cts, ksk))


@pytest.mark.parametrize("ks_l,ks_logB,nb", [(4, 3, 4096), (4, 3, 300), (7, 3, 129), (2, 7, 70)])
def test_keyswitch_mfma_four_wave_kernel(B, oracle, torch_cuda, monkeypatch, ks_l, ks_logB, nb):
    """The four-wave LDS matrix-core keyswitch (CONCRETE_HIP_KS_WAVES=4: two 32-row tiles per wave,
    each key fragment serving two MFMAs): bit-exact vs the oracle at the cfg2 batch (split-K
    over 4 workgroups), ragged batches, the widest digits, and permuted index arrays."""
    monkeypatch.setenv("CONCRETE_HIP_KS_WAVES", "4")
    p = replace(B.CFG2, ks_level=ks_l, ks_base_log=ks_logB)
    glwe_sk = B.binary_key(p.big_n, 9400 + ks_logB + ks_l)
    lwe_sk = B.binary_key(p.n, 9500 + ks_logB + ks_l)
    ksk = B.ksk_generate(p, glwe_sk, lwe_sk, 9600 + ks_logB + ks_l)
    rng = np.random.RandomState(nb + 7)
    cts = rng.randint(0, 2 ** 63, size=(nb, p.big_n + 1), dtype=np.int64).astype(np.uint64) * np.uint64(2) + \
        np.uint64(1)
    dev = "cuda:0"
    d_ksk = B.to_device(ksk, dev)
    op = oracle.Params(n=p.n, k=p.k, N=p.N, l=p.level, logB=p.base_log, ks_l=ks_l, ks_logB=ks_logB)
    rows = np.arange(nb) if nb <= 300 else np.r_[0:64, nb - 64:nb]
    ref = oracle.keyswitch_batch(op, cts[rows], ksk)
    out = B.keyswitch(p, d_ksk, B.to_device(cts, dev))
    torch_cuda.cuda.synchronize()
    assert np.array_equal(B.to_host(out)[rows], ref)
    in_idx = rng.permutation(nb).astype(np.uint64)
    out2 = B.keyswitch(p, d_ksk, B.to_device(cts, dev), in_idx=B.to_device(in_idx, dev))
    torch_cuda.cuda.synchronize()
    sel = rows[: min(len(rows), 64)]
    exp = oracle.keyswitch_batch(op, cts[in_idx[sel].astype(np.int64)], ksk)
    assert np.array_equal(B.to_host(out2)[sel], exp)


@pytest.mark.parametrize("cts_per_wg", [1, 2])
@pytest.mark.parametrize("n", [1, 2, 3])
def test_pbs_quad_tiny_n(B, oracle, torch_cuda, monkeypatch, cts_per_wg, n):
    """The four-wave kernel (pbs1024_quad.hip) over blind rotations of 1-3 steps: its key ring's
    prologue and tail, the per-step delta exchange; bit-exact vs the oracle."""
    monkeypatch.setenv("CONCRETE_HIP_PBS_QUAD", str(cts_per_wg))
    p = replace(B.CFG2, n=n)
    S = Setup(B, oracle, torch_cuda, p, 5300 + 10 * n + cts_per_wg)
    width = 2
    rng = np.random.RandomState(n)
    msgs = rng.randint(0, 4, size=5)
    cts = encrypt(B, S, msgs, width, 71 + n, std=2.0 ** -25)
    acc = lut_acc(B, S, rng.randint(0, 4, size=4), width)
    dev = "cuda:0"
    out = B.pbs(p, S.fbsk, B.to_device(cts, dev), B.to_device(acc[None, :], dev))
    torch_cuda.cuda.synchronize()
    ref, _ = oracle.pbs_batch(S.op, cts, acc[None, :], fbsk=S.fbsk_cpu)
    assert np.array_equal(B.to_host(out), ref)


@pytest.mark.parametrize("cts_per_wg", [1, 2])
@pytest.mark.parametrize("n,base_log,nb", [(1, 3, 3), (1, 7, 5), (2, 9, 4), (3, 1, 7), (12, 7, 13), (12, 3, 9),
                                           (12, 9, 6)])
def test_pbs_hex_kernel(B, oracle, torch_cuda, monkeypatch, cts_per_wg, n, base_log, nb):
    """The six-wave kernel (pbs1024_hex.hip; CONCRETE_HIP_PBS_HEX forces it with 1 or 2 ciphertexts
    per workgroup): blind rotations of 0-12 steps (its key prefetch's prologue and the last step's
    re-read), every logB of the exact range's edges, ragged batches (an odd batch leaves a workgroup's
    second ciphertext idle), permuted index arrays and per-sample LUTs; bit-exact vs the oracle with
    the measured rounding residual below the certified bound."""
    monkeypatch.setenv("CONCRETE_HIP_PBS_HEX", str(cts_per_wg))
    p = replace(B.CFG2, n=n, level=3, base_log=base_log)
    S = Setup(B, oracle, torch_cuda, p, 5400 + 10 * n + base_log)
    width = 2
    rng = np.random.RandomState(nb * 100 + n)
    tables = [rng.randint(0, 4, size=4) for _ in range(nb)]
    msgs = rng.randint(0, 4, size=nb)
    cts = encrypt(B, S, msgs, width, 61 + n, std=2.0 ** -25)
    accs = np.stack([lut_acc(B, S, t, width) for t in tables])
    in_idx = rng.permutation(nb).astype(np.uint64)
    out_idx = rng.permutation(nb).astype(np.uint64)
    lut_idx = rng.permutation(nb).astype(np.uint64)
    dev = "cuda:0"
    resid = torch_cuda.zeros(1, dtype=torch_cuda.int64, device=dev)
    out = B.pbs(p, S.fbsk, B.to_device(cts, dev), B.to_device(accs, dev), lut_idx=B.to_device(lut_idx, dev),
                in_idx=B.to_device(in_idx, dev), out_idx=B.to_device(out_idx, dev), resid=resid)
    torch_cuda.cuda.synchronize()
    got = B.to_host(out)
    ref, _ = oracle.pbs_batch(S.op, cts[in_idx.astype(np.int64)], accs, fbsk=S.fbsk_cpu, lut_idx=lut_idx)
    exp = np.zeros_like(ref)
    exp[out_idx.astype(np.int64)] = ref
    assert np.array_equal(got, exp)
    if n > 0:
        r = float(np.array([int(resid.cpu()[0])], dtype=np.int64).view(np.float64)[0])
        assert r < oracle.fft_error_bound(S.op, S.fbsk_cpu) < 0.5


@pytest.mark.parametrize("cts_per_wg", [1, 2])
def test_pbs_hex_kernel_cfg2_full(B, oracle, cfg2, torch_cuda, monkeypatch, cts_per_wg):
    """The six-wave kernel on the full cfg2 row (n = 630): 67 ciphertexts bit-exact vs the oracle,
    every one decrypting to its LUT entry."""
    monkeypatch.setenv("CONCRETE_HIP_PBS_HEX", str(cts_per_wg))
    width = 3
    rng = np.random.RandomState(70 + cts_per_wg)
    table = rng.randint(0, 8, size=8)
    msgs = rng.randint(0, 8, size=67)
    cts = encrypt(B, cfg2, msgs, width, 78 + cts_per_wg)
    acc = lut_acc(B, cfg2, table, width)
    got, resid = run_gpu(B, cfg2, cts, acc, torch_cuda, resid=True)
    ref = run_oracle(oracle, cfg2, cts, acc)
    assert np.array_equal(got, ref)
    assert resid < oracle.fft_error_bound(cfg2.op, cfg2.fbsk_cpu) < 0.5
    dec = B.lwe_decrypt(cfg2.glwe_sk, got, cfg2.p.big_n)
    assert [B.decode(d, width) for d in dec] == [int(table[m]) for m in msgs]


def test_status_is_per_stream(B, oracle, cfg2, torch_cuda):
    """the sync-timeout status is attributed to the launch's own stream.  Two
    threads run the cfg2 PBS concurrently on two streams; one forces the spin bound to one poll for
    its own launch only (concrete_hip_set_thread_spin_limit).  That thread's stream reports -4, the
    other's reports 0 and its outputs are bit-exact (sampled rows vs the oracle, every row decrypts);
    the device-wide check afterwards is clean (both words were cleared by the stream reads)."""
    import threading
    torch = torch_cuda
    width = 3
    rng = np.random.RandomState(41)
    table = rng.randint(0, 8, size=8)
    msgs = rng.randint(0, 8, size=(2, 512))
    cts = [encrypt(B, cfg2, msgs[i], width, 4141 + i) for i in range(2)]
    acc = lut_acc(B, cfg2, table, width)
    dev = "cuda:0"
    assert B.device_status(dev) == 0
    streams = [torch.cuda.Stream(dev) for _ in range(2)]
    d_in = [B.to_device(c, dev) for c in cts]
    d_acc = B.to_device(acc[None, :], dev)
    outs = [torch.zeros((512, cfg2.p.lwe_out_size), dtype=torch.int64, device=dev) for _ in range(2)]
    torch.cuda.synchronize()
    status = [None, None]
    gate = threading.Barrier(2)

    def call(i):
        try:
            if i == 0:
                B.set_thread_spin_limit(1)
            with torch.cuda.stream(streams[i]):
                gate.wait()
                B.pbs(cfg2.p, cfg2.fbsk, d_in[i], d_acc, out=outs[i])
                status[i] = B.stream_status(dev, streams[i])
        finally:
            B.set_thread_spin_limit(0)

    th = [threading.Thread(target=call, args=(i,)) for i in range(2)]
    [t.start() for t in th]
    [t.join() for t in th]
    assert status == [-4, 0], status
    assert B.device_status(dev) == 0
    got = B.to_host(outs[1])
    rows = np.array([0, 255, 511])
    assert np.array_equal(got[rows], run_oracle(oracle, cfg2, cts[1][rows], acc))
    dec = B.lwe_decrypt(cfg2.glwe_sk, got, cfg2.p.big_n)
    assert [B.decode(d, width) for d in dec] == [int(table[m]) for m in msgs[1]]


@pytest.mark.parametrize("shape", ["pair+hex1", "pair+hex2", "hex2", "hex1", "pair"])
@pytest.mark.parametrize("indexed", [False, True])
def test_pbs_split_over_kernels(B, oracle, torch_cuda, monkeypatch, shape, indexed):
    """a cfg2-shaped call between round sizes is cut into contiguous parts run by
    the pair kernel, the six-wave kernel at 2 and at 1 ciphertext per workgroup
    (concrete_amd/csrc/pbs1024_plan.hpp), back to back on the caller's stream.  Ragged batches chosen
    so the plan holds each combination of parts (batch sizes relative to the device's CU count);
    with and without permuted index arrays and per-sample LUTs, every row equals the single-kernel
    run (the pair kernel forced) and sampled rows equal the oracle."""
    from concrete_amd import _native
    L = _native.lib()
    cus = torch_cuda.cuda.get_device_properties(0).multi_processor_count
    nb = {"pair+hex1": 4 * cus + cus // 2 + 3, "pair+hex2": 4 * cus + cus + 7, "hex2": cus + 3, "hex1": 5,
          "pair": 4 * cus - 9}[shape]
    parts = (C.c_uint32 * 3)()
    L.concrete_hip_pbs1024_plan(nb, cus, parts)
    got_parts = [x > 0 for x in parts]
    assert got_parts == [s in shape.split("+") for s in ("pair", "hex2", "hex1")], (shape, list(parts))
    p = replace(B.CFG2, n=12)
    S = Setup(B, oracle, torch_cuda, p, 6100 + nb)
    width = 2
    rng = np.random.RandomState(nb)
    msgs = rng.randint(0, 4, size=nb)
    cts = encrypt(B, S, msgs, width, 6200 + nb, std=2.0 ** -25)
    ntab = 5 if indexed else 1
    tables = [rng.randint(0, 4, size=4) for _ in range(ntab)]
    accs = np.stack([lut_acc(B, S, t, width) for t in tables])
    dev = "cuda:0"
    kw = {}
    if indexed:
        in_idx = rng.permutation(nb).astype(np.uint64)
        out_idx = rng.permutation(nb).astype(np.uint64)
        lut_idx = rng.randint(0, ntab, size=nb).astype(np.uint64)
        kw = dict(in_idx=B.to_device(in_idx, dev), out_idx=B.to_device(out_idx, dev),
                  lut_idx=B.to_device(lut_idx, dev))
    d_in, d_acc = B.to_device(cts, dev), B.to_device(accs, dev)
    split = B.to_host(B.pbs(p, S.fbsk, d_in, d_acc, **kw))
    monkeypatch.setenv("CONCRETE_HIP_PBS_PAIRS", "4")
    single = B.to_host(B.pbs(p, S.fbsk, d_in, d_acc, **kw))
    torch_cuda.cuda.synchronize()
    assert np.array_equal(split, single)
    rows = np.unique(np.array([0, 1, nb // 3, nb // 2, nb - 2, nb - 1]))
    if indexed:
        src = np.zeros(nb, dtype=np.int64)
        src[out_idx.astype(np.int64)] = in_idx.astype(np.int64)  # output row -> input row
        lut_of = np.zeros(nb, dtype=np.uint64)
        lut_of[out_idx.astype(np.int64)] = lut_idx
        ref, _ = oracle.pbs_batch(S.op, cts[src[rows]], accs, fbsk=S.fbsk_cpu, lut_idx=lut_of[rows])
    else:
        ref, _ = oracle.pbs_batch(S.op, cts[rows], accs, fbsk=S.fbsk_cpu)
    assert np.array_equal(split[rows], ref)
