"""GPU parity tests of the general path (concrete_amd/csrc/pbs_generic.hip): the concrete
optimizer's parameter sets beyond the two hand-tuned kernels — k = 2..6 GLWE masks at
N = 256..1024 and k = 1 at N = 4096..16384 (compilers/concrete-optimizer/v0-parameters/ref/
v0_last_128: 1-, 3-, 4-, 6-, 7- and 8-bit rows at log norm2 0).

Every case: GPU PBS bit-exact (u64) vs the oracle's pure-integer Karatsuba product on the same
keys and inputs, the measured rounding residual below 1/2 and below the scheme's certified
bound for this key (oracle/pyoracle.py:generic_error_bound with the key's measured max|G|), and
decrypt(out) == LUT[m] for every sample.  n is cut down so the O(N^1.6) oracle stays fast; the
8-bit set also runs at its full n = 1006 (decrypt-level only).
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


# (label, k, N, n, l, logB, message bits): v0_last_128 rows with n reduced for the oracle
CASES = [
    ("1bit_k5_N256", 5, 256, 24, 1, 15, 1),
    ("2bit_k6_N256", 6, 256, 16, 1, 18, 2),  # the small-ring kernel since round 4
    ("3bit_k3_N512", 3, 512, 16, 1, 18, 3),
    ("4bit_k2_N1024", 2, 1024, 12, 1, 23, 4),
    ("k1_N2048_l2", 1, 2048, 12, 2, 10, 3),  # the N = 2048 kernel's levels since round 4
    ("6bit_k1_N4096", 1, 4096, 6, 1, 22, 6),
    ("7bit_k1_N8192", 1, 8192, 4, 1, 22, 7),
    ("8bit_k1_N16384", 1, 16384, 3, 2, 15, 8),
    # shapes off the tile kernels' instances (T = 1): k = 3, N = 512 at logB = 12 (the small-ring
    # kernel's one-sub-digit form since round 4) and the two-launch path at N = 1024
    ("k3_N512_logB12_small", 3, 512, 12, 1, 12, 3),
    ("k2_N1024_l2", 2, 1024, 10, 2, 10, 3),  # the k = 2 kernel's two-level form since round 4
    # four-step kernel with a 64-bit decomposition state (level * logB > 31): R = 4, 8, 16 rows
    ("k1_N4096_l3_wide_state", 1, 4096, 4, 3, 12, 3),
    ("k1_N8192_l2_wide_state", 1, 8192, 3, 2, 17, 4),
    ("k1_N16384_l3_wide_state", 1, 16384, 2, 3, 11, 3),
    # N = 2^15 / 2^16 (the 9- and 10-bit rows, v0_last_128:243 / :264): a polynomial spread over
    # S = 2 / 4 workgroups (gen_split_*_kernel), the key converted the same way
    ("9bit_k1_N32768", 1, 32768, 2, 2, 15, 9),
    ("10bit_k1_N65536", 1, 65536, 2, 2, 14, 10),
    # round 4: the 1- to 4-bit log-norm2-0 rows above run on their own kernels (pbs_small.hip,
    # pbs1024k2.hip), and so do the small-ring rows at l = 2, 3 whose digits fit whole and k = 4,
    # N = 512, l = 2 on 13-bit key limbs (the next three; the tile kernels serve the general-format
    # key of the shapes above, test_generic_tile_kernels_on_the_general_format_key)
    ("3bit_k4_N512_l2", 4, 512, 12, 2, 16, 3),
    ("2bit_k5_N256_l2", 5, 256, 16, 2, 10, 2),
    ("1bit_k6_N256_l2", 6, 256, 12, 2, 12, 1),
    ("3bit_k4_N512", 4, 512, 14, 1, 23, 3),  # pbs512k4.hip since round 4 (test_gpu_pbs_small.py)
    # l = 4 at N = 256 (the general path; no table row) and k = 2, N = 1024, l = 4 (br 4/9: the k = 2
    # kernel's one-level-at-a-time form since round 4)
    ("k5_N256_l4", 5, 256, 12, 4, 7, 2),
    ("k2_N1024_l4", 2, 1024, 10, 4, 9, 3),
    ("k6_N256_l4", 6, 256, 10, 4, 8, 1),
    ("k1_N2048_l5", 1, 2048, 6, 5, 8, 3),  # the general path's N = 2048 four-step kernels
    ("k3_N512_l4", 3, 512, 8, 4, 9, 2),  # the general path's two-launch kernels at N = 512
    ("k4_N512_l6", 4, 512, 8, 6, 7, 2),  # pbs512k4.hip's many-level kernel since round 4
    ("k3_N1024_l2", 3, 1024, 6, 2, 10, 2),  # the general path's two-launch kernels at N = 1024
]


def setup(B, torch, k, N, n, l, logB, seed):
    p = B.PbsParams(n=n, k=k, N=N, level=l, base_log=logB)
    assert B.pbs_supported(p), p
    lwe_sk = B.binary_key(p.n, seed)
    glwe_sk = B.binary_key(p.big_n, seed + 1)
    bsk = B.bsk_generate(p, lwe_sk, glwe_sk, seed + 2)
    fbsk = B.convert_bsk(p, bsk, "cuda:0")
    torch.cuda.synchronize()
    return p, lwe_sk, glwe_sk, bsk, fbsk


def run_case(B, oracle, torch, case, seed, batch=6):
    label, k, N, n, l, logB, width = case
    p, lwe_sk, glwe_sk, bsk, fbsk = setup(B, torch, k, N, n, l, logB, seed)
    rng = np.random.RandomState(seed)
    table = rng.randint(0, 1 << width, size=1 << width).astype(np.uint64)
    msgs = rng.randint(0, 1 << width, size=batch)
    # n is far below a secure LWE dimension here, so the curve's noise would swamp the message:
    # encrypt with a small fixed noise instead (the 8-bit full-size test uses the real one)
    cts = B.lwe_encrypt(lwe_sk, [B.encode(m, width) for m in msgs], p.n, 2.0 ** -30, seed + 3)
    acc = B.trivial_glwe(p, B.expand_lut(table, p.N, width))
    dev = "cuda:0"
    r = torch.zeros(1, dtype=torch.int64, device=dev)
    out = B.pbs(p, fbsk, B.to_device(cts, dev), B.to_device(acc[None, :], dev), resid=r)
    torch.cuda.synchronize()
    got = B.to_host(out)
    resid = float(np.array([r.item()], dtype=np.int64).view(np.float64)[0])
    return p, glwe_sk, bsk, fbsk, cts, acc, table, msgs, got, resid


@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_generic_pbs_bit_exact(B, oracle, torch_cuda, case):
    p, glwe_sk, bsk, fbsk, cts, acc, table, msgs, got, resid = run_case(B, oracle, torch_cuda, case, 7000)
    op = oracle.Params(n=p.n, k=p.k, N=p.N, l=p.level, logB=p.base_log)
    ref, _ = oracle.pbs_batch(op, cts, acc[None, :], bsk=bsk, mode=oracle.MODE_KARATSUBA)
    assert np.array_equal(got, ref), f"{case[0]}: GPU differs from the exact oracle"
    kind, limbs, bits = B.bsk_format(p)
    if kind == 2:  # N = 2048: pbs2048.hip (test_gpu_pbs2048.py)
        bound = oracle.gpu2048_error_bound(B.to_host(fbsk).view(np.float64), p.base_log, p.level)
    elif kind == 4:  # k = 2, N = 1024, l = 1 / 2: its own kernel since round 4 (test_gpu_pbs1024k2.py)
        bound = oracle.gpu1024k2_error_bound(B.to_host(fbsk).view(np.float64), p.base_log, p.level)
    elif kind == 5:  # N = 512, k = 3 / 4, N = 256, k = 5 / 6, l = 1: pbs_small.hip, pbs512k4.hip
        bound = oracle.gpu_small_error_bound(B.to_host(fbsk).view(np.float64), p.N, p.k, p.base_log, p.level)
    else:
        bound = oracle.generic_error_bound(p.k, p.N, p.level, p.base_log, bits, B.to_host(fbsk).view(np.float64))
    assert bound < 0.5, f"{case[0]}: certified bound {bound}"
    assert resid < bound, (resid, bound)
    width = case[6]
    dec = B.lwe_decrypt(glwe_sk, got, p.big_n)
    assert [B.decode(d, width) for d in dec] == [int(table[m]) for m in msgs]


@pytest.mark.parametrize("ci", [19, 23, 21, 5], ids=[CASES[i][0] for i in (19, 23, 21, 5)])
def test_generic_tile_many_workgroups(B, oracle, torch_cuda, ci):
    """The general path over many ciphertexts (67: not a multiple of any workgroup's ciphertext
    count, so the last workgroup runs empty slots): small-ring shapes off the hand-tuned kernels and the
    one-launch N = 4096 kernel (a workgroup per ciphertext), bit-exact vs the exact oracle."""
    case = CASES[ci][:3] + (4,) + CASES[ci][4:]
    p, glwe_sk, bsk, fbsk, cts, acc, table, msgs, got, resid = run_case(B, oracle, torch_cuda, case, 7500, batch=67)
    op = oracle.Params(n=p.n, k=p.k, N=p.N, l=p.level, logB=p.base_log)
    ref, _ = oracle.pbs_batch(op, cts, acc[None, :], bsk=bsk, mode=oracle.MODE_KARATSUBA)
    assert np.array_equal(got, ref)
    dec = B.lwe_decrypt(glwe_sk, got, p.big_n)
    assert [B.decode(d, case[6]) for d in dec] == [int(table[m]) for m in msgs]


def test_generic_8bit_long_chain_decrypts(B, oracle, torch_cuda):
    """v0_last_128 8-bit row (k = 1, N = 16384, l = 2, logB = 15) over a 128-step blind rotation:
    every output decrypts to LUT[m] (decrypt-level: 128 Karatsuba steps at N = 16384 are slow)."""
    p, lwe_sk, glwe_sk, bsk, fbsk = setup(B, torch_cuda, 1, 16384, 128, 2, 15, 7100)
    width = 8
    rng = np.random.RandomState(8)
    table = rng.randint(0, 256, size=256).astype(np.uint64)
    msgs = rng.randint(0, 256, size=32)
    cts = B.lwe_encrypt(lwe_sk, [B.encode(m, width) for m in msgs], p.n, 2.0 ** -30, 7103)
    acc = B.trivial_glwe(p, B.expand_lut(table, p.N, width))
    out = B.pbs(p, fbsk, B.to_device(cts, "cuda:0"), B.to_device(acc[None, :], "cuda:0"))
    torch_cuda.cuda.synchronize()
    dec = B.lwe_decrypt(glwe_sk, B.to_host(out), p.big_n)
    assert [B.decode(d, width) for d in dec] == [int(table[m]) for m in msgs]


@pytest.mark.parametrize("ci", [19, 23, 21, 25, 20], ids=[CASES[i][0] for i in (19, 23, 21, 25, 20)])
def test_generic_index_arrays(B, oracle, torch_cuda, ci):
    """Mapped LUTs and permuted input/output rows (GPUDFG.cpp:1149-1205) on the general path:
    the one-launch tile kernels (N = 256: 4 ciphertexts per workgroup, the last one partly
    empty; N = 512) and the N = 1024 two-launch path."""
    label, k, N, n, l, logB, width = CASES[ci]
    p, lwe_sk, glwe_sk, bsk, fbsk = setup(B, torch_cuda, k, N, n, l, logB, 7200)
    rng = np.random.RandomState(3)
    tables = [rng.randint(0, 1 << width, size=1 << width).astype(np.uint64) for _ in range(3)]
    luts = np.stack([B.trivial_glwe(p, B.expand_lut(t, p.N, width)) for t in tables])
    msgs = rng.randint(0, 1 << width, size=7)
    cts = B.lwe_encrypt(lwe_sk, [B.encode(m, width) for m in msgs], p.n, 2.0 ** -30, 7203)
    in_idx = np.array([6, 0, 5, 1, 4, 2, 3], dtype=np.uint64)
    out_idx = np.array([3, 4, 0, 6, 1, 5, 2], dtype=np.uint64)
    lut_idx = np.array([0, 1, 2, 0, 1, 2, 0], dtype=np.uint64)
    dev = "cuda:0"
    d = {name: B.to_device(a, dev) for name, a in (("in_idx", in_idx), ("out_idx", out_idx), ("lut_idx", lut_idx))}
    out = torch_cuda.zeros((7, p.lwe_out_size), dtype=torch_cuda.int64, device=dev)
    B.pbs(p, fbsk, B.to_device(cts, dev), B.to_device(luts, dev), out=out, **d)
    torch_cuda.cuda.synchronize()
    op = oracle.Params(n=p.n, k=p.k, N=p.N, l=p.level, logB=p.base_log)
    ref, _ = oracle.pbs_batch(op, cts, luts, bsk=bsk, mode=oracle.MODE_KARATSUBA, lut_idx=lut_idx, in_idx=in_idx,
                              out_idx=out_idx)
    assert np.array_equal(B.to_host(out), ref)


def test_generic_legacy_step_kernel(B, oracle, torch_cuda):
    """CONCRETE_HIP_GEN_FOURSTEP=0 (natural-order keys, gen_step_kernel) stays bit-exact: the
    N = 4096 and 16384 rows in a child process, since the choice is made once per process."""
    import os
    import subprocess
    import sys
    code = (
        "import sys; sys.path.insert(0, %r); import tests.test_gpu_pbs_generic as T; "
        "from concrete_amd import backend as B; import oracle.pyoracle as O; import torch, numpy as np\n"
        "for ci in (5, 7):\n"
        "    p, glwe_sk, bsk, fbsk, cts, acc, table, msgs, got, resid = T.run_case(B, O, torch, T.CASES[ci], 7600)\n"
        "    op = O.Params(n=p.n, k=p.k, N=p.N, l=p.level, logB=p.base_log)\n"
        "    ref, _ = O.pbs_batch(op, cts, acc[None, :], bsk=bsk, mode=O.MODE_KARATSUBA)\n"
        "    assert np.array_equal(got, ref), T.CASES[ci][0]\n"
        "print('legacy ok')\n" % os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    env = dict(os.environ, CONCRETE_HIP_GEN_FOURSTEP="0")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "legacy ok" in r.stdout, r.stdout[-2000:] + r.stderr[-2000:]


@pytest.mark.parametrize("streams", [0, 1, 2, 3])
@pytest.mark.parametrize("ci", [5, 7, 13, 14], ids=[CASES[i][0] for i in (5, 7, 13, 14)])
def test_generic_chunked_two_streams(B, oracle, torch_cuda, ci, streams, monkeypatch):
    """The two-launch path (N = 4096 / 16384) and the split path (N = 2^15 / 2^16, chunk groups on
    several streams since round 6) over several chunks (CONCRETE_HIP_GEN_CHUNK=3 on 7 ciphertexts: 3
    chunks of 3 + 3 + 1 on one or three streams, evened to 4 chunks of 2 + 2 + 2 + 1 for two
    streams: groups of chunks on the caller's and library streams), with permuted input / output
    rows and mapped LUTs: bit-exact vs the exact oracle."""
    label, k, N, n, l, logB, width = CASES[ci]
    p, lwe_sk, glwe_sk, bsk, fbsk = setup(B, torch_cuda, k, N, n, l, logB, 7700)
    rng = np.random.RandomState(11)
    tables = [rng.randint(0, 1 << width, size=1 << width).astype(np.uint64) for _ in range(2)]
    luts = np.stack([B.trivial_glwe(p, B.expand_lut(t, p.N, width)) for t in tables])
    msgs = rng.randint(0, 1 << width, size=7)
    cts = B.lwe_encrypt(lwe_sk, [B.encode(m, width) for m in msgs], p.n, 2.0 ** -30, 7703)
    in_idx = np.array([3, 6, 0, 5, 1, 4, 2], dtype=np.uint64)
    out_idx = np.array([5, 2, 6, 0, 3, 1, 4], dtype=np.uint64)
    lut_idx = np.array([1, 0, 1, 1, 0, 0, 1], dtype=np.uint64)
    dev = "cuda:0"
    d = {name: B.to_device(a, dev) for name, a in (("in_idx", in_idx), ("out_idx", out_idx), ("lut_idx", lut_idx))}
    out = torch_cuda.zeros((7, p.lwe_out_size), dtype=torch_cuda.int64, device=dev)
    monkeypatch.setenv("CONCRETE_HIP_GEN_CHUNK", "3")
    monkeypatch.setenv("CONCRETE_HIP_GEN_STREAMS", str(streams))
    # N = 4096 has the one-launch kernel (gen_fused_kernel): streams = 0 runs it on the same index
    # arrays, the others force the two-launch path this test is about
    monkeypatch.setenv("CONCRETE_HIP_GEN_FUSED", "1" if streams == 0 else "0")
    B.pbs(p, fbsk, B.to_device(cts, dev), B.to_device(luts, dev), out=out, **d)
    torch_cuda.cuda.synchronize()
    op = oracle.Params(n=p.n, k=p.k, N=p.N, l=p.level, logB=p.base_log)
    ref, _ = oracle.pbs_batch(op, cts, luts, bsk=bsk, mode=oracle.MODE_KARATSUBA, lut_idx=lut_idx, in_idx=in_idx,
                              out_idx=out_idx)
    assert np.array_equal(B.to_host(out), ref)


@pytest.mark.parametrize("chunk", [None, "3"])
@pytest.mark.parametrize("batch", [1, 2, 7])
def test_generic_coop_kernel(B, oracle, torch_cuda, batch, chunk, monkeypatch):
    """N = 8192 on gen_coop_kernel (one ciphertext on two workgroups that hand spectra halves to each
    other through L2 every CMUX step, round 5): odd and single-ciphertext batches, several chunks
    (CONCRETE_HIP_GEN_CHUNK=3: the flags re-zeroed per launch), permuted rows and mapped LUTs; bit-exact
    vs the exact oracle and equal to the two-launch path (CONCRETE_HIP_GEN_COOP=0) on the same inputs."""
    label, k, N, n, l, logB, width = CASES[6]
    assert N == 8192
    p, lwe_sk, glwe_sk, bsk, fbsk = setup(B, torch_cuda, k, N, n, l, logB, 7750 + batch)
    rng = np.random.RandomState(13 + batch)
    tables = [rng.randint(0, 1 << width, size=1 << width).astype(np.uint64) for _ in range(2)]
    luts = np.stack([B.trivial_glwe(p, B.expand_lut(t, p.N, width)) for t in tables])
    msgs = rng.randint(0, 1 << width, size=batch)
    cts = B.lwe_encrypt(lwe_sk, [B.encode(m, width) for m in msgs], p.n, 2.0 ** -30, 7753 + batch)
    in_idx = rng.permutation(batch).astype(np.uint64)
    out_idx = rng.permutation(batch).astype(np.uint64)
    lut_idx = rng.randint(0, 2, size=batch).astype(np.uint64)
    dev = "cuda:0"
    d = {name: B.to_device(a, dev) for name, a in (("in_idx", in_idx), ("out_idx", out_idx), ("lut_idx", lut_idx))}
    if chunk:
        monkeypatch.setenv("CONCRETE_HIP_GEN_CHUNK", chunk)
    outs = []
    for coop in ("1", "0"):
        monkeypatch.setenv("CONCRETE_HIP_GEN_COOP", coop)
        out = torch_cuda.zeros((batch, p.lwe_out_size), dtype=torch_cuda.int64, device=dev)
        r = torch_cuda.zeros(1, dtype=torch_cuda.int64, device=dev)
        B.pbs(p, fbsk, B.to_device(cts, dev), B.to_device(luts, dev), out=out, resid=r, **d)
        torch_cuda.cuda.synchronize()
        outs.append(B.to_host(out))
        resid = float(np.array([r.item()], dtype=np.int64).view(np.float64)[0])
        kind, limbs, bits = B.bsk_format(p)
        bound = oracle.generic_error_bound(p.k, p.N, p.level, p.base_log, bits, B.to_host(fbsk).view(np.float64))
        assert resid < bound < 0.5, (coop, resid, bound)
    assert B.device_status() == 0
    op = oracle.Params(n=p.n, k=p.k, N=p.N, l=p.level, logB=p.base_log)
    ref, _ = oracle.pbs_batch(op, cts, luts, bsk=bsk, mode=oracle.MODE_KARATSUBA, lut_idx=lut_idx, in_idx=in_idx,
                              out_idx=out_idx)
    assert np.array_equal(outs[0], ref), "coop kernel differs from the exact oracle"
    assert np.array_equal(outs[1], ref), "two-launch path differs from the exact oracle"


def test_generic_coop_kernel_under_load_and_bounded_waits(B, oracle, torch_cuda):
    """gen_coop_kernel's hand-offs (cdna_hip_programming.md §6 G16: test under uneven load) while a
    second stream streams 1 GB copies across the chip: bit-exact vs the oracle and no timeout; then
    with the spin bound forced to one poll for this thread's launches, the call's stream reports the
    timeout (-4) instead of hanging, and the device is clean afterwards."""
    torch = torch_cuda
    label, k, N, n, l, logB, width = CASES[6]
    p, lwe_sk, glwe_sk, bsk, fbsk = setup(B, torch, k, N, n, l, logB, 7780)
    rng = np.random.RandomState(17)
    table = rng.randint(0, 1 << width, size=1 << width).astype(np.uint64)
    msgs = rng.randint(0, 1 << width, size=96)
    cts = B.lwe_encrypt(lwe_sk, [B.encode(m, width) for m in msgs], p.n, 2.0 ** -30, 7783)
    acc = B.trivial_glwe(p, B.expand_lut(table, p.N, width))
    dev = "cuda:0"
    d_in, d_acc = B.to_device(cts, dev), B.to_device(acc[None, :], dev)
    src = torch.empty(1 << 27, dtype=torch.float64, device=dev)
    dst = torch.empty_like(src)
    side, main = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    assert B.device_status(dev) == 0
    with torch.cuda.stream(side):
        for _ in range(24):
            dst.copy_(src)
    with torch.cuda.stream(main):
        out = B.pbs(p, fbsk, d_in, d_acc)
        assert B.stream_status(dev, main) == 0
    torch.cuda.synchronize()
    rows = np.array([0, 47, 95])
    op = oracle.Params(n=p.n, k=p.k, N=p.N, l=p.level, logB=p.base_log)
    ref, _ = oracle.pbs_batch(op, cts[rows], acc[None, :], bsk=bsk, mode=oracle.MODE_KARATSUBA)
    got = B.to_host(out)
    assert np.array_equal(got[rows], ref)
    dec = B.lwe_decrypt(glwe_sk, got, p.big_n)
    assert [B.decode(d, width) for d in dec] == [int(table[m]) for m in msgs]
    try:
        B.set_thread_spin_limit(1)
        with torch.cuda.stream(main):
            B.pbs(p, fbsk, d_in, d_acc)
            st = B.stream_status(dev, main)
    finally:
        B.set_thread_spin_limit(0)
    assert st == -4, st
    assert B.device_status(dev) == 0


@pytest.mark.parametrize("ci", [5, 6, 7], ids=[CASES[i][0] for i in (5, 6, 7)])
def test_generic_edge_inputs(B, oracle, torch_cuda, ci):
    """test_gpu_pbs.py::test_pbs_edge_inputs on the large-N paths (N = 4096 one launch, N = 8192 two
    workgroups per ciphertext, N = 16384 two launches): zero mask elements (tfhe's skip rule), mask
    elements whose modulus switch is 0 but which are not 0, values just below a modulus-switch rounding
    boundary, a body that rounds up to 2N, ms = N (negation), all-zero and all-ones ciphertexts;
    bit-exact vs the oracle's Karatsuba product."""
    label, k, N, n, l, logB, width = CASES[ci]
    p, lwe_sk, glwe_sk, bsk, fbsk = setup(B, torch_cuda, k, N, n, l, logB, 7800 + ci)
    rng = np.random.RandomState(23)
    table = rng.randint(0, 1 << width, size=1 << width).astype(np.uint64)
    msgs = rng.randint(0, 1 << width, size=8)
    cts = B.lwe_encrypt(lwe_sk, [B.encode(m, width) for m in msgs], p.n, 2.0 ** -30, 7803 + ci)
    log2_2n = (2 * N).bit_length() - 1
    cts[0, : p.n // 2] = 0
    cts[1, :] = 0
    cts[2, :] = np.uint64(0xFFFFFFFFFFFFFFFF)
    cts[3, : p.n] = np.uint64(1)                                      # ms(1) == 0 but a_i != 0
    cts[4, : p.n] = np.uint64((1 << (63 - log2_2n)) - 1)              # just below a rounding boundary
    cts[5, p.n] = np.uint64(0xFFFFFFFFFFFFFFFF - 5)                   # body rounds up to 2N
    cts[6, : p.n] = np.uint64(1 << 63)                                # ms = N (negation)
    acc = B.trivial_glwe(p, B.expand_lut(table, p.N, width))
    out = B.pbs(p, fbsk, B.to_device(cts, "cuda:0"), B.to_device(acc[None, :], "cuda:0"))
    torch_cuda.cuda.synchronize()
    op = oracle.Params(n=p.n, k=p.k, N=p.N, l=p.level, logB=p.base_log)
    ref, _ = oracle.pbs_batch(op, cts, acc[None, :], bsk=bsk, mode=oracle.MODE_KARATSUBA)
    assert np.array_equal(B.to_host(out), ref)


def test_generic_outside_exact_range_refused(B):
    """Sets whose certified bound would exceed the gate are refused, not rounded wrongly."""
    assert not B.pbs_supported(B.PbsParams(n=8, k=1, N=131072, level=2, base_log=15))
    assert not B.pbs_supported(B.PbsParams(n=8, k=1, N=4096, level=1, base_log=40))


@pytest.mark.parametrize("bits", [4, 6])
def test_keyswitch_optimizer_rows(B, oracle, torch_cuda, bits):
    """Batched keyswitch kN -> n at the optimizer rows' sizes (n up to 880 + 1 output words),
    bit-exact vs the oracle (keyswitch.rs:185-223 semantics)."""
    p = B.OPTIMIZER_SETS[bits]
    glwe_sk = B.binary_key(p.big_n, 7300 + bits)
    lwe_sk = B.binary_key(p.n, 7310 + bits)
    ksk = B.ksk_generate(p, glwe_sk, lwe_sk, 7320 + bits)
    rng = np.random.RandomState(bits)
    cts = rng.randint(0, 2 ** 63, size=(9, p.big_n + 1), dtype=np.int64).astype(np.uint64) * np.uint64(2) + \
        np.uint64(1)
    dev = "cuda:0"
    out = B.keyswitch(p, B.to_device(ksk, dev), B.to_device(cts, dev))
    torch_cuda.cuda.synchronize()
    op = oracle.Params(n=p.n, k=p.k, N=p.N, l=p.level, logB=p.base_log, ks_l=p.ks_level, ks_logB=p.ks_base_log)
    assert np.array_equal(B.to_host(out), oracle.keyswitch_batch(op, cts, ksk))


@pytest.mark.parametrize("bits", list(range(1, 9)))
def test_reference_fixtures_at_optimizer_rows(B, torch_cuda, bits):
    """The reference generators' cleartext vectors (tests/golden/reference_lut_fixtures.json,
    apply_lookup_table / linalg_apply_lookup_table, every signedness variant) of width p, run at
    the optimizer's own p-bit row (full n, secure noise; v0_last_128) as one mapped-LUT batch:
    every output decodes to the reference's expected value.  p = 5 runs on the N = 2048 kernel,
    the others on the general path."""
    import json
    import math
    import os
    golden = os.path.join(os.path.dirname(__file__), "golden", "reference_lut_fixtures.json")
    fx = json.load(open(golden))
    cases = [c for c in fx["apply_lookup_table"] + fx["linalg_apply_lookup_table"]
             if int(math.log2(len(c["lut"]))) == bits and not c["description"].endswith("_2layer")]
    assert len(cases) >= 15
    p = B.OPTIMIZER_SETS[bits]
    assert B.pbs_supported(p)
    lwe_sk = B.binary_key(p.n, 7400 + bits)
    glwe_sk = B.binary_key(p.big_n, 7410 + bits)
    fbsk = B.convert_bsk(p, B.bsk_generate(p, lwe_sk, glwe_sk, 7420 + bits), "cuda:0")
    pts, lut_idx, expect, luts = [], [], [], []
    for ci, c in enumerate(cases):
        table = np.array(c["lut"], dtype=np.int64).view(np.uint64)
        luts.append(B.trivial_glwe(p, B.expand_lut(table, p.N, bits, c["input_signed"])))
        for x, e in zip(c["input"], c["expected"]):
            pt = int(B.encode(int(x) & ((1 << 64) - 1), bits))
            if c["input_signed"]:  # FHEToTFHEScalar.cpp:373-413: offset 2^(p-1) on the body
                pt = (pt + int(B.encode(1 << (bits - 1), bits))) & ((1 << 64) - 1)
            pts.append(pt)
            lut_idx.append(ci)
            expect.append((e, c["output_signed"]))
    cts = B.lwe_encrypt(lwe_sk, pts, p.n, B.secure_std(1, p.n), 7430 + bits)
    dev = "cuda:0"
    out = B.pbs(p, fbsk, B.to_device(cts, dev), B.to_device(np.stack(luts), dev),
                lut_idx=B.to_device(np.array(lut_idx, dtype=np.uint64), dev))
    torch_cuda.cuda.synchronize()
    dec = B.lwe_decrypt(glwe_sk, B.to_host(out), p.big_n)
    assert [B.decode(d, bits, s) for d, (_, s) in zip(dec, expect)] == [e for e, _ in expect]


def test_configs4_atomic_pattern_8bit(B, oracle, torch_cuda):
    """BASELINE configs[4] (an 8-bit fhe.LookupTable) as the compiler lowers it
    (FHEToTFHEScalar.cpp:373-437: encode/expand the LUT, keyswitch, bootstrap) at the optimizer's
    8-bit row (v0_last_128: k = 1, N = 16384, n = 1006, br 2/15, ks 5/4), full sizes and secure
    noise, on the reference's 8-bit fixtures (every signedness variant): the LUTs are encoded on
    the device (concrete_hip_encode_expand_lut_device), the keyswitch kN = 16384 -> n = 1006 is
    bit-exact vs the oracle, and every bootstrapped output decodes to the reference's expected
    value."""
    import json
    import os
    from concrete_amd import _native
    L = _native.lib()
    golden = os.path.join(os.path.dirname(__file__), "golden", "reference_lut_fixtures.json")
    fx = json.load(open(golden))
    cases = [c for c in fx["apply_lookup_table"] + fx["linalg_apply_lookup_table"]
             if len(c["lut"]) == 256 and not c["description"].endswith("_2layer")]
    p = B.OPTIMIZER_SETS[8]
    bits = 8
    lwe_sk = B.binary_key(p.n, 7800)
    glwe_sk = B.binary_key(p.big_n, 7801)
    bsk = B.bsk_generate(p, lwe_sk, glwe_sk, 7802)
    fbsk = B.convert_bsk(p, bsk, "cuda:0")
    ksk = B.ksk_generate(p, glwe_sk, lwe_sk, 7803)
    pts, lut_idx, expect, tables, signs = [], [], [], [], []
    for ci, c in enumerate(cases):
        tables.append(np.array(c["lut"], dtype=np.int64).view(np.uint64))
        signs.append(bool(c["input_signed"]))
        for x, e in zip(c["input"], c["expected"]):
            pt = int(B.encode(int(x) & ((1 << 64) - 1), bits))
            if c["input_signed"]:  # FHEToTFHEScalar.cpp:373-413: offset 2^(p-1) on the body
                pt = (pt + int(B.encode(1 << (bits - 1), bits))) & ((1 << 64) - 1)
            pts.append(pt)
            lut_idx.append(ci)
            expect.append((e, c["output_signed"]))
    # the client encrypts under the big (GLWE-derived) LWE key: the TLU starts with the keyswitch
    cts = B.lwe_encrypt(glwe_sk, pts, p.big_n, B.secure_std(p.k, p.N), 7804)
    dev = "cuda:0"
    s = torch_cuda.cuda.current_stream().cuda_stream
    # LUT encoding on the device, signed and unsigned tables as two batched calls
    d_tab = B.to_device(np.stack(tables), dev)
    d_lut = torch_cuda.empty((len(cases), p.N), dtype=torch_cuda.int64, device=dev)
    for signed in (False, True):
        for ci in [i for i, sg in enumerate(signs) if sg == signed]:
            assert L.concrete_hip_encode_expand_lut_device(s, 0, d_lut[ci].data_ptr(), p.N, d_tab[ci].data_ptr(),
                                                           256, 1, bits, int(signed)) == 0
    d_acc = torch_cuda.empty((len(cases), p.glwe_size), dtype=torch_cuda.int64, device=dev)
    assert L.concrete_hip_build_accumulators(s, 0, d_acc.data_ptr(), d_lut.data_ptr(), len(cases), p.k, p.N) == 0
    kb = B.RuntimeBuffer(ksk)
    try:
        d_small = B.keyswitch(p, kb, B.to_device(cts, dev))
        out = B.pbs(p, fbsk, d_small, d_acc, lut_idx=B.to_device(np.array(lut_idx, dtype=np.uint64), dev))
        torch_cuda.cuda.synchronize()
    finally:
        kb.free()
    op = oracle.Params(n=p.n, k=p.k, N=p.N, l=p.level, logB=p.base_log, ks_l=p.ks_level, ks_logB=p.ks_base_log)
    assert np.array_equal(B.to_host(d_small), oracle.keyswitch_batch(op, cts, ksk))
    host_luts = np.stack([B.expand_lut(t, p.N, bits, sg) for t, sg in zip(tables, signs)])
    assert np.array_equal(B.to_host(d_lut), host_luts)
    dec = B.lwe_decrypt(glwe_sk, B.to_host(out), p.big_n)
    assert [B.decode(d, bits, sg) for d, (_, sg) in zip(dec, expect)] == [e for e, _ in expect]
    # a full-size row bit-exact in the driver-run suite — the oracle's pure-integer
    # Karatsuba product over all n = 1006 CMUX steps (its eight products per step on the OpenMP
    # threads), on the keyswitched input and the device-encoded accumulator of that row
    row = len(pts) // 2
    ref, _ = oracle.pbs_batch(op, B.to_host(d_small)[row:row + 1], B.to_host(d_acc)[lut_idx[row]][None, :], bsk=bsk,
                              mode=oracle.MODE_KARATSUBA)
    assert np.array_equal(B.to_host(out)[row:row + 1], ref)


# the large-N paths at many CMUX steps and many ciphertexts, bit-exact vs the
# oracle's Karatsuba product (the table rows' k, N, l, logB; n cut to what the oracle finishes in
# seconds): N = 4096 (the one-launch kernel), N = 8192 (one ciphertext on two workgroups, round 5),
# N = 2^15 (a polynomial spread over two workgroups).  (label, k, N, n, l, logB, bits, batch)
LARGE_N_CASES = [
    ("6bit_k1_N4096_n64", 1, 4096, 64, 1, 22, 6, 67),
    ("7bit_k1_N8192_n64", 1, 8192, 64, 1, 22, 7, 67),
    ("8bit_k1_N16384_n24", 1, 16384, 24, 2, 15, 8, 9),
    ("9bit_k1_N32768_n16", 1, 32768, 16, 2, 15, 9, 6),
]


@pytest.mark.parametrize("case", LARGE_N_CASES, ids=[c[0] for c in LARGE_N_CASES])
def test_large_n_many_steps_bit_exact(B, oracle, torch_cuda, case):
    label, k, N, n, l, logB, width, batch = case
    p, glwe_sk, bsk, fbsk, cts, acc, table, msgs, got, resid = run_case(
        B, oracle, torch_cuda, (label, k, N, n, l, logB, width), 7900 + n, batch=batch)
    op = oracle.Params(n=p.n, k=p.k, N=p.N, l=p.level, logB=p.base_log)
    ref, _ = oracle.pbs_batch(op, cts, acc[None, :], bsk=bsk, mode=oracle.MODE_KARATSUBA)
    assert np.array_equal(got, ref), f"{label}: GPU differs from the exact oracle"
    kind, limbs, bits = B.bsk_format(p)
    bound = oracle.generic_error_bound(p.k, p.N, p.level, p.base_log, bits, B.to_host(fbsk).view(np.float64))
    assert resid < bound < 0.5, (resid, bound)
    dec = B.lwe_decrypt(glwe_sk, got, p.big_n)
    assert [B.decode(d, width) for d in dec] == [int(table[m]) for m in msgs]


# v0_last_128 rows at non-zero log norm2 (tests/golden/v0_last_128_rows.json): per width the row
# with the most decomposition levels (the caps lifted in round 4: many-level keys, (k + 1) l T
# product terms past the register-tiled products), plus the 8-bit log-norm2-17 row (14 levels of
# 3 bits).  (label, k, N, n reduced, l, logB, message bits, full n, ks_l, ks_logB)
LN2_CASES = [
    ("1bit_ln2_30", 4, 512, 8, 22, 2, 1, 625, 12, 1),
    ("2bit_ln2_29", 4, 512, 6, 44, 1, 2, 629, 12, 1),
    ("3bit_ln2_27", 4, 512, 8, 22, 2, 3, 690, 7, 2),
    ("4bit_ln2_26", 2, 1024, 6, 44, 1, 4, 727, 14, 1),
    ("5bit_ln2_24", 1, 2048, 6, 22, 2, 5, 806, 8, 2),
    ("6bit_ln2_22", 1, 4096, 4, 42, 1, 6, 833, 17, 1),
    ("7bit_ln2_20", 1, 8192, 3, 42, 1, 7, 898, 18, 1),
    ("8bit_ln2_17", 1, 16384, 2, 14, 3, 8, 1007, 11, 2),
    ("8bit_ln2_18", 1, 16384, 2, 41, 1, 8, 985, 21, 1),
    ("9bit_ln2_16", 1, 32768, 1, 41, 1, 9, 1059, 23, 1),
    ("10bit_ln2_13", 1, 65536, 1, 20, 2, 10, 1095, 12, 2),
]


@pytest.mark.parametrize("case", LN2_CASES, ids=[c[0] for c in LN2_CASES])
def test_optimizer_rows_at_nonzero_log_norm2(B, oracle, torch_cuda, case):
    """PBS bit-exact vs the exact oracle (n reduced) and the row's keyswitch into its full n
    bit-exact, at optimizer rows whose decompositions have up to 44 levels."""
    label, k, N, n, l, logB, width, n_full, ks_l, ks_logB = case
    p, glwe_sk, bsk, fbsk, cts, acc, table, msgs, got, resid = run_case(
        B, oracle, torch_cuda, (label, k, N, n, l, logB, width), 7600, batch=4)
    op = oracle.Params(n=p.n, k=p.k, N=p.N, l=p.level, logB=p.base_log)
    ref, _ = oracle.pbs_batch(op, cts, acc[None, :], bsk=bsk, mode=oracle.MODE_KARATSUBA)
    assert np.array_equal(got, ref), f"{label}: GPU differs from the exact oracle"
    assert resid < 0.5
    dec = B.lwe_decrypt(glwe_sk, got, p.big_n)
    assert [B.decode(d, width) for d in dec] == [int(table[m]) for m in msgs]
    # the row's keyswitch (ks_l, ks_logB) into the row's full n, from up to 4096 input words (the
    # 8-bit row's whole 16384 x 21 x 986-word key would be 2.7 GB)
    kN = min(k * N, 4096)
    pk = B.PbsParams(n=n_full, k=1, N=kN, level=l, base_log=logB, ks_level=ks_l, ks_base_log=ks_logB)
    lwe_sk = B.binary_key(n_full, 7610)
    ksk = B.ksk_generate(pk, B.binary_key(kN, 7611), lwe_sk, 7620)
    rng = np.random.RandomState(ks_l)
    big = rng.randint(0, 2 ** 63, size=(5, pk.big_n + 1), dtype=np.int64).astype(np.uint64) * np.uint64(2) + \
        np.uint64(1)
    out = B.keyswitch(pk, B.to_device(ksk, "cuda:0"), B.to_device(big, "cuda:0"))
    torch_cuda.cuda.synchronize()
    opk = oracle.Params(n=n_full, k=1, N=kN, l=l, logB=logB, ks_l=ks_l, ks_logB=ks_logB)
    assert np.array_equal(B.to_host(out), oracle.keyswitch_batch(opk, big, ksk))


@pytest.mark.parametrize("ci", [0, 2, 3], ids=[CASES[i][0] for i in (0, 2, 3)])
def test_generic_tile_kernels_on_the_general_format_key(B, oracle, torch_cuda, ci):
    """The one-launch tile kernels (gen_tile_kernel) run the log-norm2-0 shapes of N = 256 / 512 /
    1024 on the general-format key (concrete_hip_convert_bsk_generic + concrete_hip_pbs_generic:
    a caller-converted key, or the companion key of a wide-digit call), 67 ciphertexts; bit-exact
    vs the exact oracle."""
    from concrete_amd import _native
    label, k, N, n, l, logB, width = CASES[ci]
    L = _native.lib()
    p = B.PbsParams(n=4, k=k, N=N, level=l, base_log=logB)
    lwe_sk, glwe_sk = B.binary_key(p.n, 7800), B.binary_key(p.big_n, 7801)
    bsk = B.bsk_generate(p, lwe_sk, glwe_sk, 7802)
    rng = np.random.RandomState(ci)
    table = rng.randint(0, 1 << width, size=1 << width).astype(np.uint64)
    msgs = rng.randint(0, 1 << width, size=67)
    cts = B.lwe_encrypt(lwe_sk, [B.encode(m, width) for m in msgs], p.n, 2.0 ** -30, 7803)
    acc = B.trivial_glwe(p, B.expand_lut(table, p.N, width))
    dev = "cuda:0"
    g = torch_cuda.empty(L.concrete_hip_generic_bsk_size_bytes(p.n, p.k, p.level, p.N) // 8, dtype=torch_cuda.int64,
                         device=dev)
    st, gi = B._stream(torch_cuda.device(dev)), B._gpu_index(torch_cuda.device(dev))
    _native.check(L.concrete_hip_convert_bsk_generic(st, gi, B._ptr(g), bsk.ctypes.data, 0, p.n, p.k, p.level, p.N),
                  "convert_bsk_generic")
    d_in, d_acc = B.to_device(cts, dev), B.to_device(acc[None, :], dev)
    out = torch_cuda.zeros((67, p.lwe_out_size), dtype=torch_cuda.int64, device=dev)
    _native.check(L.concrete_hip_pbs_generic(st, gi, B._ptr(out), None, B._ptr(d_acc), None, B._ptr(d_in), None,
                                             B._ptr(g), p.n, p.k, p.N, p.base_log, p.level, 67, None), "pbs_generic")
    torch_cuda.cuda.synchronize()
    op = oracle.Params(n=p.n, k=p.k, N=p.N, l=p.level, logB=p.base_log)
    ref, _ = oracle.pbs_batch(op, cts, acc[None, :], bsk=bsk, mode=oracle.MODE_KARATSUBA)
    assert np.array_equal(B.to_host(out), ref)
