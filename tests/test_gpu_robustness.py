"""GPU tests of two robustness properties of the backend (round 6):

* status slots are recycled when a stream is destroyed, so a caller that creates and destroys a
  stream per call — the reference's memref wrappers do (compiler lib/Runtime/wrappers.cpp:129/160,
  185/255) — keeps per-stream failure attribution past 4,096 streams, and a stream that overflows
  the slab still reads the word its launches write;
* the exactness gate is evaluated with the converted key's own spectrum (concrete_amd/csrc/
  keycheck.hip): a crafted key whose limb spectra are far larger than a random key's is refused
  at the digit widths where its certified rounding bound reaches 1/2, and still runs bit-exactly
  where the bound holds.
"""
from dataclasses import replace

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def env():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a visible MI355X"
    from concrete_amd import _native
    from concrete_amd import backend as B
    from concrete_amd import runtime as R
    from oracle import pyoracle as O
    return dict(torch=torch, L=_native.lib(), B=B, R=R, O=O)


def _oparams(O, p):
    return O.Params(n=p.n, k=p.k, N=p.N, l=p.level, logB=p.base_log, ks_l=p.ks_level, ks_logB=p.ks_base_log)


def _setup(env, p, seed, bsk_std=None):
    B, O, torch = env["B"], env["O"], env["torch"]
    lwe_sk = B.binary_key(p.n, seed)
    glwe_sk = B.binary_key(p.big_n, seed + 1)
    bsk = B.bsk_generate(p, lwe_sk, glwe_sk, seed + 2, std=bsk_std)
    fbsk = B.convert_bsk(p, bsk, "cuda:0")
    torch.cuda.synchronize()
    width = 3
    table = np.array([3, 0, 6, 1, 7, 2, 5, 4], dtype=np.uint64)
    acc = B.trivial_glwe(p, B.expand_lut(table, p.N, width))
    return dict(p=p, op=_oparams(O, p), lwe_sk=lwe_sk, glwe_sk=glwe_sk, bsk=bsk, fbsk=fbsk, acc=acc, width=width,
                table=table)


def _encrypt(env, S, msgs, seed):
    """Secure LWE noise at cfg2's n; the reduced-n setups (n < 100, where the secure std is near the
    torus itself) use 2^-25, as the other reduced-n tests do — bit-exactness does not depend on it."""
    B = env["B"]
    n = S["p"].n
    return B.lwe_encrypt(S["lwe_sk"], [B.encode(m, S["width"]) for m in msgs], n,
                         B.secure_std(1, n) if n >= 100 else 2.0 ** -25, seed)


def _pbs_raw(env, S, stream, d_out, d_acc, d_in, nb):
    """concrete_hip_pbs on a raw stream handle (the cuda_* streams are not torch's)."""
    p = S["p"]
    return env["L"].concrete_hip_pbs(stream, 0, d_out.data_ptr(), None, d_acc.data_ptr(), None, d_in.data_ptr(),
                                     None, S["fbsk"].data_ptr(), p.n, p.k, p.N, p.base_log, p.level, nb, None)


def test_status_slots_recycled_past_the_slab(env):
    """More than 4,096 streams created and destroyed through cuda_create_stream /
    cuda_destroy_stream, each running one PBS (as the reference's direct route does per call):
    every stream's slot goes back to the free list, so afterwards two live streams still get
    words of their own — one forced to its spin bound reports -4, the other 0 and bit-exact."""
    import threading
    B, L, torch = env["B"], env["L"], env["torch"]
    S = _setup(env, replace(B.CFG2, n=8), 5100)
    dev = "cuda:0"
    assert B.device_status(dev) == 0
    base = L.concrete_hip_status_slots_in_use(0)
    rng = np.random.RandomState(51)
    msgs = rng.randint(0, 8, size=1)
    d_in = B.to_device(_encrypt(env, S, msgs, 5101), dev)
    d_acc = B.to_device(S["acc"][None, :], dev)
    d_out = torch.zeros((1, S["p"].lwe_out_size), dtype=torch.int64, device=dev)
    torch.cuda.synchronize()
    peak = 0
    for i in range(4200):
        s = L.cuda_create_stream(0)
        assert _pbs_raw(env, S, s, d_out, d_acc, d_in, 1) == 0
        assert L.concrete_hip_stream_status(s, 0) == 0
        peak = max(peak, L.concrete_hip_status_slots_in_use(0))
        L.cuda_destroy_stream(s, 0)
    assert peak == base + 1, (base, peak)
    assert L.concrete_hip_status_slots_in_use(0) == base
    dec = B.lwe_decrypt(S["glwe_sk"], B.to_host(d_out), S["p"].big_n)
    assert B.decode(dec[0], S["width"]) == int(S["table"][msgs[0]])

    # two live streams after the churn: attribution still per stream (cfg2's n, the batch of the
    # round-5 per-stream test, whose syncs a one-poll bound reliably trips)
    C2 = _setup(env, B.CFG2, 5200)
    msgs2 = rng.randint(0, 8, size=(2, 512))
    d_in2 = [B.to_device(_encrypt(env, C2, msgs2[i], 5210 + i), dev) for i in range(2)]
    d_acc2 = B.to_device(C2["acc"][None, :], dev)
    outs = [torch.zeros((512, C2["p"].lwe_out_size), dtype=torch.int64, device=dev) for _ in range(2)]
    torch.cuda.synchronize()
    streams = [L.cuda_create_stream(0) for _ in range(2)]
    status = [None, None]
    gate = threading.Barrier(2)

    def call(i):
        try:
            if i == 0:
                B.set_thread_spin_limit(1)
            gate.wait()
            assert _pbs_raw(env, C2, streams[i], outs[i], d_acc2, d_in2[i], 512) == 0
            status[i] = L.concrete_hip_stream_status(streams[i], 0)
        finally:
            B.set_thread_spin_limit(0)

    th = [threading.Thread(target=call, args=(i,)) for i in range(2)]
    [t.start() for t in th]
    [t.join() for t in th]
    for s in streams:
        L.cuda_destroy_stream(s, 0)
    assert status == [-4, 0], status
    assert B.device_status(dev) == 0
    assert L.concrete_hip_status_slots_in_use(0) == base
    got = B.to_host(outs[1])
    dec = B.lwe_decrypt(C2["glwe_sk"], got, C2["p"].big_n)
    assert [B.decode(d, C2["width"]) for d in dec] == [int(C2["table"][m]) for m in msgs2[1]]


def test_status_overflow_stream_reads_its_word(env):
    """With the slab capped (test hook) a second stream overflows onto the shared slot 0; its
    own status read still reports its launch's timeout (-4) — round 5 read nothing for an unmapped
    stream and returned 0 — while the stream holding a slot of its own reports 0."""
    B, L, torch = env["B"], env["L"], env["torch"]
    C2 = _setup(env, B.CFG2, 5300)
    dev = "cuda:0"
    assert B.device_status(dev) == 0
    base = L.concrete_hip_status_slots_in_use(0)
    rng = np.random.RandomState(53)
    msgs = rng.randint(0, 8, size=(2, 512))
    d_in = [B.to_device(_encrypt(env, C2, msgs[i], 5310 + i), dev) for i in range(2)]
    d_acc = B.to_device(C2["acc"][None, :], dev)
    outs = [torch.zeros((512, C2["p"].lwe_out_size), dtype=torch.int64, device=dev) for _ in range(2)]
    torch.cuda.synchronize()
    L.concrete_hip_set_status_slot_cap(base + 2)  # slot 0 + the slots in use + one more
    streams = [L.cuda_create_stream(0) for _ in range(2)]
    try:
        assert _pbs_raw(env, C2, streams[0], outs[0], d_acc, d_in[0], 512) == 0  # takes the last free slot
        assert L.concrete_hip_status_slots_in_use(0) == base + 1
        B.set_thread_spin_limit(1)
        try:
            assert _pbs_raw(env, C2, streams[1], outs[1], d_acc, d_in[1], 512) == 0  # overflows onto slot 0
        finally:
            B.set_thread_spin_limit(0)
        assert L.concrete_hip_status_slots_in_use(0) == base + 1
        assert L.concrete_hip_stream_status(streams[1], 0) == -4
        assert L.concrete_hip_stream_status(streams[0], 0) == 0
    finally:
        L.concrete_hip_set_status_slot_cap(0)
        for s in streams:
            L.cuda_destroy_stream(s, 0)
    assert B.device_status(dev) == 0
    assert L.concrete_hip_status_slots_in_use(0) == base
    dec = B.lwe_decrypt(C2["glwe_sk"], B.to_host(outs[0]), C2["p"].big_n)
    assert [B.decode(d, C2["width"]) for d in dec] == [int(C2["table"][m]) for m in msgs[0]]


CRAFTED = 0x5555555555555555  # every coefficient of every GGSW row: limb spectra ~8x a random key's


def _oracle_max_spectrum(O, op, bsk):
    f = O.bsk_to_fourier(op, bsk)
    M = op.N // 2
    g = f.reshape(-1, 2, M)  # the oracle's blocks: M real parts, then M imaginary parts
    return float(np.max(np.hypot(g[:, 0], g[:, 1]))) * M, f


def test_key_spectrum_recorded_and_gate_uses_it(env):
    """A random key and a crafted constant-coefficient key (k = 1, N = 1024, l = 1): the recorded
    max|G| equals the oracle's long-double transform's; the certified bound at logB = 11 (the
    static gate's edge, (k+1) l 2^logB = 4096) is ~0.2 for the random key and > 1/2 for the crafted
    one, whose PBS is then refused (-2, message names the bound), while at logB = 7 the same crafted
    key runs and is bit-exact vs the oracle's integer (Karatsuba) PBS."""
    B, O, L, torch = env["B"], env["O"], env["L"], env["torch"]
    p11 = replace(B.CFG2, n=6, level=1, base_log=11)
    p7 = replace(p11, base_log=7)
    # logB = 11 digits amplify the key noise 2^10 sqrt(2N)-fold: small key noise so that the random
    # key's outputs decrypt (test_gpu_runtime.py::test_wide_digits_on_the_general_path does the same)
    rnd = _setup(env, p11, 5400, bsk_std=2.0 ** -52)
    g_rnd, f_rnd = _oracle_max_spectrum(O, _oparams(O, p11), rnd["bsk"])
    key_rnd = rnd["fbsk"].data_ptr()
    assert abs(L.concrete_hip_key_spectrum_max(key_rnd) / g_rnd - 1.0) < 1e-9
    b_rnd = L.concrete_hip_key_error_bound(key_rnd, 11)
    assert abs(b_rnd / O.fft_error_bound(_oparams(O, p11), f_rnd) - 1.0) < 1e-6
    assert b_rnd < 0.5

    crafted = np.full(p11.bsk_len, CRAFTED, dtype=np.uint64)
    g_cr, f_cr = _oracle_max_spectrum(O, _oparams(O, p11), crafted)
    assert g_cr > 5 * g_rnd
    fk = B.convert_bsk(p11, crafted, "cuda:0")
    torch.cuda.synchronize()
    key = fk.data_ptr()
    assert abs(L.concrete_hip_key_spectrum_max(key) / g_cr - 1.0) < 1e-9
    b11 = L.concrete_hip_key_error_bound(key, 11)
    b7 = L.concrete_hip_key_error_bound(key, 7)
    assert abs(b11 / O.fft_error_bound(_oparams(O, p11), f_cr) - 1.0) < 1e-6
    assert b11 >= 0.5 and b7 < 0.5, (b11, b7)

    rng = np.random.RandomState(54)
    msgs = rng.randint(0, 8, size=5)
    cts = _encrypt(env, rnd, msgs, 5401)
    d_in = B.to_device(cts, "cuda:0")
    d_acc = B.to_device(rnd["acc"][None, :], "cuda:0")
    with pytest.raises(RuntimeError, match="certified rounding bound"):
        B.pbs(p11, fk, d_in, d_acc)
    got = B.to_host(B.pbs(p7, fk, d_in, d_acc))
    torch.cuda.synchronize()
    ref, _ = O.pbs_batch(_oparams(O, p7), cts, rnd["acc"][None, :], bsk=crafted, mode=O.MODE_KARATSUBA)
    assert np.array_equal(got, ref)
    # the random key still runs at the gate's edge
    out = B.pbs(p11, rnd["fbsk"], d_in, d_acc)
    torch.cuda.synchronize()
    dec = B.lwe_decrypt(rnd["glwe_sk"], B.to_host(out), p11.big_n)
    assert [B.decode(d, 3) for d in dec] == [int(rnd["table"][m]) for m in msgs]


def test_crafted_key_falls_back_to_the_general_path(env):
    """The crafted key held by a keyset (which keeps its standard key): at logB = 11 the hand-tuned
    kernel's bound fails, so the call runs on the general-format companion when that format's own
    measured bound holds — bit-exact vs the oracle's integer PBS — and is refused otherwise; the
    companion's bound is read from a caller-converted general-format copy of the same key."""
    B, R, O, L, torch = env["B"], env["R"], env["O"], env["L"], env["torch"]
    p = replace(B.CFG2, n=6, level=1, base_log=11)
    crafted = np.full(p.bsk_len, CRAFTED, dtype=np.uint64)
    gbytes = L.concrete_hip_generic_bsk_size_bytes(p.n, p.k, p.level, p.N)
    gk = torch.empty(gbytes // 8, dtype=torch.int64, device="cuda:0")
    s = torch.cuda.current_stream().cuda_stream
    from concrete_amd import _native
    _native.check(L.concrete_hip_convert_bsk_generic(s, 0, gk.data_ptr(), crafted.ctypes.data, 0, p.n, p.k, p.level,
                                                     p.N), "convert_bsk_generic")
    torch.cuda.synchronize()
    gen_bound = L.concrete_hip_key_error_bound(gk.data_ptr(), p.base_log)
    assert gen_bound > 0
    lwe_sk = B.binary_key(p.n, 5500)
    width = 3
    table = np.array([1, 6, 3, 0, 5, 2, 7, 4], dtype=np.uint64)
    tlu = B.expand_lut(table, p.N, width)
    msgs = np.random.RandomState(55).randint(0, 8, size=7)
    cts = B.lwe_encrypt(lwe_sk, [B.encode(m, width) for m in msgs], p.n, 2.0 ** -25, 5501)
    ks = R.Keyset([0])
    ks.add_bsk(0, crafted, p)
    try:
        if gen_bound < 0.5:
            got = R.batched_bootstrap(ks, p, cts, tlu)
            ref, _ = O.pbs_batch(_oparams(O, p), cts, B.trivial_glwe(p, tlu)[None, :], bsk=crafted,
                                 mode=O.MODE_KARATSUBA)
            assert np.array_equal(got, ref)
        else:
            # the keyset route aborts on a refused call (rt_die): check through the caller-held key
            d_in = B.to_device(cts, "cuda:0")
            d_acc = B.to_device(B.trivial_glwe(p, tlu)[None, :], "cuda:0")
            out = torch.zeros((len(cts), p.lwe_out_size), dtype=torch.int64, device="cuda:0")
            rc = L.concrete_hip_pbs_generic(s, 0, out.data_ptr(), None, d_acc.data_ptr(), None, d_in.data_ptr(), None,
                                            gk.data_ptr(), p.n, p.k, p.N, p.base_log, p.level, len(cts), None)
            assert rc == -2
    finally:
        ks.close()


@pytest.mark.parametrize("shape", [
    # (k, N, l, logB): one key format each (concrete_hip_bsk_format codes 1, 2, 4, 5, 3)
    (1, 1024, 3, 7),    # N1024: oracle ora_fft_error_bound
    (1, 2048, 1, 23),   # N2048: pyoracle.gpu2048_error_bound
    (2, 1024, 1, 23),   # K2N1024: pyoracle.gpu1024k2_error_bound
    (3, 512, 1, 18),    # SMALL: pyoracle.gpu_small_error_bound
    (1, 4096, 1, 22),   # GENERIC: pyoracle.generic_error_bound
], ids=["N1024", "N2048", "K2N1024", "SMALL", "GENERIC"])
def test_key_bound_matches_the_oracle_per_format(env, shape):
    """The gate's bound (keycheck.hip:certified_bound with the max|G| the conversion kernels
    recorded, times each format's stored scale) equals the bound the GPU tests certify residuals
    against (oracle/pyoracle.py, computed from the device key itself), for a random key of every key
    format — so the per-call check refuses exactly where the tests' certificate would fail."""
    import ctypes as C
    B, O, L, torch = env["B"], env["O"], env["L"], env["torch"]
    k, N, lv, logB = shape
    p = B.PbsParams(n=2, k=k, N=N, level=lv, base_log=logB, ks_level=1, ks_base_log=1)
    lwe_sk, glwe_sk = B.binary_key(p.n, 7700 + N), B.binary_key(p.big_n, 7701 + N)
    bsk = B.bsk_generate(p, lwe_sk, glwe_sk, 7702 + N)
    fk = B.convert_bsk(p, bsk, "cuda:0")
    torch.cuda.synchronize()
    got = L.concrete_hip_key_error_bound(fk.data_ptr(), logB)
    view = B.to_host(fk).view(np.float64)
    limbs, bits = C.c_uint32(), C.c_uint32()
    code = L.concrete_hip_bsk_format(k, N, lv, C.byref(limbs), C.byref(bits))
    if code == 1:
        op = O.Params(n=p.n, k=k, N=N, l=lv, logB=logB)
        want = O.fft_error_bound(op, O.bsk_to_fourier(op, bsk))
    elif code == 2:
        want = O.gpu2048_error_bound(view, logB, lv)
    elif code == 4:
        want = O.gpu1024k2_error_bound(view, logB, lv)
    elif code == 5:
        want = O.gpu_small_error_bound(view, N, k, logB, lv)
    else:
        assert code == 3
        want = O.generic_error_bound(k, N, lv, logB, bits.value, fbsk_gpu=view)
    assert 0 < got < 0.5 and abs(got / want - 1.0) < 1e-6, (code, got, want)
