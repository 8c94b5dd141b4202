"""GPU tests of the circuit-facing runtime glue (include/concrete_hip.h Part 4,
concrete_amd/csrc/runtime.hip): memref-descriptor wrappers over a native keyset, checked
bit-exactly against the oracle, including batches sharded over a device list.
"""
from dataclasses import replace

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def env():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a visible MI355X"
    from concrete_amd import backend as B
    from concrete_amd import runtime as R
    from oracle import pyoracle as O
    p = replace(B.CFG2, n=24)
    op = O.Params(n=p.n, k=p.k, N=p.N, l=p.level, logB=p.base_log, ks_l=p.ks_level, ks_logB=p.ks_base_log)
    lwe_sk = B.binary_key(p.n, 71)
    glwe_sk = B.binary_key(p.big_n, 72)
    bsk = B.bsk_generate(p, lwe_sk, glwe_sk, 73)
    ksk = B.ksk_generate(p, glwe_sk, lwe_sk, 74, std=2.0 ** -40)
    fcpu = O.bsk_to_fourier(op, bsk)
    return dict(B=B, R=R, O=O, p=p, op=op, lwe_sk=lwe_sk, glwe_sk=glwe_sk, bsk=bsk, ksk=ksk, fcpu=fcpu)


def keyset(env, devices=None):
    ks = env["R"].Keyset(devices)
    ks.add_bsk(0, env["bsk"], env["p"])
    ks.add_ksk(0, env["ksk"], env["p"])
    return ks


def inputs(env, nb, width, seed):
    B, p = env["B"], env["p"]
    rng = np.random.RandomState(seed)
    msgs = rng.randint(0, 1 << width, size=nb)
    cts = B.lwe_encrypt(env["lwe_sk"], [B.encode(m, width) for m in msgs], p.n, 2.0 ** -25, seed)
    return msgs, cts


@pytest.mark.parametrize("devices,nb", [(None, 9), ([0, 0, 0], 7), ([0, 0], 1)])
def test_batched_bootstrap(env, devices, nb):
    B, R, O, p = env["B"], env["R"], env["O"], env["p"]
    width = 3
    table = np.array([2, 7, 1, 0, 5, 5, 3, 6], dtype=np.uint64)
    tlu = B.expand_lut(table, p.N, width)
    msgs, cts = inputs(env, nb, width, 100 + nb)
    ks = keyset(env, devices)
    got = R.batched_bootstrap(ks, p, cts, tlu)
    again = R.batched_bootstrap(ks, p, cts, tlu)  # device key already resident
    into = np.full_like(got, 0xDEAD)
    R.batched_bootstrap(ks, p, cts, tlu, out=into)  # a caller-owned output memref, overwritten
    ks.close()
    ref, _ = O.pbs_batch(env["op"], cts, B.trivial_glwe(p, tlu)[None, :], fbsk=env["fcpu"])
    assert np.array_equal(got, ref) and np.array_equal(again, ref) and np.array_equal(into, ref)
    dec = B.lwe_decrypt(env["glwe_sk"], got, p.big_n)
    assert [B.decode(d, width) for d in dec] == [int(table[m]) for m in msgs]


@pytest.mark.parametrize("devices", [None, [0, 0]])
def test_batched_mapped_bootstrap(env, devices):
    B, R, O, p = env["B"], env["R"], env["O"], env["p"]
    width = 3
    nb = 6
    rng = np.random.RandomState(5)
    tables = [rng.randint(0, 8, size=8).astype(np.uint64) for _ in range(nb)]
    tlus = np.stack([B.expand_lut(t, p.N, width) for t in tables])
    msgs, cts = inputs(env, nb, width, 200)
    ks = keyset(env, devices)
    got = R.batched_mapped_bootstrap(ks, p, cts, tlus)
    one = R.batched_mapped_bootstrap(ks, p, cts, tlus[:1])  # a single LUT row serves every sample
    ks.close()
    accs = np.stack([B.trivial_glwe(p, t) for t in tlus])
    ref, _ = O.pbs_batch(env["op"], cts, accs, fbsk=env["fcpu"], lut_idx=np.arange(nb, dtype=np.uint64))
    assert np.array_equal(got, ref)
    ref1, _ = O.pbs_batch(env["op"], cts, accs[:1], fbsk=env["fcpu"])
    assert np.array_equal(one, ref1)
    dec = B.lwe_decrypt(env["glwe_sk"], got, p.big_n)
    assert [B.decode(d, width) for d in dec] == [int(tables[i][m]) for i, m in enumerate(msgs)]


def test_single_and_keyswitch_chain(env):
    """memref_bootstrap / memref_keyswitch (one ciphertext) and the batched KS -> PBS chain."""
    B, R, O, p = env["B"], env["R"], env["O"], env["p"]
    width = 2
    table = np.array([1, 3, 0, 2], dtype=np.uint64)
    tlu = B.expand_lut(table, p.N, width)
    msgs, cts = inputs(env, 5, width, 300)
    ks = keyset(env, [0, 0])
    big = R.batched_bootstrap(ks, p, cts, tlu)
    single = R.bootstrap(ks, p, cts[2], tlu)
    assert np.array_equal(single, big[2])
    small = R.batched_keyswitch(ks, p, big)
    assert np.array_equal(small, O.keyswitch_batch(env["op"], big, env["ksk"]))
    assert np.array_equal(R.keyswitch(ks, p, big[4]), small[4])
    out = R.batched_bootstrap(ks, p, small, tlu)
    ks.close()
    dec = B.lwe_decrypt(env["glwe_sk"], out, p.big_n)
    # table applied twice: m -> T[T[m]]
    assert [B.decode(d, width) for d in dec] == [int(table[table[m]]) for m in msgs]


def test_batched_bootstrap_n2048(env):
    """The runtime glue drives the N = 2048 kernel too (cfg4 shape, small n)."""
    B, R, O = env["B"], env["R"], env["O"]
    p = replace(B.CFG4, n=12)
    op = O.Params(n=p.n, k=p.k, N=p.N, l=p.level, logB=p.base_log, limbs=O.limbs_for(p.N))
    lwe_sk = B.binary_key(p.n, 81)
    glwe_sk = B.binary_key(p.big_n, 82)
    bsk = B.bsk_generate(p, lwe_sk, glwe_sk, 83)
    width = 4
    table = np.arange(16, dtype=np.uint64)[::-1].copy()
    tlu = B.expand_lut(table, p.N, width)
    msgs = np.array([0, 3, 9, 15, 7])
    cts = B.lwe_encrypt(lwe_sk, [B.encode(m, width) for m in msgs], p.n, 2.0 ** -30, 84)
    ks = R.Keyset([0, 0])
    ks.add_bsk(0, bsk, p)
    got = R.batched_bootstrap(ks, p, cts, tlu)
    ks.close()
    ref, _ = O.pbs_batch(op, cts, B.trivial_glwe(p, tlu)[None, :], fbsk=O.bsk_to_fourier(op, bsk))
    assert np.array_equal(got, ref)


def test_batched_bootstrap_general_path(env):
    """The runtime glue drives the general path (k = 3, N = 512: the optimizer's 3-bit row,
    small n), sharded over two device entries; bit-exact vs the oracle's Karatsuba product."""
    B, R, O = env["B"], env["R"], env["O"]
    p = replace(B.OPTIMIZER_SETS[3], n=12)
    lwe_sk = B.binary_key(p.n, 91)
    glwe_sk = B.binary_key(p.big_n, 92)
    bsk = B.bsk_generate(p, lwe_sk, glwe_sk, 93)
    width = 3
    table = np.array([3, 1, 4, 1, 5, 2, 6, 5], dtype=np.uint64)
    tlu = B.expand_lut(table, p.N, width)
    msgs = np.array([0, 1, 2, 3, 4, 5, 6, 7, 2])
    cts = B.lwe_encrypt(lwe_sk, [B.encode(m, width) for m in msgs], p.n, 2.0 ** -30, 94)
    ks = R.Keyset([0, 0])
    ks.add_bsk(0, bsk, p)
    got = R.batched_bootstrap(ks, p, cts, tlu)
    ks.close()
    op = O.Params(n=p.n, k=p.k, N=p.N, l=p.level, logB=p.base_log)
    ref, _ = O.pbs_batch(op, cts, B.trivial_glwe(p, tlu)[None, :], bsk=bsk, mode=O.MODE_KARATSUBA)
    assert np.array_equal(got, ref)
    dec = B.lwe_decrypt(glwe_sk, got, p.big_n)
    assert [B.decode(d, width) for d in dec] == [int(table[m]) for m in msgs]


def test_slices_overlap_and_bit_exact(env):
    """Slices of one call are issued concurrently (one host thread, stream and buffer set per
    slice): no slice waits for another's outputs (the round-2 loop
    issued slice r + 1 only after slice r's pageable D2H had returned; an outgrown buffer's hipFree
    also synchronised the device mid-call until it was deferred to after the join)."""
    B, R, O = env["B"], env["R"], env["O"]
    p = B.CFG2  # full n: each slice's kernel runs for milliseconds
    lwe_sk = B.binary_key(p.n, 61)
    glwe_sk = B.binary_key(p.big_n, 62)
    bsk = B.bsk_generate(p, lwe_sk, glwe_sk, 63)
    width = 3
    table = np.array([6, 1, 7, 0, 3, 2, 5, 4], dtype=np.uint64)
    tlu = B.expand_lut(table, p.N, width)
    nb = 1024
    rng = np.random.RandomState(64)
    msgs = rng.randint(0, 1 << width, size=nb)
    cts = B.lwe_encrypt(lwe_sk, [B.encode(m, width) for m in msgs], p.n, B.secure_std(1, p.n), 65)
    ks = R.Keyset([0, 0, 0, 0])
    ks.add_bsk(0, bsk, p)
    # key conversion and the slices' device buffers (grown by hipMalloc, which can wait for the
    # device) outside the recorded call: the steady state of a runtime issuing repeated batches
    R.batched_bootstrap(ks, p, cts, tlu)
    ks.set_timing(True)
    got = R.batched_bootstrap(ks, p, cts, tlu)
    tl = ks.timeline()
    ks.close()
    assert tl.shape == (4, 6) and list(tl[:, 5]) == [256] * 4
    # columns: device, start, inputs copied (kernel issue), kernel done, outputs copied, count.
    # Every slice starts while another slice's kernel is still running (round 2 issued slice r + 1
    # only after slice r's D2H, so its last slice started after every other kernel was done).  On
    # one device the kernels queue for CUs (each 256-sample launch fills the chip), and a slice
    # thread's first HIP call can wait while another thread sits in a blocking pageable copy on the
    # same device, so neither kernel overlap nor a fixed issue order is asserted.
    for r in range(1, 4):
        others = [tl[q, 3] for q in range(4) if q != r]
        assert tl[r, 1] < max(others), tl
    assert int((tl[1:, 1] < tl[0, 3]).sum()) >= 1, tl
    dec = B.lwe_decrypt(glwe_sk, got, p.big_n)
    assert [B.decode(d, width) for d in dec] == [int(table[m]) for m in msgs]
    op = O.Params(n=p.n, k=p.k, N=p.N, l=p.level, logB=p.base_log)
    rows = np.array([0, 255, 256, 511, 767, 1023])
    ref, _ = O.pbs_batch(op, cts[rows], B.trivial_glwe(p, tlu)[None, :], fbsk=O.bsk_to_fourier(op, bsk))
    assert np.array_equal(got[rows], ref)


def test_concurrent_calls_on_one_keyset_overlap(env):
    """Two threads run memref_batched_bootstrap_lwe_cuda_u64 on ONE shared keyset (two runtime
    contexts bound to it, as INTEGRATION.md §4 recommends): each call takes a slot set of its own and
    reads the device status on its own stream, so the second call is issued while the first call's
    kernel is still running (round 3 held one lock for the whole call and synchronised the device
    after it).  HIP events on a common time base show the overlap; both results are bit-exact."""
    import ctypes as C
    import threading
    B, R, O = env["B"], env["R"], env["O"]
    p = B.CFG2  # full n: kernels of tens of ms
    lwe_sk = B.binary_key(p.n, 81)
    glwe_sk = B.binary_key(p.big_n, 82)
    bsk = B.bsk_generate(p, lwe_sk, glwe_sk, 83)
    width = 3
    table = np.array([1, 3, 5, 7, 0, 2, 4, 6], dtype=np.uint64)
    tlu = B.expand_lut(table, p.N, width)
    nb = 2048
    rng = np.random.RandomState(84)
    msgs = rng.randint(0, 1 << width, size=(2, nb))
    cts = [B.lwe_encrypt(lwe_sk, [B.encode(m, width) for m in msgs[i]], p.n, B.secure_std(1, p.n), 85 + i)
           for i in range(2)]
    ks = R.Keyset([0])
    ks.add_bsk(0, bsk, p)
    ctx = [C.create_string_buffer(64) for _ in range(2)]  # two RuntimeContexts, one keyset
    for c in ctx:
        ks.bind(C.addressof(c))
    for i in range(2):  # key conversion and both slot sets' buffers outside the recorded calls
        R.batched_bootstrap_cuda(C.addressof(ctx[i]), p, cts[i], tlu)
    outs = [None, None]
    gate = threading.Barrier(2)

    def call(i):
        gate.wait()
        outs[i] = R.batched_bootstrap_cuda(C.addressof(ctx[i]), p, cts[i], tlu)

    for _ in range(2):  # warm both slot sets under concurrency too
        th = [threading.Thread(target=call, args=(i,)) for i in range(2)]
        [t.start() for t in th]
        [t.join() for t in th]
    ks.set_timing(True)
    th = [threading.Thread(target=call, args=(i,)) for i in range(2)]
    [t.start() for t in th]
    [t.join() for t in th]
    tl = ks.timeline()
    ks.close()
    assert tl.shape == (2, 6) and list(tl[:, 5]) == [nb, nb], tl
    # columns: device, start, inputs copied (kernel issue), kernel done, outputs copied, count
    first, second = (0, 1) if tl[0, 1] <= tl[1, 1] else (1, 0)
    assert tl[second, 1] < tl[first, 3], f"the second call waited for the first call's kernel: {tl}"
    for i in range(2):
        dec = B.lwe_decrypt(glwe_sk, outs[i], p.big_n)
        assert [B.decode(d, width) for d in dec] == [int(table[m]) for m in msgs[i]]
    op = O.Params(n=p.n, k=p.k, N=p.N, l=p.level, logB=p.base_log)
    rows = np.array([0, 777, nb - 1])
    fcpu = O.bsk_to_fourier(op, bsk)
    for i in range(2):
        ref, _ = O.pbs_batch(op, cts[i][rows], B.trivial_glwe(p, tlu)[None, :], fbsk=fcpu)
        assert np.array_equal(outs[i][rows], ref)


def test_cuda_names_resolve_the_runtime_context(env):
    """memref_*_cuda_u64 under the reference's names take the circuit's RuntimeContext pointer:
    bound with concrete_hip_context_bind, or answered by a registered resolver."""
    import ctypes as C
    B, R, O, p = env["B"], env["R"], env["O"], env["p"]
    width = 3
    table = np.array([2, 7, 1, 0, 5, 5, 3, 6], dtype=np.uint64)
    tlu = B.expand_lut(table, p.N, width)
    msgs, cts = inputs(env, 6, width, 400)
    ks = keyset(env, [0, 0])
    fake_ctx = C.create_string_buffer(64)  # stands for a RuntimeContext object
    ctx = C.addressof(fake_ctx)
    ks.bind(ctx)
    big = R.batched_bootstrap_cuda(ctx, p, cts, tlu)
    ref, _ = O.pbs_batch(env["op"], cts, B.trivial_glwe(p, tlu)[None, :], fbsk=env["fcpu"])
    assert np.array_equal(big, ref)
    assert np.array_equal(R.bootstrap_cuda(ctx, p, cts[3], tlu), ref[3])
    small = R.batched_keyswitch_cuda(ctx, p, big)
    assert np.array_equal(small, O.keyswitch_batch(env["op"], big, env["ksk"]))
    assert np.array_equal(R.keyswitch_cuda(ctx, p, big[1]), small[1])
    tlus = np.stack([tlu, tlu[::-1].copy()] * 3)
    mapped = R.batched_mapped_bootstrap_cuda(ctx, p, cts, tlus)
    accs = np.stack([B.trivial_glwe(p, t) for t in tlus])
    refm, _ = O.pbs_batch(env["op"], cts, accs, fbsk=env["fcpu"], lut_idx=np.arange(6, dtype=np.uint64))
    assert np.array_equal(mapped, refm)
    # a resolver answers for contexts nobody bound (e.g. one RuntimeContext per invocation)
    L = ks.lib
    seen = []
    RESOLVER = C.CFUNCTYPE(C.c_void_p, C.c_void_p, C.c_void_p)

    @RESOLVER
    def resolve(c, user):
        seen.append(c)
        return ks.h

    L.concrete_hip_set_context_resolver(C.cast(resolve, C.c_void_p), None)
    other = C.create_string_buffer(64)
    try:
        again = R.batched_bootstrap_cuda(C.addressof(other), p, cts, tlu)
        again2 = R.batched_bootstrap_cuda(C.addressof(other), p, cts, tlu)  # cached: resolver asked once
    finally:
        L.concrete_hip_set_context_resolver(None, None)
    assert seen == [C.addressof(other)]
    assert np.array_equal(again, ref) and np.array_equal(again2, ref)
    ks.close()


def test_device_lut_encoding_and_accumulators(env):
    """LUT encoding and trivial-GLWE accumulators on the device (lut.hip) equal the runtime's host
    forms (wrappers.cpp:388-450, 199-209) for every width, signedness and mega-case size."""
    import torch
    B, p = env["B"], env["p"]
    L = env["R"]._native.lib()
    rng = np.random.RandomState(9)
    s = torch.cuda.current_stream().cuda_stream
    for bits in (1, 2, 3, 4, 6, 8):
        for signed in (False, True):
            for N in (256, 1024, 4096):
                if (N >> bits) < 2:
                    continue
                rows = 3
                tabs = rng.randint(0, 1 << bits, size=(rows, 1 << bits)).astype(np.uint64)
                d_in = B.to_device(tabs, "cuda:0")
                d_out = torch.empty((rows, N), dtype=torch.int64, device="cuda:0")
                assert L.concrete_hip_encode_expand_lut_device(s, 0, d_out.data_ptr(), N, d_in.data_ptr(), 1 << bits,
                                                               rows, bits, int(signed)) == 0
                got = B.to_host(d_out)
                for r in range(rows):
                    assert np.array_equal(got[r], B.expand_lut(tabs[r], N, bits, signed)), (bits, signed, N, r)
    tl = np.stack([B.expand_lut(rng.randint(0, 8, size=8).astype(np.uint64), p.N, 3) for _ in range(4)])
    for k in (1, 2):
        d_l = B.to_device(tl, "cuda:0")
        d_acc = torch.empty((4, (k + 1) * p.N), dtype=torch.int64, device="cuda:0")
        assert L.concrete_hip_build_accumulators(s, 0, d_acc.data_ptr(), d_l.data_ptr(), 4, k, p.N) == 0
        acc = B.to_host(d_acc)
        for r in range(4):
            want = np.zeros((k + 1) * p.N, dtype=np.uint64)
            want[k * p.N:] = tl[r]
            assert np.array_equal(acc[r], want)
    assert L.concrete_hip_encode_expand_lut_device(s, 0, 1, 1000, 1, 8, 1, 3, 0) == -3  # 1000 / 8 is odd


@pytest.mark.parametrize("layout", ["flat", "mixed"])
def test_keyset_from_wire_format(env, layout):
    """A server keyset serialized in the concrete-protocol wire form (include/concrete_hip.h Part 6)
    loads into a runtime keyset and runs the PBS -> KS -> PBS chain bit-exactly (oracle)."""
    from concrete_amd import keys as K
    B, R, O, p = env["B"], env["R"], env["O"], env["p"]
    width = 2
    table = np.array([2, 0, 3, 1], dtype=np.uint64)
    tlu = B.expand_lut(table, p.N, width)
    msgs, cts = inputs(env, 6, width, 500)
    data = K.serialize_server_keyset([(K.bsk_info(p), env["bsk"])], [(K.ksk_info(p), env["ksk"])],
                                     layout=layout, blob_words=4096)
    sk = K.ServerKeyset.deserialize(data)
    ks = R.Keyset([0, 0])
    sk.add_to(ks)
    sk.close()
    big = R.batched_bootstrap(ks, p, cts, tlu)
    small = R.batched_keyswitch(ks, p, big)
    out = R.batched_bootstrap(ks, p, small, tlu)
    ks.close()
    ref, _ = O.pbs_batch(env["op"], cts, B.trivial_glwe(p, tlu)[None, :], fbsk=env["fcpu"])
    assert np.array_equal(big, ref)
    assert np.array_equal(small, O.keyswitch_batch(env["op"], big, env["ksk"]))
    dec = B.lwe_decrypt(env["glwe_sk"], out, p.big_n)
    assert [B.decode(d, width) for d in dec] == [int(table[table[m]]) for m in msgs]


@pytest.mark.parametrize("level,base_log", [(1, 15), (2, 12), (1, 23)])
def test_wide_digits_on_the_general_path(env, level, base_log):
    """k = 1, N = 1024 with digits wider than the pair kernel's exactness gate ((k+1) l 2^logB <=
    4096): the general path runs them on a general-format companion of the key, built from the
    standard key the keyset holds (memref route) or that the legacy conversion left in `dest`
    (cuda_* route), and on a caller-converted key (concrete_hip_pbs_generic); bit-exact vs the
    oracle's pure-integer Karatsuba PBS (these sets were refused)."""
    import ctypes as C
    from concrete_amd import _native
    B, R, O = env["B"], env["R"], env["O"]
    L = _native.lib()
    p = replace(B.CFG2, n=12, level=level, base_log=base_log)
    assert L.concrete_hip_pbs_supported(p.k, p.N, p.level, p.base_log) == 1
    lwe_sk = B.binary_key(p.n, 81)
    glwe_sk = B.binary_key(p.big_n, 82)
    # such wide digits amplify the key noise 2^(logB-1) sqrt((k+1) l N)-fold: with the secure GLWE
    # noise for N = 1024 nothing would decrypt (why no optimizer table picks them), so the key is
    # encrypted with small noise here; bit-exactness does not depend on it
    bsk = B.bsk_generate(p, lwe_sk, glwe_sk, 83, std=2.0 ** -52)
    width = 3
    table = np.array([4, 1, 6, 3, 0, 7, 2, 5], dtype=np.uint64)
    tlu = B.expand_lut(table, p.N, width)
    acc = B.trivial_glwe(p, tlu)
    rng = np.random.RandomState(level * 100 + base_log)
    msgs = rng.randint(0, 1 << width, size=9)
    cts = B.lwe_encrypt(lwe_sk, [B.encode(m, width) for m in msgs], p.n, 2.0 ** -25, 84)
    op = O.Params(n=p.n, k=p.k, N=p.N, l=p.level, logB=p.base_log)
    ref, _ = O.pbs_batch(op, cts, acc[None, :], bsk=bsk, mode=O.MODE_KARATSUBA)
    dec = B.lwe_decrypt(glwe_sk, ref, p.big_n)
    assert [B.decode(d, width) for d in dec] == [int(table[m]) for m in msgs]
    # memref route: keyset on [0, 0] (two slices)
    ks = R.Keyset([0, 0])
    ks.add_bsk(0, bsk, p)
    got = R.batched_bootstrap(ks, p, cts, tlu)
    again = R.batched_bootstrap(ks, p, cts, tlu)  # companion already built
    ks.close()
    assert np.array_equal(got, ref) and np.array_equal(again, ref)
    # cuda_* route: the registry's conversion, then the runtime's PBS call
    s = L.cuda_create_stream(0)
    d_bsk = L.cuda_malloc_async(bsk.nbytes, s, 0)
    L.cuda_convert_lwe_programmable_bootstrap_key_64(s, 0, d_bsk, bsk.ctypes.data, p.n, p.k, p.level, p.N)
    nb = len(msgs)
    d_in = L.cuda_malloc_async(cts.nbytes, s, 0)
    L.cuda_memcpy_async_to_gpu(d_in, cts.ctypes.data, cts.nbytes, s, 0)
    d_out = L.cuda_malloc_async(nb * (p.k * p.N + 1) * 8, s, 0)
    d_acc = L.cuda_malloc_async(acc.nbytes, s, 0)
    L.cuda_memcpy_async_to_gpu(d_acc, acc.ctypes.data, acc.nbytes, s, 0)
    idx = np.arange(nb, dtype=np.uint64)
    zeros = np.zeros(nb, dtype=np.uint64)
    d_idx = L.cuda_malloc_async(idx.nbytes, s, 0)
    d_lidx = L.cuda_malloc_async(idx.nbytes, s, 0)
    L.cuda_memcpy_async_to_gpu(d_idx, idx.ctypes.data, idx.nbytes, s, 0)
    L.cuda_memcpy_async_to_gpu(d_lidx, zeros.ctypes.data, zeros.nbytes, s, 0)
    L.cuda_programmable_bootstrap_lwe_ciphertext_vector_64(s, 0, d_out, d_idx, d_acc, d_lidx, d_in, d_idx, d_bsk,
                                                          None, p.n, p.k, p.N, p.base_log, p.level, nb, 1, 1)
    out = np.zeros((nb, p.k * p.N + 1), dtype=np.uint64)
    L.cuda_memcpy_async_to_cpu(out.ctypes.data, d_out, out.nbytes, s, 0)
    L.cuda_synchronize_device(0)
    # caller-held key in the general format: concrete_hip_pbs_generic
    gbytes = L.concrete_hip_generic_bsk_size_bytes(p.n, p.k, p.level, p.N)
    d_g = L.cuda_malloc_async(gbytes, s, 0)
    _native.check(L.concrete_hip_convert_bsk_generic(s, 0, d_g, bsk.ctypes.data, 0, p.n, p.k, p.level, p.N),
                  "convert_bsk_generic")
    _native.check(L.concrete_hip_pbs_generic(s, 0, d_out, None, d_acc, None, d_in, None, d_g, p.n, p.k, p.N,
                                             p.base_log, p.level, nb, None), "pbs_generic")
    out2 = np.zeros_like(out)
    L.cuda_memcpy_async_to_cpu(out2.ctypes.data, d_out, out2.nbytes, s, 0)
    L.cuda_synchronize_device(0)
    for ptr in (d_in, d_out, d_acc, d_idx, d_lidx, d_g):
        L.cuda_drop_async(ptr, s, 0)
    L.cuda_drop(d_bsk, 0)
    L.cuda_destroy_stream(s, 0)
    assert np.array_equal(out, ref) and np.array_equal(out2, ref)
