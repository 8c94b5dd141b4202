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
    ks.close()
    ref, _ = O.pbs_batch(env["op"], cts, B.trivial_glwe(p, tlu)[None, :], fbsk=env["fcpu"])
    assert np.array_equal(got, ref) and np.array_equal(again, ref)
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
