"""GPU tests of the SDFG stream emulator (include/concrete_hip.h Part 5, concrete_amd/csrc/sdfg.hip):
tests/c_client/sdfg_client.c replays the call sequence a compiled KS -> PBS circuit emits
(SDFGToStreamEmulator.cpp:25-73: init, make streams / processes, run, put, get, delete) through
the C ABI, and every output is checked bit-exactly against the oracle, on the default device list
and on two entries of device 0 (two shards, two host threads)."""
import os
import shutil
import subprocess
from dataclasses import replace

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBDIR = os.path.join(ROOT, "concrete_amd")


@pytest.fixture(scope="module")
def client(tmp_path_factory):
    if shutil.which("gcc") is None:
        pytest.skip("gcc not installed")
    # (round 3 opened the GPU here before the client processes ran, after an abort in the next
    # module's first HIP call; round 4's experiment, tools/microbench/child_first_init.py,
    # profiles/r04_child_first_init.jsonl, found the device visible to a parent whose first HIP call
    # follows GPU-using children in every scenario, so the pre-open is gone: DESIGN.md §7)
    exe = tmp_path_factory.mktemp("sdfg") / "sdfg_client"
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Wextra", "-Werror", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "c_client", "sdfg_client.c"), "-L", LIBDIR, "-lconcrete_hip",
                    f"-Wl,-rpath,{LIBDIR}", "-o", str(exe)], check=True)
    return str(exe)


def _case(p, nb, seed, width):
    from concrete_amd import backend as B
    lwe_sk = B.binary_key(p.n, seed)
    glwe_sk = B.binary_key(p.big_n, seed + 1)
    bsk = B.bsk_generate(p, lwe_sk, glwe_sk, seed + 2)
    ksk = B.ksk_generate(p, glwe_sk, lwe_sk, seed + 3, std=2.0 ** -40)
    rng = np.random.RandomState(seed)
    msgs = rng.randint(0, (1 << width) - 1, size=nb)  # x + 1 stays in range
    cts = B.lwe_encrypt(glwe_sk, [B.encode(m, width) for m in msgs], p.big_n, 2.0 ** -40, seed + 4)
    tables = [rng.randint(0, 1 << width, size=1 << width).astype(np.uint64) for _ in range(nb)]
    luts = np.stack([B.expand_lut(t, p.N, width) for t in tables])
    return dict(lwe_sk=lwe_sk, glwe_sk=glwe_sk, bsk=bsk, ksk=ksk, msgs=msgs, cts=cts, tables=tables, luts=luts)


@pytest.mark.parametrize("devices", [None, "0,0"])
def test_sdfg_ks_pbs_circuit_replay(client, tmp_path, devices):
    from concrete_amd import backend as B
    from oracle import pyoracle as O
    p = replace(B.CFG2, n=24)
    width = 2
    nb = 10
    c = _case(p, nb, 500, width)
    pt = int(B.encode(1, width))
    hdr = np.array([p.n, p.k, p.N, p.level, p.base_log, p.ks_level, p.ks_base_log, nb], dtype=np.uint64)
    blob = np.concatenate([hdr, c["bsk"], c["ksk"], c["cts"].ravel(), np.array([pt], dtype=np.uint64),
                           c["luts"].ravel()])
    fin, fout = tmp_path / "in.bin", tmp_path / "out.bin"
    blob.tofile(fin)
    env = dict(os.environ)
    env.pop("CONCRETE_HIP_SDFG_DEVICES", None)
    if devices:
        env["CONCRETE_HIP_SDFG_DEVICES"] = devices
    res = subprocess.run([client, str(fin), str(fout)], env=env, capture_output=True, text=True, timeout=300)
    assert res.returncode == 0 and "sdfg_client ok" in res.stdout, res.stderr
    W = p.big_n + 1
    out = np.fromfile(fout, dtype=np.uint64).reshape(5, nb, W)
    # oracle: x + p -> KS -> PBS(lut0);  -r1;  rerun on reversed rows;  mapped;  single ciphertext
    op = O.Params(n=p.n, k=p.k, N=p.N, l=p.level, logB=p.base_log, ks_l=p.ks_level, ks_logB=p.ks_base_log)
    fcpu = O.bsk_to_fourier(op, c["bsk"])
    xp = c["cts"].copy()
    xp[:, -1] += np.uint64(pt)
    small = O.keyswitch_batch(op, xp, c["ksk"])
    acc0 = B.trivial_glwe(p, c["luts"][0])[None, :]
    r1, _ = O.pbs_batch(op, small, acc0, fbsk=fcpu)
    assert np.array_equal(out[0], r1)
    assert np.array_equal(out[1], (np.uint64(0) - r1).astype(np.uint64))
    assert np.array_equal(out[2], r1[::-1])
    small0 = O.keyswitch_batch(op, c["cts"], c["ksk"])
    accs = np.stack([B.trivial_glwe(p, l) for l in c["luts"]])
    r4, _ = O.pbs_batch(op, small0, accs, fbsk=fcpu, lut_idx=np.arange(nb, dtype=np.uint64))
    assert np.array_equal(out[3], r4)
    assert np.array_equal(out[4][0], r4[0] if nb == 1 else O.pbs_batch(op, small0[:1], acc0, fbsk=fcpu)[0][0])
    # and the circuit's meaning: lut0(m + 1), per-sample luts
    dec = B.lwe_decrypt(c["glwe_sk"], out[0], p.big_n)
    assert [B.decode(d, width) for d in dec] == [int(c["tables"][0][m + 1]) for m in c["msgs"]]
    dec4 = B.lwe_decrypt(c["glwe_sk"], out[3], p.big_n)
    assert [B.decode(d, width) for d in dec4] == [int(c["tables"][i][m]) for i, m in enumerate(c["msgs"])]


def test_sdfg_python_driver_reruns_into_caller_buffer(client):
    """concrete_amd.runtime.Dfg (the bench's route): KS -> PBS in this process, two puts of different
    batches read back into one caller-owned array, each bit-exact vs the oracle."""
    from concrete_amd import backend as B
    from concrete_amd import runtime as R
    from oracle import pyoracle as O
    p = replace(B.CFG2, n=24)
    width = 2
    nb = 6
    c = _case(p, nb, 700, width)
    kset = R.Keyset([0])
    kset.add_bsk(0, c["bsk"], p)
    kset.add_ksk(0, c["ksk"], p)
    ctx = 0x7A11
    kset.bind(ctx)
    g = R.Dfg()
    s_in = g.batch_stream("in", R.TS_X86_TO_TOPO)
    s_lut = g.memref_stream("lut", R.TS_X86_TO_TOPO)
    s_mid = g.batch_stream("mid")
    s_res = g.batch_stream("out", R.TS_TOPO_TO_X86)
    g.keyswitch(s_in, s_mid, p, ctx)
    g.bootstrap(s_mid, s_lut, s_res, p, ctx)
    g.run()
    g.put_memref(s_lut, c["luts"][0])
    op = O.Params(n=p.n, k=p.k, N=p.N, l=p.level, logB=p.base_log, ks_l=p.ks_level, ks_logB=p.ks_base_log)
    fcpu = O.bsk_to_fourier(op, c["bsk"])
    acc0 = B.trivial_glwe(p, c["luts"][0])[None, :]
    out = np.full((nb, p.big_n + 1), 0xBEEF, dtype=np.uint64)
    try:
        for batch in (c["cts"], c["cts"][::-1].copy()):
            g.put_batch(s_in, batch)
            got = g.get_batch(s_res, nb, p.big_n + 1, out=out)
            assert got is out
            ref, _ = O.pbs_batch(op, O.keyswitch_batch(op, batch, c["ksk"]), acc0, fbsk=fcpu)
            assert np.array_equal(out, ref)
        with pytest.raises(ValueError):
            g.get_batch(s_res, nb, p.big_n + 1, out=np.zeros((nb, p.big_n), dtype=np.uint64))
        # a put on the intermediate stream makes the downstream result stale (eff() had
        # ignored puts on produced streams, so this get returned the previous run's outputs)
        small = O.keyswitch_batch(op, c["cts"], c["ksk"])
        g.put_batch(s_mid, small)
        got = g.get_batch(s_res, nb, p.big_n + 1, out=out)
        ref, _ = O.pbs_batch(op, small, acc0, fbsk=fcpu)
        assert np.array_equal(got, ref)
    finally:
        g.close()
        kset.close()
