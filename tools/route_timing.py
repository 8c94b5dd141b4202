"""GPU box: where the direct memref route's time goes at cfg2 batch 4096 (keyset timeline vs wall)."""
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from concrete_amd import backend as B  # noqa: E402
from concrete_amd import runtime as R  # noqa: E402

if "--torch" in sys.argv:  # torch's GPU context and streams in the same process, as in bench.py
    import torch
    a = torch.randn(2048, 2048, device="cuda")
    for _ in range(10):
        a = (a @ a).tanh()
    torch.cuda.synchronize()

p = B.CFG2
lwe_sk = B.binary_key(p.n, 1)
glwe_sk = B.binary_key(p.big_n, 2)
bsk = B.bsk_generate(p, lwe_sk, glwe_sk, 3)
width = 3
table = np.array([5, 3, 0, 7, 1, 6, 2, 4], dtype=np.uint64)
tlu = B.expand_lut(table, p.N, width)
msgs = np.arange(4096) % 8
cts = B.lwe_encrypt(lwe_sk, [B.encode(m, width) for m in msgs], p.n, 2.0 ** -25, 4)
ks = R.Keyset([0])
ks.add_bsk(0, bsk, p)
R.batched_bootstrap(ks, p, cts, tlu)
ks.set_timing(True)
for it in range(3):
    t0 = time.perf_counter()
    out = R.batched_bootstrap(ks, p, cts, tlu)
    t1 = time.perf_counter()
    print(f"call {it}: wall {1e3 * (t1 - t0):.2f} ms; timeline (dev, start, in, kernel, out, n):",
          np.round(ks.timeline(), 3).tolist(), flush=True)
t0 = time.perf_counter()
z = np.zeros((4096, p.k * p.N + 1), dtype=np.uint64)
print(f"np.zeros of the output: {1e3 * (time.perf_counter() - t0):.2f} ms")

# the bench's order: the stream-emulator graph on a keyset with both keys, then the direct route
ksk = B.ksk_generate(p, glwe_sk, lwe_sk, 6)
kset = R.Keyset([0])
kset.add_bsk(0, bsk, p)
kset.add_ksk(0, ksk, p)
ctx = 0x5DF6
kset.bind(ctx)
g = R.Dfg()
s_in = g.batch_stream("in", R.TS_X86_TO_TOPO)
s_lut = g.memref_stream("lut", R.TS_X86_TO_TOPO)
s_mid = g.batch_stream("mid")
s_res = g.batch_stream("out", R.TS_TOPO_TO_X86)
g.keyswitch(s_in, s_mid, p, ctx)
g.bootstrap(s_mid, s_lut, s_res, p, ctx)
g.run()
big_in = B.lwe_encrypt(glwe_sk, [B.encode(int(m) % 4, 2) for m in msgs], p.big_n, 2.0 ** -30, 18)
g.put_memref(s_lut, B.expand_lut(np.array([3, 0, 2, 1], dtype=np.uint64), p.N, 2))
for it in range(3):
    t0 = time.perf_counter()
    g.put_batch(s_in, big_in)
    res = g.get_batch(s_res, 4096, p.k * p.N + 1)
    print(f"sdfg run {it}: wall {1e3 * (time.perf_counter() - t0):.2f} ms", flush=True)
g.close()
kset.set_timing(True)
for it in range(3):
    t0 = time.perf_counter()
    out = R.batched_bootstrap(kset, p, cts, tlu)
    t1 = time.perf_counter()
    print(f"direct after sdfg {it}: wall {1e3 * (t1 - t0):.2f} ms; timeline:", np.round(kset.timeline(), 3).tolist(),
          flush=True)
