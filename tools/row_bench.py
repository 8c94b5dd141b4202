"""PBS/s of one parameter row at batch B (timing helper for rows without a bench.py config).
Usage: python tools/row_bench.py k N n l logB [B]  (synthetic keys; 2 rows checked bit-exact).
GENERIC=1: the general path on its own key format (concrete_hip_convert_bsk_generic +
concrete_hip_pbs_generic), for comparison with a hand-tuned kernel."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from concrete_amd import backend as B
from oracle import pyoracle as O

k, N, n, l, logB = (int(x) for x in sys.argv[1:6])
nb = int(sys.argv[6]) if len(sys.argv) > 6 else 4096
p = B.PbsParams(n=n, k=k, N=N, level=l, base_log=logB)
lwe_sk, glwe_sk = B.binary_key(p.n, 1), B.binary_key(p.big_n, 2)
bsk = B.bsk_generate(p, lwe_sk, glwe_sk, 3)
generic = os.environ.get("GENERIC") == "1"
rng = np.random.RandomState(0)
cts = B.lwe_encrypt(lwe_sk, [B.encode(m, 2) for m in rng.randint(0, 4, nb)], p.n, B.secure_std(1, p.n), 5)
acc = B.trivial_glwe(p, B.expand_lut(np.arange(4, dtype=np.uint64), p.N, 2))
d_in, d_lut = B.to_device(cts, "cuda:0"), B.to_device(acc[None, :], "cuda:0")
if generic:
    from concrete_amd import _native
    L = _native.lib()
    dev = torch.device("cuda:0")
    st, gi = B._stream(dev), B._gpu_index(dev)
    g = torch.empty(L.concrete_hip_generic_bsk_size_bytes(p.n, p.k, p.level, p.N) // 8, dtype=torch.int64, device=dev)
    _native.check(L.concrete_hip_convert_bsk_generic(st, gi, B._ptr(g), bsk.ctypes.data, 0, p.n, p.k, p.level, p.N),
                  "convert_bsk_generic")
    out = torch.zeros((nb, p.lwe_out_size), dtype=torch.int64, device=dev)

    def run():
        _native.check(L.concrete_hip_pbs_generic(st, gi, B._ptr(out), None, B._ptr(d_lut), None, B._ptr(d_in), None,
                                                 B._ptr(g), p.n, p.k, p.N, p.base_log, p.level, nb, None), "pbs_generic")
else:
    fbsk = B.convert_bsk(p, bsk, "cuda:0")
    out = B.pbs(p, fbsk, d_in, d_lut)

    def run():
        B.pbs(p, fbsk, d_in, d_lut, out=out)
run()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(3):
    run()
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / 3
ref, _ = O.pbs_batch(O.Params(n=p.n, k=p.k, N=p.N, l=p.level, logB=p.base_log), cts[:2], acc[None, :], bsk=bsk,
                     mode=O.MODE_KARATSUBA)
print({"k": k, "N": N, "n": n, "l": l, "logB": logB, "batch": nb, "format": 3 if generic else B.bsk_format(p)[0],
       "pbs_per_s": round(nb / dt, 1), "bitexact_2": bool(np.array_equal(B.to_host(out)[:2], ref))})
