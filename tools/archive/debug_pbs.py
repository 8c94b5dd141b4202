"""Diagnostic: GPU vs oracle PBS on hand-made inputs (prints where they differ)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dataclasses import replace
import numpy as np, torch
from concrete_amd import backend as B
from oracle import pyoracle as O

p = replace(B.CFG2, n=4)
op = O.Params(n=p.n, k=p.k, N=p.N, l=p.level, logB=p.base_log)
lwe_sk = B.binary_key(p.n, 1); glwe_sk = B.binary_key(p.big_n, 2)
bsk = B.bsk_generate(p, lwe_sk, glwe_sk, 3)
fbsk = B.convert_bsk(p, bsk, "cuda:0"); fc = O.bsk_to_fourier(op, bsk)
acc = B.trivial_glwe(p, B.expand_lut(np.array([1,2,3,4,5,6,7,0], dtype=np.uint64), p.N, 3))
rng = np.random.RandomState(0)
cases = {}
c = rng.randint(0, 2**63, size=(1, p.n + 1), dtype=np.int64).view(np.uint64) * np.uint64(2)
z = c.copy(); z[0, :p.n] = 0; cases["no_cmux"] = z
o = c.copy(); o[0, 1:p.n] = 0; cases["one_cmux"] = o
t = c.copy(); t[0, [0, 2, 3]] = 0; cases["only_a1"] = t
t = c.copy(); t[0, [2, 3]] = 0; cases["a0_a1"] = t
t = c.copy(); t[0, [1, 2, 3]] = 0; t[0, 0] = np.uint64(1 << 60); cases["a0_small_rot"] = t
cases["all"] = c
for name, cts in cases.items():
    out = B.pbs(p, fbsk, B.to_device(cts, "cuda:0"), B.to_device(acc[None, :], "cuda:0"))
    torch.cuda.synchronize()
    got = B.to_host(out)
    ref, _ = O.pbs_batch(op, cts, acc[None, :], fbsk=fc)
    eq = np.array_equal(got, ref)
    print(name, "equal" if eq else "DIFF", flush=True)
    if not eq:
        d = (got[0].astype(object) - ref[0].astype(object)) % (1 << 64)
        nz = np.nonzero(got[0] != ref[0])[0]
        print("  n_diff", len(nz), "first idx", nz[:10], "diffs", [hex(int(x)) for x in d[nz[:6]]])
        print("  got", [hex(int(x)) for x in got[0][:4]], "ref", [hex(int(x)) for x in ref[0][:4]])
