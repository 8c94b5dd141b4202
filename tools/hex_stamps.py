"""Diagnostic: per-phase cycle shares of the six-wave kernel (pbs1024_hex.hip, STAMPS build).
Usage: python tools/hex_stamps.py [batch]"""
import os, sys
os.environ["CONCRETE_HIP_PBS_STAMPS"] = "1"
os.environ["CONCRETE_HIP_PBS_HEX"] = "2"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from concrete_amd import backend as B
p = B.CFG2
nb = int(sys.argv[1]) if len(sys.argv) > 1 else 512
lwe_sk = B.binary_key(p.n, 1); glwe_sk = B.binary_key(p.big_n, 2)
bsk = B.bsk_generate(p, lwe_sk, glwe_sk, 3)
fbsk = B.convert_bsk(p, bsk, "cuda:0")
rng = np.random.RandomState(0)
cts = B.lwe_encrypt(lwe_sk, [B.encode(m, 3) for m in rng.randint(0, 8, nb)], p.n, B.secure_std(1, p.n), 5)
acc = B.trivial_glwe(p, B.expand_lut(np.arange(8, dtype=np.uint64), p.N, 3))
nw = 6 * 2 * ((nb + 1) // 2)
NS = 10  # kernel_util.hpp NSTAMP
buf = torch.zeros(nw * NS, dtype=torch.int64, device="cuda:0")
d_in, d_lut = B.to_device(cts, "cuda:0"), B.to_device(acc[None, :], "cuda:0")
B.pbs(p, fbsk, d_in, d_lut, resid=buf); torch.cuda.synchronize()
buf.zero_()
t0 = torch.cuda.Event(enable_timing=True); t1 = torch.cuda.Event(enable_timing=True)
t0.record(); B.pbs(p, fbsk, d_in, d_lut, resid=buf); t1.record(); torch.cuda.synchronize()
st = buf.cpu().numpy().reshape(nw, NS).astype(np.float64)
names = {0: "rot+state", 1: "digits+fwd+publish", 2: "wait A", 3: "key products", 4: "wait B",
         5: "inv+round+atomics", 7: "wait C"}
tot = st[:, 6].mean()
print(f"kernel {t0.elapsed_time(t1):.2f} ms (stamp build), batch {nb}, mean wave cycles {tot:.3g}")
for k, nme in names.items():
    print(f"  {nme:20s} {st[:, k].mean() / tot * 100:6.1f} %   per step {st[:, k].mean() / p.n:9.0f}")
for u in range(6):
    print(f"  role {u}: " + " ".join(f"{st[u::6, k].mean() / p.n:7.0f}" for k in names))
