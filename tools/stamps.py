"""Diagnostic: per-phase cycle shares of the PBS kernel (CONCRETE_HIP_PBS_STAMPS build)."""
import os, sys
os.environ["CONCRETE_HIP_PBS_STAMPS"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from concrete_amd import backend as B
p = B.CFG2
nb = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
lwe_sk = B.binary_key(p.n, 1); glwe_sk = B.binary_key(p.big_n, 2)
bsk = B.bsk_generate(p, lwe_sk, glwe_sk, 3)
fbsk = B.convert_bsk(p, bsk, "cuda:0")
rng = np.random.RandomState(0)
cts = B.lwe_encrypt(lwe_sk, [B.encode(m, 3) for m in rng.randint(0, 8, nb)], p.n, B.secure_std(1, p.n), 5)
acc = B.trivial_glwe(p, B.expand_lut(np.arange(8, dtype=np.uint64), p.N, 3))
P = int(os.environ.get("CONCRETE_HIP_PBS_PAIRS", "4"))
nw = 2 * ((nb + P - 1) // P) * P  # pair kernel: two waves per ciphertext, P pairs per workgroup
NS = 10  # kernel_util.hpp NSTAMP
buf = torch.zeros(nw * NS, dtype=torch.int64, device="cuda:0")
d_in, d_lut = B.to_device(cts, "cuda:0"), B.to_device(acc[None, :], "cuda:0")
B.pbs(p, fbsk, d_in, d_lut, resid=buf); torch.cuda.synchronize()
buf.zero_()
t0 = torch.cuda.Event(enable_timing=True); t1 = torch.cuda.Event(enable_timing=True)
t0.record(); B.pbs(p, fbsk, d_in, d_lut, resid=buf); t1.record(); torch.cuda.synchronize()
st = buf.cpu().numpy().reshape(nw, NS).astype(np.float64)
names = ["rot+decomp", "fwd+xchg", "mac", "y-xchg", "inv+recomb", "ring-barrier", "total", "work_steps", "vmcnt-wait"]
tot = st[:, 6].mean()
print(f"kernel {t0.elapsed_time(t1):.2f} ms (stamp build), batch {nb}, mean wave cycles {tot:.3g} (memtime ticks)")
for k in (0, 1, 2, 8, 3, 4, 5):
    nme = names[k]
    print(f"  {nme:14s} {st[:, k].mean() / tot * 100:6.1f} %   per step {st[:, k].mean() / p.n:9.0f}")
print(f"  work steps {st[:, 7].mean():.1f}")
