"""Phase shares of gen_coop_kernel (N = 8192, two workgroups per ciphertext) from a timing build
made with tools/archive/coop_stamps.patch (tools/variant.sh coopstamps after applying it; the build
sums s_memtime deltas per phase into the resid buffer: every wave's cycles, all launches).
Usage on the GPU box: CONCRETE_HIP_LIB=variants/libconcrete_hip_coopstamps.so python tools/coop_stamps.py [batch] [n]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from concrete_amd import backend as B  # noqa: E402

batch = int(sys.argv[1]) if len(sys.argv) > 1 else 512
n = int(sys.argv[2]) if len(sys.argv) > 2 else 64
p = B.PbsParams(n=n, k=1, N=8192, level=1, base_log=22)
lwe_sk, glwe_sk = B.binary_key(p.n, 1), B.binary_key(p.big_n, 2)
fbsk = B.convert_bsk(p, B.bsk_generate(p, lwe_sk, glwe_sk, 3), "cuda:0")
rng = np.random.RandomState(4)
cts = B.lwe_encrypt(lwe_sk, [B.encode(int(m), 7) for m in rng.randint(0, 128, size=batch)], p.n, 2.0 ** -30, 5)
acc = B.trivial_glwe(p, B.expand_lut(np.arange(128, dtype=np.uint64), p.N, 7))
d_in, d_acc = B.to_device(cts, "cuda:0"), B.to_device(acc[None, :], "cuda:0")
r = torch.zeros(8, dtype=torch.int64, device="cuda:0")
B.pbs(p, fbsk, d_in, d_acc)  # warm-up
r.zero_()
torch.cuda.synchronize()
B.pbs(p, fbsk, d_in, d_acc, resid=r)
torch.cuda.synchronize()
v = r.cpu().numpy().astype(np.float64)
names = {0: "rotation + decomposition", 1: "forward + column DFT + X stores", 2: "X hand-off wait",
         4: "X loads (slot 0) + products", 3: "Y stores", 5: "Y hand-off wait (publish + consume)",
         6: "Y loads + inverse column DFT + barrier", 7: "row inverse + recombination + barrier"}
order = [0, 1, 2, 4, 3, 5, 6, 7]
tot = v.sum()
per = tot / (2 * batch * 8 * n)  # per wave and CMUX step
print(f"batch {batch}, n {n}: {per:.0f} cycles per wave and step")
for q in order:
    print(f"  {names[q]:42s} {100 * v[q] / tot:5.1f} %  {v[q] / (2 * batch * 8 * n):8.0f}")
