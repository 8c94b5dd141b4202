import os, sys, numpy as np
sys.path.insert(0, os.getcwd())
os.environ["CONCRETE_HIP_SDFG_TRACE"] = "1"
from dataclasses import replace
import tests.test_gpu_sdfg as T
from concrete_amd import backend as B, runtime as R
from oracle import pyoracle as O
p = replace(B.CFG2, n=24); nb = 10; width = 2
c = T._case(p, nb, 500, width)
pt = int(B.encode(1, width))
op = O.Params(n=p.n, k=p.k, N=p.N, l=p.level, logB=p.base_log, ks_l=p.ks_level, ks_logB=p.ks_base_log)
ks = R.Keyset(); ks.add_bsk(0, c["bsk"], p); ks.add_ksk(0, c["ksk"], p)
g = R.Dfg()
sx = g.batch_stream("x", R.TS_X86_TO_TOPO); sp = g.uint64_stream("p"); sxp = g.batch_stream("xp", R.TS_TOPO_TO_BOTH)
ssm = g.batch_stream("ks", R.TS_TOPO_TO_BOTH); sl = g.memref_stream("lut", R.TS_X86_TO_TOPO); sr = g.batch_stream("r1", R.TS_TOPO_TO_BOTH)
g.linear("add_pt_cst", sx, sp, sxp); g.keyswitch(sxp, ssm, p, ks.h); g.bootstrap(ssm, sl, sr, p, ks.h); g.run()
g.put_batch(sx, c["cts"]); g.put_uint64(sp, pt); g.put_memref(sl, c["luts"][0])
r1 = g.get_batch(sr, nb, p.big_n + 1)
xp1 = g.get_batch(sxp, nb, p.big_n + 1); ks1 = g.get_batch(ssm, nb, p.n + 1)
x2 = c["cts"][::-1].copy()
g.put_batch(sx, x2)
r3 = g.get_batch(sr, nb, p.big_n + 1)
xp3 = g.get_batch(sxp, nb, p.big_n + 1); ks3 = g.get_batch(ssm, nb, p.n + 1)
xpw = x2.copy(); xpw[:, -1] += np.uint64(pt)
print("xp3 ok", np.array_equal(xp3, xpw), "xp1 ok", np.array_equal(xp1[::-1], xpw))
print("ks3 ok", np.array_equal(ks3, O.keyswitch_batch(op, xpw, c["ksk"])), "ks1 rev", np.array_equal(ks1[::-1], ks3))
print("r3 == r1 rev", np.array_equal(r3, r1[::-1]), "r3==r1", np.array_equal(r3, r1))

print("rows eq xpw:", [bool(np.array_equal(xp3[i], xpw[i])) for i in range(nb)])
print("rows eq x2:", [bool(np.array_equal(xp3[i], x2[i])) for i in range(nb)])
print("rows eq xp1:", [bool(np.array_equal(xp3[i], xp1[i])) for i in range(nb)])
d = (xp3 != xpw); print("diff cols", np.nonzero(d.any(axis=0))[0][:20], d.sum())
print(xp3[0, -3:], xpw[0, -3:], xp1[0,-3:])
g.close(); ks.close()
