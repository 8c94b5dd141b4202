"""PBS/s of every distinct (k, N, l, logB) shape of the optimizer's table at N <= 2048, on the kernel
the backend picks (its key format) and on the general path (concrete_hip_convert_bsk_generic +
concrete_hip_pbs_generic), at the largest n among the shape's rows; 2 rows checked bit-exact against
the oracle per run.  One process, one GPU.
Usage: python tools/row_census.py OUT.json [batch]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from concrete_amd import _native
from concrete_amd import backend as B
from oracle import pyoracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
out_path = sys.argv[1]
nb = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
rows = json.load(open(os.path.join(ROOT, "tests", "golden", "v0_last_128_rows.json")))["rows"]
shapes = {}
for r in rows:
    if r["N"] > 2048:
        continue
    key = (r["k"], r["N"], r["br_l"], r["br_b"])
    s = shapes.setdefault(key, {"rows": 0, "n": 0, "bits": set()})
    s["rows"] += 1
    s["n"] = max(s["n"], r["n"])
    s["bits"].add(r["bits"])
L = _native.lib()
dev = torch.device("cuda:0")
results = []


def timed(run):
    run()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(2):
        run()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / 2


for (k, N, l, logB), s in sorted(shapes.items(), key=lambda x: (x[0][1], x[0][0], x[0][2])):
    p = B.PbsParams(n=s["n"], k=k, N=N, level=l, base_log=logB)
    lwe_sk, glwe_sk = B.binary_key(p.n, 1), B.binary_key(p.big_n, 2)
    bsk = B.bsk_generate(p, lwe_sk, glwe_sk, 3)
    rng = np.random.RandomState(0)
    cts = B.lwe_encrypt(lwe_sk, [B.encode(m, 2) for m in rng.randint(0, 4, nb)], p.n, B.secure_std(1, p.n), 5)
    acc = B.trivial_glwe(p, B.expand_lut(np.arange(4, dtype=np.uint64), p.N, 2))
    d_in, d_lut = B.to_device(cts, "cuda:0"), B.to_device(acc[None, :], "cuda:0")
    ref, _ = O.pbs_batch(O.Params(n=p.n, k=k, N=N, l=l, logB=logB), cts[:2], acc[None, :], bsk=bsk,
                         mode=O.MODE_KARATSUBA)
    entry = {"k": k, "N": N, "l": l, "logB": logB, "n": p.n, "rows": s["rows"], "bits": sorted(s["bits"]),
             "format": B.bsk_format(p)[0], "batch": nb}
    fbsk = B.convert_bsk(p, bsk, "cuda:0")
    out = B.pbs(p, fbsk, d_in, d_lut)
    dt = timed(lambda: B.pbs(p, fbsk, d_in, d_lut, out=out))
    entry["pbs_per_s"] = round(nb / dt, 1)
    entry["bitexact_2"] = bool(np.array_equal(B.to_host(out)[:2], ref))
    del fbsk, out
    if entry["format"] != 3:  # a hand-tuned kernel: the general path on the same row for comparison
        st, gi = B._stream(dev), B._gpu_index(dev)
        g = torch.empty(L.concrete_hip_generic_bsk_size_bytes(p.n, k, l, N) // 8, dtype=torch.int64, device=dev)
        _native.check(L.concrete_hip_convert_bsk_generic(st, gi, B._ptr(g), bsk.ctypes.data, 0, p.n, k, l, N),
                      "convert_bsk_generic")
        og = torch.zeros((nb, p.lwe_out_size), dtype=torch.int64, device=dev)

        def run_gen():
            _native.check(L.concrete_hip_pbs_generic(st, gi, B._ptr(og), None, B._ptr(d_lut), None, B._ptr(d_in), None,
                                                     B._ptr(g), p.n, k, N, logB, l, nb, None), "pbs_generic")
        dtg = timed(run_gen)
        entry["general_path_pbs_per_s"] = round(nb / dtg, 1)
        entry["general_bitexact_2"] = bool(np.array_equal(B.to_host(og)[:2], ref))
        del g, og
    torch.cuda.empty_cache()
    results.append(entry)
    print(json.dumps(entry), flush=True)
json.dump({"note": "tools/row_census.py: every (k, N, l, logB) shape of v0_last_128 at N <= 2048, the largest n "
                   "of its rows, batch %d; format 3 = the general path" % nb, "shapes": results},
          open(out_path, "w"), indent=1)
