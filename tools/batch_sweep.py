"""cfg2 batch sweep: PBS/s at B = 256 .. 4096 in steps of 256 on one GPU for the
default dispatch (the planner's split over the pair and six-wave kernels, pbs1024_plan.hpp) beside
each single-kernel choice (the pair kernel forced, the six-wave kernel forced at 2 per workgroup).
Every B's outputs are checked equal to the same rows of the B = 4096 run.  Kernel time from HIP
events around `--reps` calls after one warm-up call.

    python tools/batch_sweep.py --out gpurun_out/r06c/batch_sweep.json
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--step", type=int, default=256)
    ap.add_argument("--max", type=int, default=4096)
    args = ap.parse_args()
    import torch
    from concrete_amd import _native
    from concrete_amd import backend as B
    L = _native.lib()
    p = B.CFG2
    dev = "cuda:0"
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    t0 = time.time()
    lwe_sk = B.binary_key(p.n, 900)
    glwe_sk = B.binary_key(p.big_n, 901)
    bsk = B.bsk_generate(p, lwe_sk, glwe_sk, 902)
    fbsk = B.convert_bsk(p, bsk, dev)
    width = 3
    table = np.arange(8, dtype=np.uint64)[::-1].copy()
    acc = B.trivial_glwe(p, B.expand_lut(table, p.N, width))
    rng = np.random.RandomState(903)
    msgs = rng.randint(0, 8, size=args.max)
    cts = B.lwe_encrypt(lwe_sk, [B.encode(m, width) for m in msgs], p.n, B.secure_std(1, p.n), 904)
    d_in = B.to_device(cts, dev)
    d_acc = B.to_device(acc[None, :], dev)
    out = torch.zeros((args.max, p.lwe_out_size), dtype=torch.int64, device=dev)
    torch.cuda.synchronize()
    print(f"setup {time.time() - t0:.1f} s, {cus} CUs", flush=True)

    def run(nb, env):
        old = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        try:
            o = out[:nb]
            B.pbs(p, fbsk, d_in[:nb], d_acc, out=o)
            torch.cuda.synchronize()
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            ev[0].record()
            for _ in range(args.reps):
                B.pbs(p, fbsk, d_in[:nb], d_acc, out=o)
            ev[1].record()
            torch.cuda.synchronize()
            ms = ev[0].elapsed_time(ev[1]) / args.reps
            return ms, B.to_host(o)
        finally:
            for k, v in old.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v

    _, full = run(args.max, {})
    dec = B.lwe_decrypt(glwe_sk, full, p.big_n)
    assert [B.decode(d, width) for d in dec] == [int(table[m]) for m in msgs], "B = max does not decrypt"
    rows = []
    for nb in range(args.step, args.max + 1, args.step):
        parts = (C.c_uint32 * 3)()
        L.concrete_hip_pbs1024_plan(nb, cus, parts)
        rec = {"batch": nb, "plan": {"pair": parts[0], "hex2": parts[1], "hex1": parts[2]}}
        for name, env in (("dispatch", {}), ("pair_only", {"CONCRETE_HIP_PBS_PAIRS": "4"}),
                          ("hex_only", {"CONCRETE_HIP_PBS_HEX": "2"})):
            ms, got = run(nb, env)
            assert np.array_equal(got, full[:nb]), (nb, name)
            rec[name] = {"ms": round(ms, 3), "pbs_per_s": round(nb / ms * 1e3, 1)}
        rows.append(rec)
        print(json.dumps(rec), flush=True)
    top = rows[-1]["dispatch"]["pbs_per_s"]
    for r in rows:
        r["dispatch"]["frac_of_max_batch"] = round(r["dispatch"]["pbs_per_s"] / top, 4)
    res = {"config": "cfg2 N=1024 k=1 n=630 l=3 logB=7", "cus": cus, "reps": args.reps,
           "note": "kernel time per call from HIP events; every batch's outputs equal the B = max run's rows",
           "rows": rows}
    os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
    with open(args.out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
