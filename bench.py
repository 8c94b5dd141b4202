"""Benchmark: batched programmable bootstrap (PBS) throughput on MI355X.

Workload = BASELINE.json metric config: N=1024, k=1, n=630, l=3, logB=7 (configs[1]'s
parameters) at the metric's batch of 4096.  A step = one batched PBS (one kernel launch per
rank) over resident LWE ciphertexts.  Multi-GPU = the metric's whole-node batch of 4096 split
into contiguous shards (strong scaling: 512 per GPU on 8 GPUs), with weak scaling (4096 per
GPU) measured as a secondary row; the device-format bootstrapping key is produced once on
rank 0 and broadcast over RCCL (xGMI); there is no collective in the data path.

Usage: python bench.py [--gpus N --steps K --warmup W]
       (N>1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
# FP64 vector peak: AMD's published MI355X figure (78.6 TFLOP/s; MI355X_MICROARCH.md has no FP64 row).
# The issue rate measured on gfx950 (~5 cycles per f64 wave-instruction per SIMD)
# puts the reachable ceiling near 256 CU x 4 SIMD x 64 lanes x 2 flop / 5 cycles x 2.4 GHz = 63 TFLOP/s.
FP64_PEAK_TFS = 78.6
# int8 matrix cores: v_mfma_i32_32x32x32_i8 runs the cycles of the BF16 form of the same M x N at twice
# the K, i.e. 2x the dense BF16 rate (MI355X_MICROARCH.md, Matrix cores: ~2.5 PF dense BF16)
I8_PEAK_TOPS = 5000.0
METRIC = "PBS/sec (whole node) at N=1024 batch=4096; achieved HBM GB/s"


# the sources a config's PMC record was measured on (a record is used only while they are unchanged)
KERNEL_HEADERS = ("concrete_amd/csrc/pbs.hpp", "concrete_amd/csrc/fft512.hpp", "concrete_amd/csrc/kernel_util.hpp",
                  "concrete_amd/csrc/common.hpp")
KERNEL_SOURCES = {"cfg2": ("concrete_amd/csrc/pbs.hip", "concrete_amd/csrc/pbs1024_hex.hip",
                           "concrete_amd/csrc/pbs_hex.hpp", "concrete_amd/csrc/Makefile") + KERNEL_HEADERS,
                  "cfg4": ("concrete_amd/csrc/pbs2048.hip",) + KERNEL_HEADERS,
                  "opt4": ("concrete_amd/csrc/pbs1024k2.hip",) + KERNEL_HEADERS,
                  "opt5": ("concrete_amd/csrc/pbs2048.hip",) + KERNEL_HEADERS,
                  **{c: ("concrete_amd/csrc/pbs_small.hip",) + KERNEL_HEADERS for c in ("opt1", "opt2", "opt3")}}


def _code_only(text: str) -> str:
    """C/C++ source without comments and whitespace (a comment edit does not change the kernel)."""
    import re
    text = re.sub(r"/\*.*?\*/", " ", text, flags=re.S)
    text = re.sub(r"//[^\n]*", " ", text)
    return "".join(text.split())


def kernel_source_hash(config: str = "cfg2") -> str:
    """Hash of the code (comments and whitespace stripped, round 5) of the sources a config's kernel
    is built from: a committed PMC record is used only while it matches."""
    import hashlib
    h = hashlib.sha1()
    for f in KERNEL_SOURCES.get(config, ("concrete_amd/csrc/pbs_generic.hip",) + KERNEL_HEADERS):
        with open(os.path.join(ROOT, f), encoding="utf-8") as fh:
            h.update(_code_only(fh.read()).encode())
    return h.hexdigest()[:16]


def pmc_records(config: str):
    """Committed PMC records (tools/pmc_record.py, older tools/pmc_traffic.py) measured on these
    kernel sources for this config, newest first."""
    import glob
    out = []
    files = glob.glob(os.path.join(ROOT, "profiles", "*_pmc.json")) + \
        glob.glob(os.path.join(ROOT, "profiles", "*_pbs_traffic.json"))
    for f in sorted(files, key=os.path.basename, reverse=True):
        with open(f) as fh:
            rec = json.load(fh)
        if rec.get("source_hash") == kernel_source_hash(config) and rec.get("config", "cfg2") == config:
            rec["src"] = os.path.relpath(f, ROOT)
            out.append(rec)
    return out


# environment overrides that change which kernels a call runs (A/B and diagnostic runs): a PMC
# record taken on the default dispatch does not describe them
DISPATCH_OVERRIDES = ("CONCRETE_HIP_LIB", "CONCRETE_HIP_GEN_COOP", "CONCRETE_HIP_GEN_FUSED", "CONCRETE_HIP_GEN_FUSEDY",
                      "CONCRETE_HIP_PBS_PAIRS", "CONCRETE_HIP_PBS_HEX")


def dispatch_overridden() -> bool:
    return any(os.environ.get(v) not in (None, "") for v in DISPATCH_OVERRIDES)


def pmc_traffic(batch: int, config: str, cus: int = 256):
    """Per-launch HBM bytes from a committed PMC record measured at this batch; else a record of the
    same kernel at another batch scaled by the batch ratio (the general path's rows at N >= 32768,
    whose profiler passes finish only at small batches: labelled as scaled); else None."""
    if dispatch_overridden():
        return None, None
    recs = [r for r in pmc_records(config) if "traffic_bytes" in r]
    for rec in recs:
        if rec.get("batch") == batch:
            return rec["traffic_bytes"], rec["src"]
    kern = dispatched_kernel(batch, config, cus)
    for rec in recs:
        if kern is not None and rec.get("kernel") == kern:
            return rec["traffic_bytes"] * batch / rec["batch"], rec["src"] + f" (scaled from batch {rec['batch']}, same kernel)"
    return None, None


def dispatched_kernel(batch: int, config: str, cus: int = 256):
    """The kernel (PMC record `kernel` field) that runs a whole call of `batch` ciphertexts, or None
    when the call is split over several kernels (cfg2: concrete_amd/csrc/pbs1024_plan.hpp)."""
    if config == "cfg2":
        import ctypes as C
        from concrete_amd import _native
        parts = (C.c_uint32 * 3)()
        _native.lib().concrete_hip_pbs1024_plan(batch, cus, parts)
        used = [k for k, x in zip(("pbs1024_pair", "pbs1024_hex", "pbs1024_hex"), parts) if x]
        return used[0] if len(set(used)) == 1 else None
    # the general path's records sum every gen_* launch of one call (the same launches at any batch)
    return PMC_KERNEL.get(config, "gen_* (sum over one PBS call)" if config.startswith("opt") else None)


# kernel-name substrings of the PMC records (tools/pmc_record.py KERNEL)
PMC_KERNEL = {"cfg4": "pbs2048", "opt5": "pbs2048", "opt4": "pbs1024k2", "opt1": "pbs_small", "opt2": "pbs_small",
              "opt3": "pbs_small"}


def pmc_f64_flop(batch: int, config: str, cus: int = 256):
    """f64 FLOP per launch from a committed PMC record (SQ f64 instruction mix).  A record at this
    batch is used as is; the work is per ciphertext, so a record at another batch is scaled by the
    batch ratio, but only when it was taken on the kernel this batch's call runs (cfg2
    runs the six-wave kernel at <= 2 x CUs, the pair kernel above, and a split between)."""
    if dispatch_overridden():
        return None, None
    recs = [r for r in pmc_records(config) if "f64_flop" in r]
    for rec in recs:
        if rec.get("batch") == batch:
            return rec["f64_flop"], rec["src"]
    kern = dispatched_kernel(batch, config, cus)
    for rec in recs:
        if kern is not None and rec.get("kernel") == kern:
            scale = batch / rec["batch"]
            return rec["f64_flop"] * scale, rec["src"] + f" (scaled from batch {rec['batch']}, same kernel)"
    return None, None


def pmc_ks_record(batch: int, config: str):
    """The keyswitch's PMC record at this batch (tools/pmc_record.py on the ks_mfma kernel): L2 (TCC)
    requests and HBM bytes per launch of the matrix-core kernel; None without one."""
    import glob
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_ks_pmc.json")), reverse=True):
        with open(f) as fh:
            rec = json.load(fh)
        if rec.get("batch") == batch and rec.get("config") == config + "_ks":
            out = {k: rec[k] for k in ("kernel", "traffic_bytes", "l2_bytes", "l2_read_requests", "l2_hit", "i8_ops",
                                       "mfma_busy") if k in rec}
            out["src"] = os.path.relpath(f, ROOT)
            return out
    return None


def ref_cost_model(p, pbs_per_s):
    """SURVEY.md §8(d) secondary compute figure: the reference optimizer's cost model of one PBS,
    n [(k+1) l (N log2 N + N) + (k+1) (N log2 N + N) + (k+1)^2 l N] operations (concrete-optimizer
    cmux.rs:31-50, pbs.rs:11-18; cfg2 64,512,000, cfg4 79,020,032), and the rate it implies."""
    import math
    k1, N, lg = p.k + 1, p.N, math.log2(p.N)
    ops = p.n * (k1 * p.level * (N * lg + N) + k1 * (N * lg + N) + k1 * k1 * p.level * N)
    return {"ops_per_pbs": int(ops), "achieved_gops": round(ops * pbs_per_s / 1e9, 1),
            "note": "the reference cost model's operation count (not this backend's exact-arithmetic work)"}


def host_cpus():
    """CPUs this process may use on this host: the affinity mask, capped by a cgroup CPU quota."""
    n_aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
    except Exception:
        pass
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except Exception:
        pass
    usable = n_aff if quota is None else max(1, min(n_aff, int(quota)))
    return {"nproc": os.cpu_count(), "affinity": n_aff, "cgroup_quota": quota, "usable": usable, "model": model}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--config", choices=("cfg2", "cfg4") + tuple(f"opt{b}" for b in range(1, 11)), default="cfg2",
                    help="cfg2: N=1024 n=630 l=3 logB=7 (the metric's config); cfg4: N=2048 n=742 l=1 logB=23; "
                         "optB: the optimizer's B-bit row of v0_last_128 (backend.OPTIMIZER_SETS)")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=4096, help="PBS per GPU per step (weak scaling: --weak)")
    ap.add_argument("--global-batch", type=int, default=0,
                    help="strong scaling: this many PBS per step for the whole job, split over the ranks "
                         "(default for cfg2: the metric's whole-node batch 4096, i.e. 512 per GPU on 8 GPUs)")
    ap.add_argument("--weak", action="store_true",
                    help="weak scaling as the main line: --batch PBS per GPU (cfg2 N>1 reports it as "
                         "secondary.weak_scaling anyway)")
    ap.add_argument("--cpu-sample", type=int, default=0,
                    help="PBS in the bounded CPU-baseline sample (default: cfg2 4096 = one full batch, "
                         "cfg4 1024; ~10-20 s)")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="threads of the CPU baseline (default: every CPU this job may use on the host)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--verify", type=int, default=8, help="rows checked bit-exactly against the oracle (rank 0)")
    ap.add_argument("--no-ks", action="store_true", help="skip the secondary keyswitch measurement")
    ap.add_argument("--no-share", action="store_true",
                    help="skip the secondary B = 512 row (the whole-node metric's per-GPU batch on 8 GPUs)")
    ap.add_argument("--no-sdfg", action="store_true", help="skip the stream-emulator (SDFG route) measurement")
    ap.add_argument("--no-e2e", action="store_true",
                    help="skip the PCIe-inclusive leg (PMC passes: exactly warmup + steps PBS calls per process)")
    ap.add_argument("--check-gather", action="store_true",
                    help="rank 0 checks the whole gathered batch: every row decrypts to its rank's LUT[m], and "
                         "two rows per rank are bit-exact vs the oracle (inputs regenerated from the seeds)")
    return ap.parse_args()




def _progress(msg: str) -> None:
    """Stage marks on stderr when CONCRETE_BENCH_PROGRESS=1 (long profiler passes show where they are)."""
    if os.environ.get("CONCRETE_BENCH_PROGRESS") == "1":
        print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    from concrete_amd import backend as B
    from concrete_amd import dist as D

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    # The metric is "PBS/sec (whole node) at N=1024 batch=4096": for cfg2 the job's batch is 4096
    # however many GPUs share it (strong scaling, BASELINE.json); weak scaling (4096 per GPU) is
    # measured as a secondary row on N > 1.
    if args.global_batch == 0 and args.config == "cfg2" and not args.weak:
        args.global_batch = 4096
    strong = args.global_batch > 0
    if strong:
        # contiguous shards of the job's batch (the first global % world ranks get one more)
        base, extra = divmod(args.global_batch, world)
        args.batch = base + (1 if rank < extra else 0)
        if args.batch == 0:
            raise SystemExit(f"--global-batch {args.global_batch} leaves rank {rank} without work")
    # one process per GPU; CONCRETE_HIP_DIST_BACKEND=gloo rehearses N ranks on fewer GPUs
    backend = os.environ.get("CONCRETE_HIP_DIST_BACKEND", "nccl")
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    if args.config.startswith("opt"):
        width = int(args.config[3:])
        p = B.OPTIMIZER_SETS[width]
    else:
        p = B.CFG2 if args.config == "cfg2" else B.CFG4
        width = 3 if args.config == "cfg2" else 5
    if not args.cpu_sample:
        # about 10-30 s of CPU work on 16 host cores (fft64 restatement, OpenMP over ciphertexts)
        args.cpu_sample = {"cfg2": 4096, "cfg4": 1024}.get(
            args.config, 512 if p.N <= 1024 else 128 if p.N <= 4096 else 32 if p.N <= 16384 else 4)
    # ---- keys: deterministic synthetic keyset (product keygen); device key on rank 0 -> RCCL bcast
    lwe_sk = B.binary_key(p.n, 1)
    glwe_sk = B.binary_key(p.big_n, 2)
    fbytes = B.fourier_bsk_bytes(p)
    t0 = time.perf_counter()
    if rank == 0:
        _progress("keygen")
        bsk = B.bsk_generate(p, lwe_sk, glwe_sk, 3)
        _progress("key conversion")
        fbsk = B.convert_bsk(p, bsk, dev)
        _progress("key converted")
    else:
        bsk = None
        fbsk = torch.empty(fbytes // 8, dtype=torch.int64, device=dev)
    torch.cuda.synchronize()
    t_key = time.perf_counter() - t0
    t_bcast = 0.0
    if world > 1:
        dist.barrier()
        t0 = time.perf_counter()
        D.broadcast_key(fbsk, src=0)
        torch.cuda.synchronize()
        t_bcast = time.perf_counter() - t0

    # ---- this rank's shard: fresh encryptions of random `width`-bit messages, one LUT per rank
    def shard_inputs(r, count):
        rng = np.random.RandomState(1000 + r)
        table = rng.randint(0, 1 << width, size=1 << width).astype(np.uint64)
        msgs = rng.randint(0, 1 << width, size=count)
        cts = B.lwe_encrypt(lwe_sk, [B.encode(m, width) for m in msgs], p.n, B.secure_std(1, p.n), 5000 + r)
        return table, msgs, cts

    table, msgs, cts = shard_inputs(rank, args.batch)
    acc = B.trivial_glwe(p, B.expand_lut(table, p.N, width))
    d_in = B.to_device(cts, dev)
    d_lut = B.to_device(acc[None, :], dev)
    d_out = torch.empty((args.batch, p.lwe_out_size), dtype=torch.int64, device=dev)

    def step():
        B.pbs(p, fbsk, d_in, d_lut, out=d_out)

    _progress("warm-up")
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    _progress("timed steps")
    # kernel events on the stream the kernels are launched on (torch's current stream)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    t0 = time.perf_counter()
    for i in range(args.steps):
        ev[i][0].record()
        step()
        ev[i][1].record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    kern_each = [a.elapsed_time(b) for a, b in ev]
    kern_ms = float(np.mean(kern_each))
    kern_med = float(np.median(kern_each))  # the median of the timed reps too
    total_done = args.batch * args.steps
    if world > 1:
        t = torch.tensor([wall, kern_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        wall, kern_ms = float(t[0]), float(t[1])
        t = torch.tensor([total_done, args.batch], dtype=torch.int64, device=dev)
        dist.all_reduce(t)
        total_done, global_batch = int(t[0]), int(t[1])
    else:
        global_batch = args.batch

    # ---- weak scaling (cfg2, N > 1): every rank its own full batch of 4096, same timing rule
    weak_res = None
    if strong and world > 1 and args.config == "cfg2" and not args.weak:
        _, _, cts_w = shard_inputs(rank, 4096)
        d_in_w = B.to_device(cts_w, dev)
        d_out_w = torch.empty((4096, p.lwe_out_size), dtype=torch.int64, device=dev)
        for _ in range(args.warmup):
            B.pbs(p, fbsk, d_in_w, d_lut, out=d_out_w)
        torch.cuda.synchronize()
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            B.pbs(p, fbsk, d_in_w, d_lut, out=d_out_w)
        torch.cuda.synchronize()
        dist.barrier()
        torch.cuda.synchronize()
        t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        weak_res = {"metric": f"PBS/sec (whole node), 4096 per GPU ({4096 * world} per step)",
                    "value": round(4096 * world * args.steps / float(t[0]), 1), "unit": "PBS/s",
                    "ms_per_step": round(float(t[0]) / args.steps * 1e3, 3), "batch_per_gpu": 4096,
                    "scaling": "weak"}
        del d_in_w, d_out_w

    # ---- the whole-node metric's per-GPU share (cfg2, one GPU): 4096 / 8 = 512 ciphertexts, what each
    #      of 8 GPUs runs in the strong-scaling 8-GPU job (the six-wave kernel's batch);
    #      timed the same way on this GPU, its 8x is a projection, not an 8-GPU measurement
    share_res = None
    if world == 1 and args.config == "cfg2" and strong and args.global_batch == 4096 and not args.no_share:
        nb_s = 512
        d_out_s = torch.empty((nb_s, p.lwe_out_size), dtype=torch.int64, device=dev)
        d_in_s = d_in[:nb_s]
        for _ in range(max(2, args.warmup)):
            B.pbs(p, fbsk, d_in_s, d_lut, out=d_out_s)
        torch.cuda.synchronize()
        sev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(10)]
        t0 = time.perf_counter()
        for a_, b_ in sev:
            a_.record()
            B.pbs(p, fbsk, d_in_s, d_lut, out=d_out_s)
            b_.record()
        torch.cuda.synchronize()
        wall_s = time.perf_counter() - t0
        kms_s = float(np.mean([a_.elapsed_time(b_) for a_, b_ in sev]))
        same = bool(np.array_equal(B.to_host(d_out_s), B.to_host(d_out[:nb_s])))
        share_res = {"metric": "PBS/sec per GPU at the whole-node metric's per-GPU batch (4096 / 8 GPUs = 512)",
                     "value": round(nb_s * len(sev) / wall_s, 1), "unit": "PBS/s", "batch": nb_s,
                     "ms_per_step": round(wall_s / len(sev) * 1e3, 3), "kernel_ms": round(kms_s, 3),
                     "projected_8gpu_whole_node": round(8 * nb_s * len(sev) / wall_s, 1),
                     "outputs_equal_full_batch_rows": same,
                     "note": "timed on this GPU; the 8-GPU figure is 8x this rate (independent shards, no "
                             "data-path collective), a projection, not a measurement"}
        del d_out_s

    # ---- secondary row: batched keyswitch kN -> n of this batch, after the PBS
    ks_res = None
    if not args.no_ks:
        ksk = B.ksk_generate(p, glwe_sk, lwe_sk, 6)
        # allocated the runtime's way (cuda_malloc_async, context.h:134-139): the int8 key bytes of
        # the matrix-core path are then built once and reused across calls
        d_ksk = B.RuntimeBuffer(ksk, gpu=local)
        d_small = torch.empty((args.batch, p.n + 1), dtype=torch.int64, device=dev)
        for _ in range(max(1, args.warmup)):
            B.keyswitch(p, d_ksk, d_out, out=d_small)
        torch.cuda.synchronize()
        kev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
        for a_, b_ in kev:
            a_.record()
            B.keyswitch(p, d_ksk, d_out, out=d_small)
            b_.record()
        torch.cuda.synchronize()
        ks_ms = float(np.mean([a_.elapsed_time(b_) for a_, b_ in kev]))
        ks_bytes = 8 * (p.ksk_len + p.lwe_out_size + p.lwe_in_size)  # SURVEY.md §8d per-KS figure
        # One launch reads the shared KSK once plus every row in and out: the unique bytes per
        # launch.  The per-KS figure x batch would exceed the HBM peak (KSK rows are shared by all
        # ciphertexts of a tile), so the roofline is priced on unique bytes; the kernel is bound by
        # its digit x key-word integer products, not by HBM.
        ks_launch_bytes = 8 * (p.ksk_len + args.batch * (p.lwe_out_size + p.lwe_in_size))
        ks_rate = args.batch / (ks_ms * 1e-3)
        ks_gbs = ks_launch_bytes / (ks_ms * 1e-3) / 1e9
        # the keyswitch as int8 matrix products: out = (0..b) - sum_c 2^(8c) D K_c over the
        # 8 byte chunks of every KSK word, D the batch x (kN l) digit matrix: 2 ops per multiply-add
        ks_ops = 2.0 * 8 * args.batch * (p.big_n * p.ks_level) * (p.n + 1)
        ks_ks = pmc_ks_record(args.batch, args.config)
        ks_mfma = {"achieved": round(ks_ops / (ks_ms * 1e-3) / 1e12, 1), "peak": I8_PEAK_TOPS, "unit": "TOP/s",
                   "frac": round(ks_ops / (ks_ms * 1e-3) / 1e12 / I8_PEAK_TOPS, 4), "ops_per_call": ks_ops,
                   "note": "algorithmic int8 multiply-adds x 2 (8 byte chunks x batch x kN l x (n + 1)) / the whole "
                           "call's time (digit kernel + matrix-core kernel); peak = 2x dense BF16 (I8 MFMA rate)"}
        if ks_ks:
            ks_mfma["pmc"] = ks_ks
        ks_res = {"metric": f"KS/sec per GPU at kN={p.big_n} -> n={p.n}, l={p.ks_level} logB={p.ks_base_log}",
                  "value": round(ks_rate, 1), "unit": "KS/s", "kernel_ms": round(ks_ms, 4),
                  # not HBM-bound: the unique bytes per launch are a small fraction of the peak, so
                  # no HBM fraction is claimed
                  "hbm": {"achieved": round(ks_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                          "bytes_per_launch": ks_launch_bytes, "bytes_per_ks_8d": ks_bytes,
                          "note": "unique bytes per launch (the KSK once + every row in and out)"},
                  "bound": "mfma", "mfma": ks_mfma}
        if rank == 0 and args.verify:
            from oracle import pyoracle as O
            op = O.Params(n=p.n, k=p.k, N=p.N, l=p.level, logB=p.base_log, ks_l=p.ks_level, ks_logB=p.ks_base_log)
            rows = B.to_host(d_out[: args.verify])
            ks_res["bitexact"] = bool(np.array_equal(B.to_host(d_small[: args.verify]),
                                                     O.keyswitch_batch(op, rows, ksk)))
        d_ksk.free()
        del d_ksk, d_small

    # ---- end-to-end including PCIe: host inputs -> H2D -> PBS -> D2H -> host outputs (DESIGN.md §6;
    # never `value`, which is the device-resident rate)
    e2e = None
    if not args.no_e2e:
        h_in = torch.from_numpy(cts.view(np.int64)).pin_memory()
        h_out = torch.empty((args.batch, p.lwe_out_size), dtype=torch.int64).pin_memory()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            d_in.copy_(h_in, non_blocking=True)
            step()
            h_out.copy_(d_out, non_blocking=True)
        torch.cuda.synchronize()
        e2e = args.batch * args.steps / (time.perf_counter() - t0)

    # ---- the circuit-facing SDFG route (the default GPU route of a compiled circuit,
    # stream_emulator_*): a KS -> PBS table lookup on host memrefs, timed end to end per run (put
    # the batch, get the outputs: H2D, keyswitch, bootstrap, D2H, intermediates resident in HBM)
    sdfg_res = None
    if world == 1 and args.config == "cfg2" and not args.no_ks and not args.no_sdfg:
        from concrete_amd import runtime as R
        width_s = 2  # KS -> PBS chains keep p <= 2 at the cfg2 keyswitch noise
        table_s = np.array([3, 0, 2, 1], dtype=np.uint64)
        rng_s = np.random.RandomState(17)
        msgs_s = rng_s.randint(0, 1 << width_s, size=args.batch)
        big_in = B.lwe_encrypt(glwe_sk, [B.encode(m, width_s) for m in msgs_s], p.big_n, 2.0 ** -30, 18)
        kset = R.Keyset([local])
        kset.add_bsk(0, bsk if bsk is not None else B.bsk_generate(p, lwe_sk, glwe_sk, 3), p)
        kset.add_ksk(0, ksk, p)
        ctx = 0x5DF6  # the RuntimeContext pointer a circuit would pass (bound, never dereferenced)
        kset.bind(ctx)
        g = R.Dfg()
        s_in = g.batch_stream("in", R.TS_X86_TO_TOPO)
        s_lut = g.memref_stream("lut", R.TS_X86_TO_TOPO)
        s_mid = g.batch_stream("mid")
        s_res = g.batch_stream("out", R.TS_TOPO_TO_X86)
        g.keyswitch(s_in, s_mid, p, ctx)
        g.bootstrap(s_mid, s_lut, s_res, p, ctx)
        g.run()
        g.put_memref(s_lut, B.expand_lut(table_s, p.N, width_s))
        g.put_batch(s_in, big_in)
        res = g.get_batch(s_res, args.batch, p.lwe_out_size)  # warm-up: device keys, buffers
        t0 = time.perf_counter()
        for _ in range(args.steps):
            g.put_batch(s_in, big_in)
            res = g.get_batch(s_res, args.batch, p.lwe_out_size, out=res)  # the caller's output memref
        sdfg_s = (time.perf_counter() - t0) / args.steps
        dec_s = B.lwe_decrypt(glwe_sk, res, p.big_n)
        ok_s = int(sum(B.decode(d, width_s) == int(table_s[m]) for d, m in zip(dec_s, msgs_s)))
        sdfg_res = {"metric": "KS -> PBS table lookups/sec through stream_emulator_* (host memrefs in and out)",
                    "value": round(args.batch / sdfg_s, 1), "unit": "TLU/s", "ms_per_run": round(sdfg_s * 1e3, 3),
                    "decrypt_ok": f"{ok_s}/{args.batch}"}
        g.close()
            # the direct route (memref_batched_bootstrap_lwe_*_u64, wrappers.cpp:164-256): host rows in,
        # host rows out, on the same keyset, into one caller-owned output memref reused across calls
        # (a fresh 33.6 MB array per call is unmapped the next call, and in this process that stalls
        # the GPU queue ~25 ms on alternate calls: DESIGN.md §7)
        tlu_d = B.expand_lut(table, p.N, width)
        res_d = R.batched_bootstrap(kset, p, cts, tlu_d)  # warm-up
        if os.environ.get("CONCRETE_HIP_BENCH_TIMELINE"):
            kset.set_timing(True)
        t0 = time.perf_counter()
        for _ in range(args.steps):
            t_call = time.perf_counter()
            res_d = R.batched_bootstrap(kset, p, cts, tlu_d, out=res_d)
            if os.environ.get("CONCRETE_HIP_BENCH_TIMELINE"):
                print("direct route timeline (dev, start, in, kernel, out, n):", kset.timeline().round(3).tolist(),
                      f"call wall {1e3 * (time.perf_counter() - t_call):.2f} ms", file=sys.stderr, flush=True)
        direct_s = (time.perf_counter() - t0) / args.steps
        dec_d = B.lwe_decrypt(glwe_sk, res_d, p.big_n)
        ok_d = int(sum(B.decode(d, width) == int(table[m]) for d, m in zip(dec_d, msgs)))
        sdfg_res["direct_route"] = {"metric": "PBS/sec through memref_batched_bootstrap_lwe_*_u64 (host memrefs)",
                                    "value": round(args.batch / direct_s, 1), "unit": "PBS/s",
                                    "ms_per_call": round(direct_s * 1e3, 3), "decrypt_ok": f"{ok_d}/{args.batch}"}
        kset.close()

    # ---- final gather of the output rows onto rank 0 (outside the timed PBS region)
    t_gather = 0.0
    gather_check = None

    def check_gather(rows, world_, total):
        """Every gathered row decrypts to its rank's LUT[m]; two rows per rank bit-exact (oracle)."""
        from concrete_amd.dist import shard_range
        from oracle import pyoracle as O  # checker only, after the timed region
        op = O.Params(n=p.n, k=p.k, N=p.N, l=p.level, logB=p.base_log, limbs=O.limbs_for(p.N))
        key = B.bsk_generate(p, lwe_sk, glwe_sk, 3) if bsk is None else bsk
        fcpu = O.bsk_to_fourier(op, key)
        dec_ok, exact = 0, True
        for r in range(world_):
            start, count = shard_range(total, world_, r)
            tab_r, msgs_r, cts_r = shard_inputs(r, count)
            mine = rows[start:start + count]
            dec = B.lwe_decrypt(glwe_sk, mine, p.big_n)
            dec_ok += sum(int(B.decode(d, width) == tab_r[m]) for d, m in zip(dec, msgs_r))
            pick = np.array([0, count - 1])
            acc_r = B.trivial_glwe(p, B.expand_lut(tab_r, p.N, width))
            ref, _ = O.pbs_batch(op, cts_r[pick], acc_r[None, :], fbsk=fcpu)
            exact &= bool(np.array_equal(ref, mine[pick]))
        return {"rows": int(rows.shape[0]), "decrypt_ok": f"{dec_ok}/{total}", "bitexact_rows": 2 * world_,
                "bitexact": exact}
    if world > 1:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        full = D.gather_rows(d_out, global_batch, dst=0)
        torch.cuda.synchronize()
        t_gather = time.perf_counter() - t0
        if rank == 0 and args.check_gather:
            gather_check = check_gather(B.to_host(full), world, global_batch)
        del full

    # ---- correctness of what was timed: decrypt-level on every row, bit-exact sample (rank 0)
    out = B.to_host(d_out)
    dec = B.lwe_decrypt(glwe_sk, out, p.big_n)
    ok = sum(int(B.decode(d, width) == table[m]) for d, m in zip(dec, msgs))
    ok_all = ok
    if world > 1:
        t = torch.tensor([ok], dtype=torch.int64, device=dev)
        dist.all_reduce(t)
        ok_all = int(t.item())
    cpu_threads = args.cpu_threads or host_cpus()["usable"]

    result = None
    if rank == 0:
        value = total_done / wall
        bytes_per_pbs = p.bsk_bytes_per_pbs()
        achieved = bytes_per_pbs * args.batch / (kern_ms * 1e-3) / 1e9
        bitexact = None
        cpu = None
        traffic, traffic_src = pmc_traffic(args.batch, args.config,
                                           torch.cuda.get_device_properties(dev).multi_processor_count)
        flop, flop_src = pmc_f64_flop(args.batch, args.config,
                                      torch.cuda.get_device_properties(dev).multi_processor_count)
        kern_s = kern_ms * 1e-3
        valu = None if flop is None else {
            "achieved": round(flop / kern_s / 1e12, 2), "peak": FP64_PEAK_TFS, "unit": "TFLOP/s",
            "frac": round(flop / kern_s / 1e12 / FP64_PEAK_TFS, 4), "f64_flop_per_launch": flop, "src": flop_src,
            "note": "f64 FLOP = 64 x (2 FMA + ADD + MUL) wave-instructions (SQ_INSTS_VALU_*_F64) per launch / "
                    "kernel time; peak = AMD's FP64 vector figure (~63 TFLOP/s at the measured issue rate)"}
        dram = None if traffic is None else {
            "achieved": round(traffic / kern_s / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(traffic / kern_s / 1e9 / HBM_PEAK_GBS, 4),
            "note": "measured DRAM bytes (roofline.traffic) per launch / kernel time"}
        # the CPU baseline is timed at N = 1 only (a reported baseline, not part of the scaling runs)
        cpu_leg = not args.no_cpu_baseline and world == 1
        if args.verify or cpu_leg:
            from oracle import pyoracle as O  # checker / CPU baseline only
            opt = args.config.startswith("opt")
            if bsk is None:
                bsk = B.bsk_generate(p, lwe_sk, glwe_sk, 3)
            if opt:
                # optimizer rows: the oracle's pure-integer Karatsuba product (exact for every row;
                # its limb-FFT path is tuned to cfg2/cfg4), on the standard key
                op = O.Params(n=p.n, k=p.k, N=p.N, l=p.level, logB=p.base_log)
                kw = {"bsk": bsk, "mode": O.MODE_KARATSUBA}
                desc = "pure-integer Karatsuba restatement"
            else:
                op = O.Params(n=p.n, k=p.k, N=p.N, l=p.level, logB=p.base_log, limbs=O.limbs_for(p.N))
                kw = {"fbsk": O.bsk_to_fourier(op, bsk)}
                desc = f"exact-limb f64 FFT restatement, {op.limbs} limbs"
            if args.verify:
                ref, _ = O.pbs_batch(op, cts[: args.verify], acc[None, :], nthreads=cpu_threads, **kw)
                bitexact = bool(np.array_equal(ref, out[: args.verify]))
            if cpu_leg:
                sample = cts[: args.cpu_sample]
                # the reference's own arithmetic for every config (concrete-cpu's fft64: one f64
                # spectrum of the u64 key, f64 products rounded mod 2^64, output noise in the low
                # bits), not the exact limb split the GPU and the checker use
                op = O.Params(n=p.n, k=p.k, N=p.N, l=p.level, logB=p.base_log, limbs=1)
                kw = {"fbsk": O.bsk_to_fourier(op, bsk), "mode": O.MODE_FFT64}
                desc = ("fft64 arithmetic restated: one f64 key spectrum, f64 products rounded mod 2^64 "
                        "(radix-2 FFT, not concrete-fft's SIMD kernels)")
                t1 = time.perf_counter()
                O.pbs_batch(op, sample, acc[None, :], nthreads=cpu_threads, **kw)
                dt = time.perf_counter() - t1
                hc = host_cpus()
                cpu = {"value": round(len(sample) / dt, 2), "unit": "PBS/s", "cores": cpu_threads,
                       "kind": "port",
                       "label": f"concrete-cpu semantics, restated: {desc}",
                       "host": hc,
                       "sample": f"{len(sample)} PBS of the same {args.config} workload ({desc}, OpenMP over "
                                 f"ciphertexts on {cpu_threads} threads = every CPU this job may use: affinity "
                                 f"{hc['affinity']}, cgroup quota {hc['cgroup_quota']}, nproc {hc['nproc']}), "
                                 f"{dt:.2f} s wall"}
        result = {
            "metric": METRIC if args.config == "cfg2" else f"PBS/sec (whole node) at N={p.N} batch={global_batch}",
            "value": round(value, 1),
            "unit": "PBS/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(wall / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None,
            "dtype": "u64",
            "data": f"synthetic (seeded keygen + fresh LWE encryptions of random {width}-bit messages)",
            "config": {"workload": f"batched PBS {args.config}: N={p.N} k={p.k} n={p.n} l={p.level} logB={p.base_log}",
                       "batch_per_gpu": args.batch, "global_batch": global_batch,
                       "parallelism": f"shard{world}", "key_bcast_s": round(t_bcast, 4), "gather_s": round(t_gather, 4),
                       "key_convert_s": round(t_key, 3)},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_src": traffic_src,
                         "kernel_ms": round(kern_ms, 3), "kernel_ms_median": round(kern_med, 3),
                         "bytes_per_pbs": bytes_per_pbs, "dram": dram, "valu": valu,
                         "ref_cost_model": ref_cost_model(p, value)},
            "cpu_baseline": cpu,
            "secondary": {"keyswitch": ks_res, "sdfg_route": sdfg_res, "weak_scaling": weak_res,
                          "whole_node_share_b512": share_res,
                          "pcie_inclusive_pbs_per_s": None if e2e is None else round(e2e * world, 1)},
            "checks": {"decrypt_ok": f"{ok_all}/{global_batch}", "bitexact_rows": args.verify, "gather": gather_check,
                       "bitexact": bitexact},
        }
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return result


if __name__ == "__main__":
    main()
