"""Two-rank rehearsal of bench.py's multi-GPU path on one GPU (gloo; ranks share cuda:0):
key built on rank 0 and broadcast, contiguous shards, barrier + max-over-ranks timing, final
gather — every row decrypts to LUT[m] and the sampled rows are bit-exact vs the oracle."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_bench_two_ranks():
    """The driver's default multi-GPU line: the metric's whole-node batch of 4096 split over the
    ranks (strong scaling), plus the weak-scaling secondary row (4096 per rank)."""
    env = dict(os.environ, CONCRETE_HIP_DIST_BACKEND="gloo")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "1", "--warmup", "1", "--no-cpu-baseline", "--no-ks", "--verify", "4"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["scaling"] == "strong"
    assert d["config"]["global_batch"] == 4096 and d["config"]["batch_per_gpu"] == 2048
    assert d["checks"]["decrypt_ok"] == "4096/4096"
    assert d["checks"]["bitexact"] is True
    w = d["secondary"]["weak_scaling"]
    assert w["batch_per_gpu"] == 4096 and w["value"] > 0


def test_bench_eight_ranks_configs2_shape():
    """BASELINE configs[2] rehearsed on one GPU: 8 gloo ranks (sharing cuda:0) bootstrap 8,192
    ciphertexts each (global batch 65,536); the key is built on rank 0 and broadcast; rank 0
    gathers the whole batch and checks it: every row decrypts to its rank's LUT[m] and two rows
    per rank are bit-exact vs the oracle."""
    env = dict(os.environ, CONCRETE_HIP_DIST_BACKEND="gloo", OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "8", "--steps", "1", "--warmup", "0", "--weak", "--batch", "8192", "--no-cpu-baseline", "--no-ks",
           "--verify", "2", "--check-gather"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 8 and d["config"]["global_batch"] == 65536
    assert d["checks"]["decrypt_ok"] == "65536/65536"
    g = d["checks"]["gather"]
    assert g["rows"] == 65536 and g["decrypt_ok"] == "65536/65536" and g["bitexact"] is True


RCCL_SCRIPT = r'''
import os, sys
import numpy as np
import torch, torch.distributed as dist
sys.path.insert(0, os.environ["REPO_ROOT"])
from dataclasses import replace
from concrete_amd import backend as B, dist as D
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", device_id=dev)
assert dist.get_backend() == "nccl" and dist.get_world_size() == 1
p = replace(B.CFG2, n=16)
lwe_sk, glwe_sk = B.binary_key(p.n, 11), B.binary_key(p.big_n, 12)
bsk = B.bsk_generate(p, lwe_sk, glwe_sk, 13)
ref_key = B.convert_bsk(p, bsk, dev)
key = torch.zeros_like(ref_key)
key.copy_(ref_key)
D.broadcast_key(key, src=0)                         # the RCCL broadcast of the device key
assert torch.equal(key, ref_key)
table = np.array([3, 1, 0, 2], dtype=np.uint64)
acc = B.trivial_glwe(p, B.expand_lut(table, p.N, 2))
msgs = np.arange(37) % 4
cts = B.lwe_encrypt(lwe_sk, [B.encode(m, 2) for m in msgs], p.n, 2.0 ** -25, 14)
start, count = D.shard_range(len(msgs), 1, 0)
out = B.pbs(p, key, B.to_device(cts[start:start + count], dev), B.to_device(acc[None, :], dev))
full = D.gather_rows(out, len(msgs), dst=0)         # the RCCL gather of the output rows
torch.cuda.synchronize()
got = B.to_host(full)
assert np.array_equal(got, B.to_host(out))
dec = B.lwe_decrypt(glwe_sk, got, p.big_n)
assert [B.decode(d, 2) for d in dec] == [int(table[m]) for m in msgs]
dist.destroy_process_group()
print("rccl ok")
'''


def test_rccl_collectives_single_rank(tmp_path):
    """The RCCL (backend "nccl") branch of concrete_amd/dist.py on hardware: one rank per GPU is all
    one box allows (RCCL refuses two ranks on one device), so world size 1 — the process group comes
    up on RCCL with device_id, the device key goes through broadcast_key and the outputs through
    gather_rows, and the gathered rows equal the PBS outputs and decrypt (the RCCL
    branch had run in no test).  The N > 1 data movement is covered by the gloo rehearsals above."""
    script = tmp_path / "rccl_one.py"
    script.write_text(RCCL_SCRIPT)
    env = dict(os.environ, REPO_ROOT=ROOT)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), str(script)]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "rccl ok" in r.stdout
