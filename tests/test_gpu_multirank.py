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
