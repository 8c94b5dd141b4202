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
    env = dict(os.environ, CONCRETE_HIP_DIST_BACKEND="gloo")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "1", "--warmup", "1", "--batch", "256", "--no-cpu-baseline", "--no-ks",
           "--verify", "4"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["global_batch"] == 512
    assert d["checks"]["decrypt_ok"] == "512/512"
    assert d["checks"]["bitexact"] is True
