"""World-size-2 gloo tests of the multi-GPU sharding logic (concrete_amd/dist.py).

No GPU here, so the per-rank PBS is the oracle (test infrastructure standing in for the HIP
kernel, which tests/test_gpu_pbs.py checks against the same oracle).  What is under test is
the host logic around it: shard ranges, the key broadcast and the final gather must give
exactly the single-process batch result, for even and ragged batches.
"""
import os
import socket

import numpy as np
import pytest

from concrete_amd.dist import shard_range


def test_shard_range_partitions():
    for total in (0, 1, 5, 8, 4096, 65536, 65537):
        for world in (1, 2, 3, 8):
            spans = [shard_range(total, world, r) for r in range(world)]
            assert spans[0][0] == 0
            for (s0, c0), (s1, _) in zip(spans, spans[1:]):
                assert s0 + c0 == s1
            assert sum(c for _, c in spans) == total
            assert max(c for _, c in spans) - min(c for _, c in spans) <= 1
    with pytest.raises(ValueError):
        shard_range(4, 2, 2)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, total, outdir):
    import torch
    import torch.distributed as dist

    from concrete_amd import dist as D
    from oracle import pyoracle as O

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        p = O.SMALL
        width = 2
        lwe_sk = O.binary_key(p.n, 11)
        glwe_sk = O.binary_key(p.big_n, 12)
        # key built on rank 0 only, then broadcast (rank 1 starts from garbage)
        flen = p.n * p.l * (p.k + 1) ** 2 * p.limbs * (p.N // 2) * 2
        if rank == 0:
            bsk = O.keygen_bsk(p, lwe_sk, glwe_sk, 13, std=2.0 ** -40)
            fkey = torch.from_numpy(O.bsk_to_fourier(p, bsk))
        else:
            fkey = torch.full((flen,), float("nan"), dtype=torch.float64)
        D.broadcast_key(fkey, src=0)
        # every rank derives the same batch, keeps only its shard
        rng = np.random.RandomState(7)
        msgs = rng.randint(0, 1 << width, size=total)
        table = np.array([3, 1, 0, 2], dtype=np.uint64)
        cts = O.lwe_encrypt_batch(lwe_sk, [O.encode(int(m), width) for m in msgs], p.n, 2.0 ** -30, 21)
        acc = O.trivial_glwe(p, O.expand_lut(table, p.N, width))
        s, c = D.shard_range(total, world, rank)
        out, _ = O.pbs_batch(p, cts[s:s + c], acc[None, :], fbsk=fkey.numpy(), nthreads=2)
        rows = torch.from_numpy(out.view(np.int64))
        full = D.gather_rows(rows, total, dst=0)
        if rank == 0:
            ref, _ = O.pbs_batch(p, cts, acc[None, :], fbsk=fkey.numpy(), nthreads=2)
            got = full.numpy().view(np.uint64)
            dec = O.lwe_decrypt_batch(glwe_sk, got, p.big_n)
            exact = np.array_equal(got, ref)
            lut_ok = [O.decode(int(d), width) for d in dec] == [int(table[m]) for m in msgs]
            with open(os.path.join(outdir, "result"), "w") as f:
                f.write(f"exact={exact} decrypt={lut_ok}")
        else:
            assert full is None
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("total", [6, 7])
def test_two_rank_shard_broadcast_gather(tmp_path, total, oracle):
    import torch.multiprocessing as mp

    mp.spawn(_worker, args=(2, _free_port(), total, str(tmp_path)), nprocs=2, join=True)
    assert (tmp_path / "result").read_text() == "exact=True decrypt=True"
