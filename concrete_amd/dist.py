"""Multi-GPU batch sharding for the batched PBS.

Ciphertexts of a batch are independent: each PBS reads its own LWE input, the shared LUT and
the shared bootstrapping key.  The reference's SDFG scheduler splits a batch into round-robin
chunks over the devices and uploads/converts the key once per device
(compiler lib/Runtime/GPUDFG.cpp:846-849, context.h:86-115).  Here one process drives one GPU
(torch.distributed, backend "nccl" = RCCL over xGMI):

  * shard_range   contiguous B/G shards (the first B mod G ranks get one extra ciphertext),
  * broadcast_key the device-format (Fourier) key is built once on the source rank and
                  broadcast, instead of G host uploads + G conversions,
  * gather_rows   the final gather of the (kN+1)-word output rows onto one rank.

There is no collective inside the PBS itself.  Everything here is plumbing over
torch.distributed; it runs unchanged on gloo (CPU tests) and nccl (GPU).
"""
from __future__ import annotations


def shard_range(total: int, world: int, rank: int) -> tuple[int, int]:
    """(start, count) of this rank's contiguous shard of a `total`-ciphertext batch."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} for world size {world}")
    if total < 0:
        raise ValueError("negative batch")
    base, extra = divmod(total, world)
    count = base + (1 if rank < extra else 0)
    start = rank * base + min(rank, extra)
    return start, count


def _host_staged(t, group) -> bool:
    """gloo collectives run on host tensors: device tensors are staged through host memory."""
    import torch.distributed as dist

    return t.is_cuda and dist.get_backend(group) == "gloo"


def broadcast_key(key, src: int = 0, group=None):
    """Broadcast the device-format key tensor from `src` in place (one RCCL broadcast)."""
    import torch.distributed as dist

    if _host_staged(key, group):
        h = key.cpu()
        dist.broadcast(h, src=src, group=group)
        key.copy_(h)
    else:
        dist.broadcast(key, src=src, group=group)
    return key


def gather_rows(rows, total: int, dst: int = 0, group=None):
    """Gather every rank's contiguous shard of output rows (shape (count, width)) onto `dst`.

    Returns the (total, width) tensor on `dst` (rows in batch order) and None elsewhere.
    Shards may be ragged (shard_range); they are padded to the largest shard for the
    collective and trimmed on the destination.
    """
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    width = rows.shape[1]
    start, count = shard_range(total, world, rank)
    if rows.shape[0] != count:
        raise ValueError(f"rank {rank}: {rows.shape[0]} rows, shard is {count}")
    cap = shard_range(total, world, 0)[1]
    device = rows.device
    if _host_staged(rows, group):
        rows = rows.cpu()
    buf = rows
    if count != cap:
        buf = torch.zeros((cap, width), dtype=rows.dtype, device=rows.device)
        buf[:count] = rows
    parts = [torch.empty_like(buf) for _ in range(world)] if rank == dst else None
    dist.gather(buf.contiguous(), gather_list=parts, dst=dst, group=group)
    if rank != dst:
        return None
    out = torch.empty((total, width), dtype=rows.dtype, device=device)
    for r in range(world):
        s, c = shard_range(total, world, r)
        out[s:s + c] = parts[r][:c]
    return out
