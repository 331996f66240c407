"""Patch-parallel execution over the GPUs of one node (one process per GPU).

The reference has no distributed code.  Images are independent
units, so a batch is split into contiguous per-rank shards and each rank runs the whole
encode -> decode on its own GPU with no exchange on the data path.  The only collectives
are the ones the workload itself asks for (BASELINE config 3):

* ``broadcast_weights`` -- the fp32 weights (3.25 MB) from rank 0, once at setup;
* ``gather_rows``       -- u8 latents / reconstructions / entropy values of every shard to
                           one rank (or all ranks) after the step, padded for ragged shards.

On ROCm ``torch.distributed``'s "nccl" backend is RCCL (over xGMI between MI355X GPUs);
the same code runs on "gloo" with CPU tensors, which is how tests/test_parallel.py covers
it without a GPU.
"""
from __future__ import annotations

from typing import Optional, Tuple

import numpy as np

from . import weights as W


def shard_range(n_total: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous [lo, hi) of rank ``rank``; the first n_total % world ranks get one extra."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} / world {world}")
    base, extra = divmod(n_total, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def _device_for(dist):
    import torch

    backend = dist.get_backend()
    if backend == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def broadcast_weights(weights: Optional[W.Weights], dist, src: int = 0) -> W.Weights:
    """Broadcast the full weight dict from ``src`` as one flat fp32 buffer (one collective)."""
    import torch

    keys = W.keys()
    shapes = [W.expected_shape(k) for k in keys]
    sizes = [int(np.prod(s)) for s in shapes]
    dev = _device_for(dist)
    flat = torch.empty(sum(sizes), dtype=torch.float32, device=dev)
    if dist.get_rank() == src:
        if weights is None:
            raise ValueError("source rank must hold the weights")
        W.validate(weights)
        flat.copy_(torch.from_numpy(np.concatenate([np.ascontiguousarray(weights[k]).ravel() for k in keys])))
    dist.broadcast(flat, src=src)
    host = flat.cpu().numpy()
    out, o = {}, 0
    for k, shp, n in zip(keys, shapes, sizes):
        out[k] = host[o:o + n].reshape(shp).copy()
        o += n
    return out


def gather_rows(local, n_total: int, dist, dst: Optional[int] = 0):
    """Gather per-rank shards (leading dim = shard rows, from :func:`shard_range`) into the
    full ``n_total``-row tensor on ``dst`` (or on every rank when dst is None).

    Equal-sized padded blocks (RCCL/gloo friendly), padding dropped afterwards.  With a
    single destination this is one ``gather``: only ``dst`` receives the world's blocks (an
    all_gather would move world-fold the bytes over xGMI, every other rank discarding them);
    ``dst=None`` is one ``all_gather``.  Returns None on non-destination ranks.
    """
    import torch

    world, rank = dist.get_world_size(), dist.get_rank()
    per = -(-n_total // world)
    lo, hi = shard_range(n_total, world, rank)
    if local.shape[0] != hi - lo:
        raise ValueError(f"rank {rank}: shard has {local.shape[0]} rows, expected {hi - lo}")
    block = torch.zeros((per,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    block[: hi - lo] = local
    if dst is None:
        blocks = [torch.empty_like(block) for _ in range(world)]
        dist.all_gather(blocks, block)
    else:
        blocks = [torch.empty_like(block) for _ in range(world)] if rank == dst else None
        dist.gather(block, gather_list=blocks, dst=dst)
        if rank != dst:
            return None
    parts = []
    for r in range(world):
        a, b = shard_range(n_total, world, r)
        parts.append(blocks[r][: b - a])
    return torch.cat(parts, dim=0)


def run_sharded(codec, x_local, n_total: int, dist, dst: Optional[int] = 0, entropy: bool = True):
    """BASELINE config 3 on one rank: encode -> decode (and histogram entropy) of this
    rank's shard on its own GPU, then the shards' u8 latents (N,h,w,96), u8 recons
    (N,8h,8w,3) and per-image entropy rows (N,3) gathered to ``dst`` in global order.

    ``codec`` is a :class:`codec.Codec` on this rank's device (or any object with the same
    encode / decode / entropy methods).  Returns (latents, recons, bits) on ``dst`` (bits is
    None without ``entropy``), (None, None, None) elsewhere."""
    z = codec.encode(x_local)
    r = codec.decode(z)
    n = x_local.shape[0]
    bits = codec.entropy(z).view(3, n).t().contiguous() if entropy else None  # plane-major -> (n, 3)
    zg = gather_rows(z, n_total, dist, dst)
    rg = gather_rows(r, n_total, dist, dst)
    bg = gather_rows(bits, n_total, dist, dst) if entropy else None
    return zg, rg, bg
