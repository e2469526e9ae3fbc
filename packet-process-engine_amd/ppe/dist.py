"""Batch sharding across ranks (one process per GPU).

The stateless decode + classify path shards without any data-path exchange: rank r owns the contiguous packet
range shard_range(n, world, r); results are only gathered for the consumer.  The reference's own
scale-out is the same shape: Octeon hardware steers packets to cores, each core runs to completion with per-core
counters (dataplane/src/platform/oct-init.c:133-155, main.c:250).  Counters are summed across ranks, exactly as
dp_show_pkt_stat sums the per-core pktstat[] (dataplane/src/common/dp_cmd.c:844).
"""
from __future__ import annotations

import numpy as np


def shard_range(n: int, world: int, rank: int) -> tuple[int, int]:
    """[lo, hi) of rank's contiguous, tile-aligned shard; sizes differ by at most one tile plus the partial tail."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    tiles = (n + 63) // 64
    per, extra = divmod(tiles, world)
    t0 = rank * per + min(rank, extra)
    t1 = t0 + per + (1 if rank < extra else 0)
    return min(n, t0 * 64), min(n, t1 * 64)


def gather_results(dist, local: dict, n_total: int, world: int, device=None) -> dict | None:
    """all_gather each rank's result arrays (torch tensors of identical dtype) into full-batch arrays on every rank.
    Works with the gloo (CPU tensors) and nccl/RCCL (GPU tensors) backends.  Shards are padded to equal length."""
    import torch

    sizes = [shard_range(n_total, world, r) for r in range(world)]
    maxlen = max(hi - lo for lo, hi in sizes)
    out = {}
    for k, t in local.items():
        pad = torch.zeros((maxlen,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        pad[: t.shape[0]] = t
        parts = [torch.empty_like(pad) for _ in range(world)]
        dist.all_gather(parts, pad)
        out[k] = torch.cat([p[: hi - lo] for p, (lo, hi) in zip(parts, sizes)])
    return out


def allreduce_counters(dist, counters: np.ndarray, device=None) -> np.ndarray:
    import torch

    t = torch.from_numpy(np.asarray(counters, dtype=np.int64).copy())
    if device is not None:
        t = t.to(device)
    dist.all_reduce(t)
    return t.cpu().numpy()
