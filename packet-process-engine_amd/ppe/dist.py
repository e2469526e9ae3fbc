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


# ---------------------------------------------------------------------------------------------------------------
# Stateful path across GPUs: flow-hash steering.  Every GPU keeps one flow table (the reference
# keeps one per core); a packet must be classified by the GPU that owns its flow, flow_hash % world, as Octeon's PIP
# tag steering sends a flow to one core (dataplane/src/platform/oct-init.c:139-151).  Per batch:
#   1. stateless classify (verdict + flow hash), ppe_steer_partition → perm grouped by owner, counts per owner;
#   2. all-to-all of the counts, then of the header windows and lengths gathered in perm order (RCCL over xGMI);
#   3. ppe_classify_flow on the received packets: source rank 0's packets first, each source in its original order;
#   4. reverse all-to-all of (verdict, flow hash, ACL hit), scattered back to the original positions.
# The device work is behind an `ops` object (DeviceSteerOps: libppe_hip.so kernels; tests also drive the same
# orchestration with host stand-ins over gloo).

class DeviceSteerOps:
    """The GPU implementation: libppe_hip.so kernels on torch tensors of the engine's device."""

    def __init__(self, eng):
        import torch
        self.eng, self.torch = eng, torch
        self.dev = torch.device("cuda", eng.device)

    def _s(self):
        return self.torch.cuda.current_stream(self.dev).cuda_stream

    def classify_stateless(self, hdr, lens, cfg):
        t = self.torch
        n = lens.numel()
        out = {"verdict": t.empty(n, dtype=t.int32, device=self.dev), "flow_hash": t.empty(n, dtype=t.int32, device=self.dev)}
        self.eng.classify_torch(hdr, lens, out, cfg=cfg)
        return out["verdict"], out["flow_hash"]

    def partition(self, verdict, flow_hash, world, rank):
        t = self.torch
        n = verdict.numel()
        perm = t.empty(n, dtype=t.int32, device=self.dev)
        counts = t.empty(world, dtype=t.int32, device=self.dev)
        self.eng._check(self.eng.lib.ppe_steer_partition(self.eng.ctx, verdict.data_ptr(), flow_hash.data_ptr(), n,
                                                          world, rank, perm.data_ptr(), counts.data_ptr(), self._s()),
                        "ppe_steer_partition")
        return perm, counts

    def gather(self, src, perm):
        out = self.torch.empty((perm.numel(),) + tuple(src.shape[1:]), dtype=src.dtype, device=self.dev)
        row = src[0].numel() * src.element_size() if src.numel() else 4
        self.eng._check(self.eng.lib.ppe_gather_rows(self.eng.ctx, src.data_ptr(), row, perm.data_ptr(), perm.numel(),
                                                     out.data_ptr(), self._s()), "ppe_gather_rows")
        return out

    def scatter(self, src, perm):
        out = self.torch.empty_like(src)
        row = src[0].numel() * src.element_size() if src.numel() else 4
        self.eng._check(self.eng.lib.ppe_scatter_rows(self.eng.ctx, src.data_ptr(), row, perm.data_ptr(), perm.numel(),
                                                      out.data_ptr(), self._s()), "ppe_scatter_rows")
        return out

    def classify_flow(self, hdr, lens, cfg):
        t = self.torch
        n = lens.numel()
        res = t.empty((n, 4), dtype=t.int32, device=self.dev)  # verdict, flow hash, acl hit, pad (16-B rows)
        if n:
            cols = {k: t.empty(n, dtype=t.int32, device=self.dev) for k in ("verdict", "flow_hash", "acl_hit")}
            self.eng.classify_flow_torch(hdr, lens, cols, cfg=cfg)
            res[:, 0], res[:, 1], res[:, 2] = cols["verdict"], cols["flow_hash"], cols["acl_hit"]
            res[:, 3] = 0
        return res


def steer_prepare(ops, hdr, lens, cfg, world: int, rank: int):
    """Phase 1: owners and the send buffers in owner-grouped order."""
    verdict, flow_hash = ops.classify_stateless(hdr, lens, cfg)
    perm, counts = ops.partition(verdict, flow_hash, world, rank)
    return perm, counts, ops.gather(hdr, perm), ops.gather(lens, perm)


def steer_finish(ops, back, perm) -> dict:
    """Phase 4: results (n × 4 rows, owner-grouped order) back to the original packet order."""
    out = ops.scatter(back, perm)
    return {"verdict": out[:, 0], "flow_hash": out[:, 1], "acl_hit": out[:, 2]}


def steered_classify_flow(ops, dist, hdr, lens, cfg, world: int, rank: int) -> dict:
    """One batch of this rank through the flow tables of all ranks (collective: every rank calls it)."""
    import torch
    perm, counts, send_hdr, send_len = steer_prepare(ops, hdr, lens, cfg, world, rank)
    send_counts = counts.to(torch.int64)
    recv_counts = torch.empty_like(send_counts)
    dist.all_to_all_single(recv_counts, send_counts)
    sc, rc = send_counts.cpu().tolist(), recv_counts.cpu().tolist()
    recv_hdr = torch.empty((sum(rc),) + tuple(hdr.shape[1:]), dtype=hdr.dtype, device=hdr.device)
    recv_len = torch.empty(sum(rc), dtype=lens.dtype, device=lens.device)
    dist.all_to_all_single(recv_hdr, send_hdr, output_split_sizes=rc, input_split_sizes=sc)
    dist.all_to_all_single(recv_len, send_len, output_split_sizes=rc, input_split_sizes=sc)
    res = ops.classify_flow(recv_hdr, recv_len, cfg)
    back = torch.empty((sum(sc), 4), dtype=res.dtype, device=res.device)
    dist.all_to_all_single(back, res, output_split_sizes=sc, input_split_sizes=rc)
    return steer_finish(ops, back, perm)
