#!/usr/bin/env python3
"""Benchmark: device-resident decode + 5-tuple ACL classify on MI355X (BASELINE.json metric).

A step = one classify launch over one resident batch (default config C1: 1M × 64 B IPv4/UDP packets, 256
five-tuple ACL rules).  Steps rotate over --nbufs distinct batches (inputs + outputs ≈ 84 MB each) so the working
set exceeds the 256 MiB Infinity Cache and every step streams its packets from HBM.  The K timed steps go through
ppe_classify_batches, which pipelines consecutive batches over two streams (a batch's launch ramp-up overlaps the
previous one's tail), as a dataplane feeding batch after batch would.  With --gpus N (launched by
torch.distributed.run) each rank classifies its own 1M-packet shard (weak scaling, no data-path collective);
`value` = all packets processed ÷ the slowest rank's time.

Prints ONE JSON line (rank 0).  Also: `roofline` from HIP-event kernel durations on the launch stream, and
`cpu_baseline` = the oracle's C restatement (tree-walk ACL, run-to-completion pthread shards like mainloop) timed on
this host's cores (rank 0, N=1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path[:0] = [str(ROOT / "packet-process-engine_amd"), str(ROOT / "oracle")]

import numpy as np  # noqa: E402
import torch  # noqa: E402  (load torch's HIP runtime before libppe_hip.so so both share it)

from ppe import Engine, synth  # noqa: E402

METRIC = "Mpps device-resident decode+ACL classify, 64B & 1500B pkts, 1/2/4/8 GPUs"
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
NOW = 1_700_000_000


def algorithmic_bytes(stride: int) -> tuple[float, float]:
    """(read, write) bytes per packet the kernel must move: the 64-B header window + 4-B length
    read; verdict + flow hash + ACL hit (12 B) + the packet's entry in its tile's FW/PUNT/DROP partition list (4 B)
    written.  Payload bytes past the window are never touched (IMIX included)."""
    return float(min(stride, 64)) + 4.0, 12.0 + 4.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=48)
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--config", default="C1", choices=sorted(synth.CONFIGS))
    ap.add_argument("--n", type=int, default=0, help="packets per GPU (default: the config's)")
    ap.add_argument("--stride", type=int, default=64)
    ap.add_argument("--nbufs", type=int, default=0, help="distinct resident batches (default: >= 8 and > 600 MB total)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-host-inclusive", action="store_true")
    ap.add_argument("--streams", type=int, default=2, choices=(1, 2),
                    help="2: the K batches go through one ppe_classify_batches call (launches of 2 batches "
                         "alternating over two streams); 1: launches of 2 batches serialized on one stream, no "
                         "overlap (profiling: kernel durations = step times)")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline sample length (16 threads)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    cfgd = synth.CONFIGS[args.config]
    if "flows" in cfgd:
        return run_flow(args, cfgd, dev, world, rank, dist)
    n = args.n or cfgd["n"]
    stride = args.stride
    rules = synth.make_rules(cfgd["rules"])
    per_buf = n * (stride + 4 + 16)
    # distinct resident batches: at least PPE_MAX_BATCH (a ppe_classify_batches launch groups up to 8 batches, and no
    # batch may repeat inside one launch) and > 2x the 256 MiB MALL, so every timed read is served by HBM
    nbufs = args.nbufs or max(8, int(np.ceil(600e6 / per_buf)))

    eng = Engine(local)
    acl = eng.commit(rules, default_action=1)
    cfg = eng.cfg(now_seconds=NOW)

    bufs = []
    lens0 = None
    for b in range(nbufs):
        pk = synth.make_packets(n, rules, seed=synth.SEED + 1 + 7919 * (rank * 64 + b), kind=cfgd["kind"],
                                stride=stride)
        if lens0 is None:
            lens0 = pk["len"]
        hdr = torch.from_numpy(pk["hdr"]).to(dev)
        lens = torch.from_numpy(pk["len"].view(np.int32)).to(dev)
        out = {"verdict": torch.empty(n, dtype=torch.int32, device=dev),
               "flow_hash": torch.empty(n, dtype=torch.int32, device=dev),
               "acl_hit": torch.empty(n, dtype=torch.int32, device=dev),
               # the ballot-compacted FW / DROP lists in the partition layout (one list, ppe_hip.h)
               "part_idx": torch.empty(n, dtype=torch.int32, device=dev)}
        bufs.append((hdr, lens, out, pk if b == 0 else None))
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream(dev)

    # pre-built C argument blocks: a step is one ppe_classify call (no per-step Python object building)
    import ctypes as C
    from ppe import abi
    calls = []
    for hdr, lens, out, _ in bufs:
        b = abi.Batch(hdr.data_ptr(), lens.data_ptr(), None, n, stride)
        r = abi.Result(out["verdict"].data_ptr(), out["flow_hash"].data_ptr(), out["acl_hit"].data_ptr(),
                       out["part_idx"].data_ptr(), out["part_idx"].data_ptr(), None, None)
        calls.append((C.byref(b), C.byref(r), b, r))
    cfg_ref = C.byref(cfg)
    sptr = C.c_void_p(stream.cuda_stream)
    classify = eng.lib.ppe_classify
    ctx = eng.ctx

    def step(i):
        bb, rr, _, _ = calls[i % nbufs]
        rc = classify(ctx, bb, rr, cfg_ref, sptr)
        if rc:
            raise RuntimeError(f"ppe_classify failed: {rc}")

    # the throughput path: ppe_classify_batches, K batches (rotating over the resident ones) pipelined over the
    # engine's two streams, stream-ordered on `stream` (one C call for the whole timed region)
    def batch_arrays(k):
        ins = (abi.Batch * k)(*(calls[i % nbufs][2] for i in range(k)))
        outs = (abi.Result * k)(*(calls[i % nbufs][3] for i in range(k)))
        return ins, outs

    def steps_pipelined(arrs):
        ins, outs = arrs
        rc = eng.lib.ppe_classify_batches(ctx, ins, outs, len(ins), cfg_ref, sptr)
        if rc:
            raise RuntimeError(f"ppe_classify_batches failed: {rc}")

    # the same batches as launches of GROUP batches each, serialized on `stream` (one ppe_classify_batches call per
    # group: its single launch goes on the caller's stream), so launch durations do not overlap
    GROUP = 2  # = the engine's batches per launch (kBatchesPerLaunch): one launch per call

    def steps_grouped(k):
        for g0 in range(0, k, GROUP):
            m = min(GROUP, k - g0)
            ins = (abi.Batch * m)(*(calls[(g0 + i) % nbufs][2] for i in range(m)))
            outs = (abi.Result * m)(*(calls[(g0 + i) % nbufs][3] for i in range(m)))
            rc = eng.lib.ppe_classify_batches(ctx, ins, outs, m, cfg_ref, sptr)
            if rc:
                raise RuntimeError(f"ppe_classify_batches failed: {rc}")

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    warm, timed = batch_arrays(max(args.warmup, 1)), batch_arrays(args.steps)
    if args.warmup and args.streams == 2:
        steps_pipelined(warm)
    elif args.warmup:
        steps_grouped(args.warmup)
    # timed region 1 (value): K batches, barrier + synchronize on both sides, no per-launch events
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    barrier()
    ev0.record(stream)
    if args.streams == 2:
        steps_pipelined(timed)
    else:
        steps_grouped(args.steps)
    ev1.record(stream)
    barrier()
    elapsed_ms = ev0.elapsed_time(ev1)
    # timed region 2 (roofline): the same K batches as launches of 2 batches serialized on `stream` (no overlap
    # between launches), with the dispatch's own start / end timestamps (hipExtLaunchKernelGGL events) around each
    eng.timing(True)
    eng.timing_read(reset=True)
    barrier()
    steps_grouped(args.steps)
    barrier()
    kern_ms, launches = eng.timing_read(reset=True)
    eng.timing(False)
    my_ms = max(elapsed_ms, 1e-9)
    # N > 1: the consumer-side verdict gather, timed apart from `value` (the classify path itself
    # exchanges nothing): all_gather over RCCL of one batch's verdict + flow hash + ACL hit (12 B per packet per rank)
    gather = None
    if dist is not None:
        try:
            _, _, out0, _ = bufs[0]
            src = torch.stack([out0["verdict"], out0["flow_hash"], out0["acl_hit"]])
            dst = torch.empty((world,) + tuple(src.shape), dtype=src.dtype, device=dev)
            ts = []
            for _ in range(6):
                barrier()
                t0 = time.perf_counter()
                dist.all_gather_into_tensor(dst, src)
                torch.cuda.synchronize()
                ts.append(time.perf_counter() - t0)
            g_ms = float(np.median(ts[1:])) * 1e3
            gt = torch.tensor([g_ms], dtype=torch.float64, device=dev)
            dist.all_reduce(gt, op=dist.ReduceOp.MAX)
            g_ms = float(gt.item())
            gather = {"ms_per_batch": round(g_ms, 4), "bytes_per_rank": 12 * n, "collective": "all_gather (RCCL)"}
        except Exception as e:  # a failed measurement must not lose the throughput line
            gather = {"error": str(e)[:200]}
    if dist is not None:
        t = torch.tensor([my_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        my_ms = float(t.item())

    total_pkts = n * args.steps * world
    mpps = total_pkts / (my_ms / 1e3) / 1e6
    rd, wr = algorithmic_bytes(stride)
    kern_avg_ms = kern_ms / max(launches, 1)
    achieved = (rd + wr) * n * args.steps / (kern_ms / 1e3) / 1e9

    # ---- parity spot check of the timed buffers (batch 0) against the oracle, 1/16 sample ----
    parity = None
    if rank == 0:
        import pyoracle
        hdr, lens, out, pk = bufs[0]
        o = pyoracle.Oracle(rules, default_action=1)
        m = min(n, 1 << 16)
        ref = o.classify_batch(pk["hdr"][:m], pk["len"][:m], cfg=o.cfg(now_seconds=NOW), nthreads=8)
        got_v = out["verdict"][:m].cpu().numpy().view(np.uint32)
        got_h = out["flow_hash"][:m].cpu().numpy().view(np.uint32)
        got_a = out["acl_hit"][:m].cpu().numpy()
        # packets whose headers reach past the window must be WINDOW_PUNT; every other one bit-exact
        far = ref["reach"] > stride
        ok = ~far
        # the partition list of those tiles: FW, PUNT, DROP per tile, each ascending, entry = index | action << 30
        act = (got_v >> 8) & 0xFF
        order = np.argsort((np.arange(m) // 64) * 4 + np.array([0, 2, 1], np.int64)[act], kind="stable")
        want_part = (order.astype(np.uint32) | (act[order] << 30)).astype(np.uint32)
        got_p = out["part_idx"][:m].cpu().numpy().view(np.uint32)
        parity = bool(np.array_equal(got_v[ok], ref["verdict"][ok]) and np.array_equal(got_h[ok], ref["flow_hash"][ok])
                      and np.array_equal(got_a[ok], ref["acl_hit"][ok]) and ((got_v[far] & 0xFF) == 18).all()
                      and np.array_equal(got_p, want_part))

    # ---- live rule commit: host build + upload + publish of the same rule set, between
    # batches (the double-buffer swap of dp_acl_rule_commit, dataplane/src/common/dp_cmd.c:1987-2053) ----
    commit_ms = []
    for _ in range(3):
        tc0 = time.perf_counter()
        acl = eng.commit(rules, default_action=1)
        commit_ms.append((time.perf_counter() - tc0) * 1e3)

    # ---- host-inclusive rate (pinned host buffers, H2D + classify + D2H pipeline) ----
    host_mpps = None
    if rank == 0 and world == 1 and not args.no_host_inclusive:
        pk = bufs[0][3]
        ph = torch.from_numpy(pk["hdr"]).pin_memory()
        pl = torch.from_numpy(pk["len"].view(np.int32)).pin_memory()
        res = {k: torch.empty(n, dtype=torch.int32).pin_memory() for k in ("verdict", "flow_hash", "acl_hit")}
        from ppe import abi
        import ctypes as C
        b = abi.Batch(ph.data_ptr(), pl.data_ptr(), None, n, stride)
        r = abi.Result(res["verdict"].data_ptr(), res["flow_hash"].data_ptr(), res["acl_hit"].data_ptr(),
                       None, None, None, None)
        reps = 5
        eng.lib.ppe_classify_host(eng.ctx, C.byref(b), C.byref(r), C.byref(cfg), 1 << 18)
        th = time.perf_counter()
        for _ in range(reps):
            rc = eng.lib.ppe_classify_host(eng.ctx, C.byref(b), C.byref(r), C.byref(cfg), 1 << 18)
            assert rc == 0
        host_mpps = n * reps / (time.perf_counter() - th) / 1e6

    # ---- CPU baseline: oracle restatement (tree-walk ACL) on this host, rank 0, N = 1 ----
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        import pyoracle
        pk = bufs[0][3]
        img = eng.image()
        o = pyoracle.Oracle(rules, default_action=1, image=img)
        thr = max(1, min(args.cpu_threads, os.cpu_count() or 1))
        o.classify_batch(pk["hdr"], pk["len"], cfg=o.cfg(now_seconds=NOW), nthreads=thr, use_tree=True)
        # bounded sample: whole passes over the batch until ~10 s of wall time (x thr cores), then a ~2 s 1-thread run
        reps = 0
        tc = time.perf_counter()
        while time.perf_counter() - tc < args.cpu_seconds:
            o.classify_batch(pk["hdr"], pk["len"], cfg=o.cfg(now_seconds=NOW), nthreads=thr, use_tree=True)
            reps += 1
        cpu_s = time.perf_counter() - tc
        ones = 0
        t1 = time.perf_counter()
        while time.perf_counter() - t1 < args.cpu_seconds / 5:
            o.classify_batch(pk["hdr"], pk["len"], cfg=o.cfg(now_seconds=NOW), nthreads=1, use_tree=True)
            ones += 1
        one_s = (time.perf_counter() - t1) / ones
        cpu = {"value": n * reps / cpu_s / 1e6, "unit": "Mpps", "cores": thr, "kind": "port",
               "sample": f"{reps} passes over the {n}-packet {args.config} batch ({n * reps} packets, {cpu_s:.1f} s), "
                         f"{thr} pthreads run-to-completion shards; 1-thread rate {n / one_s / 1e6:.2f} Mpps "
                         f"({ones} passes)",
               "single_thread_mpps": n / one_s / 1e6}

    # HBM bytes per launch from the committed rocprofv3 PMC profile of this config (tools/collect_traffic.py)
    traffic = None
    tfiles = sorted(Path(__file__).resolve().parent.glob(f"profiles/*traffic_{args.config}.json"))
    if tfiles and n == cfgd["n"] and stride == 64:
        tj = json.load(open(tfiles[-1]))
        if tj.get("n_packets") == n * GROUP:  # per launch of GROUP batches
            traffic = round(tj["traffic_bytes"])

    if rank == 0:
        li = eng.launch_info()
        line = {
            "metric": METRIC, "value": round(mpps, 2), "unit": "Mpps", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(my_ms / args.steps, 5), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic",
            "config": {"workload": f"{args.config}: {n} x {'64B IPv4/UDP' if cfgd['kind'] == 'udp64' else 'IMIX'}"
                                   f" packets per GPU, {cfgd['rules']} five-tuple ACL rules",
                       "packets_per_gpu": n, "rules": cfgd["rules"], "window_bytes": stride, "resident_batches": nbufs,
                       "streams": args.streams,
                       "parallelism": f"batch-sharded x{world}"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": traffic,
                         "kernel_avg_us": round(kern_avg_ms * 1e3, 3), "bytes_per_pkt": rd + wr,
                         "launches_timed": launches, "packets_per_launch": n * GROUP if args.steps % GROUP == 0 else None,
                         # the value's own rate in the same bytes: consecutive batches overlap on two streams
                         "pipelined_GBps": round(mpps * 1e6 / world * (rd + wr) / 1e9, 1)},
            "cpu_baseline": cpu,
            "host_inclusive_mpps": round(host_mpps, 2) if host_mpps else None,
            "parity_sample_ok": parity,
            "acl": {**{k: acl[k] for k in ("n_rules", "n_nodes", "max_depth", "blob_bytes", "lds_resident")},
                    "build_ms": round(acl["build_ms"], 3), "commit_ms": round(float(np.median(commit_ms)), 3)},
            "launch": li,
        }
        if gather is not None:
            if "ms_per_batch" in gather:
                gather["value_with_gather"] = round(n * world / ((my_ms / args.steps + gather["ms_per_batch"]) / 1e3)
                                                    / 1e6, 2)
            line["gather"] = gather
        print(json.dumps(line), flush=True)
    eng.close()
    if dist is not None:
        dist.destroy_process_group()


FLOW_METRIC = "Mpps device-resident decode+flow-table+ACL classify (stateful FlowHandlePacket)"


def flow_bytes(stride: int) -> float:
    """Algorithmic bytes per packet of the flow-mode classify kernel on the hit path: the stateless kernel's 84 B
    (window + length read; verdict, hash, hit, partition entry written) plus the flow slot's 16-B key read, its
    16-B direction counters read and written (two 8-B atomics) and the 8-B last-seen store, and the 8-B tile mask
    per 64 packets."""
    rd, wr = algorithmic_bytes(stride)
    return rd + wr + 16.0 + 32.0 + 8.0 + 8.0 / 64.0


def run_flow(args, cfgd, dev, world, rank, dist):
    """--config F1: ppe_classify_flow batch after batch (one stream: each batch sees the table the previous ones
    left) over a fixed population of bidirectional flows established during the warmup."""
    import ctypes as C
    from ppe import abi
    n = args.n or cfgd["n"]
    stride = args.stride
    rules = synth.make_rules(cfgd["rules"])
    flows = cfgd["flows"]
    nbufs = args.nbufs or 8
    eng = Engine(int(os.environ.get("LOCAL_RANK", "0")))
    acl = eng.commit(rules, default_action=abi.ACL_RULE_ACTION_FW)
    # N = 1: one flow population.  N > 1: the ranks share one population and every batch is steered by flow hash
    # to the owning GPU (ppe.dist.steered_classify_flow: all-to-all over RCCL), so flows span ranks as on a NIC that
    # does not steer by flow
    steer = world > 1
    tseed = synth.SEED + 977 * (1 if steer else rank + 1)

    # parity sample first: a fresh table, four 64k batches, against the oracle's sequential flow table
    parity = None
    if rank == 0:
        import pyoracle
        m = 1 << 16
        eng.flow_create(2 * flows, m)
        o = pyoracle.Oracle(rules, default_action=abi.ACL_RULE_ACTION_FW)
        ft = pyoracle.OracleFlow(o, capacity=2 * flows)
        ok = True
        for b in range(4):
            pk = synth.make_flow_packets(m, rules, flows // 16, seed=tseed + 31 * b, template_seed=tseed, stride=stride)
            th = torch.from_numpy(pk["hdr"]).to(dev)
            tl = torch.from_numpy(pk["len"].view(np.int32)).to(dev)
            out = {k: torch.empty(m, dtype=torch.int32, device=dev) for k in ("verdict", "flow_hash", "acl_hit")}
            eng.classify_flow_torch(th, tl, out, cfg=eng.cfg(now_seconds=NOW + b))
            ref = ft.classify_batch(pk["hdr"], pk["len"], cfg=o.cfg(0, 1, NOW + b))
            torch.cuda.synchronize()
            for k in ("verdict", "flow_hash", "acl_hit"):
                g = out[k].cpu().numpy()
                ok = ok and np.array_equal(g if k == "acl_hit" else g.view(np.uint32), ref[k])
        parity = bool(ok and len(eng.flow_dump()) == ft.stats()["live"])
        ft.close()

    eng.flow_create(2 * flows, 2 * n if steer else n)  # a steered batch may exceed n (uneven owners)
    bufs = []
    for b in range(nbufs):
        pk = synth.make_flow_packets(n, rules, flows, seed=tseed + 7919 * (b + 1), template_seed=tseed, stride=stride)
        hdr = torch.from_numpy(pk["hdr"]).to(dev)
        lens = torch.from_numpy(pk["len"].view(np.int32)).to(dev)
        out = torch.empty((3, n), dtype=torch.int32, device=dev)
        part = torch.empty(n, dtype=torch.int32, device=dev)
        bufs.append((hdr, lens, out, part, pk if b == 0 else None))
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream(dev)
    sptr = C.c_void_p(stream.cuda_stream)
    calls = []
    for hdr, lens, out, part, _ in bufs:
        bb = abi.Batch(hdr.data_ptr(), lens.data_ptr(), None, n, stride)
        rr = abi.Result(out[0].data_ptr(), out[1].data_ptr(), out[2].data_ptr(), part.data_ptr(), part.data_ptr(),
                        None, None)
        calls.append((bb, rr))
    cfgs = [eng.cfg(now_seconds=NOW + i) for i in range(args.warmup + 2 * args.steps + 1)]
    fn = eng.lib.ppe_classify_flow

    sops = None
    if steer:
        from ppe.dist import DeviceSteerOps, steered_classify_flow
        sops = DeviceSteerOps(eng)

    def step(i):
        if steer:
            hdr, lens, _, _, _ = bufs[i % nbufs]
            steered_classify_flow(sops, dist, hdr, lens, cfgs[i], world, rank)
            return
        bb, rr = calls[i % nbufs]
        rc = fn(eng.ctx, C.byref(bb), C.byref(rr), C.byref(cfgs[i]), sptr)
        if rc:
            raise RuntimeError(f"ppe_classify_flow failed: {rc}")

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    for i in range(max(args.warmup, 1)):
        step(i)
    eng.clear_counters()
    new0 = eng.flow_info()["new_flow"]
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    barrier()
    ev0.record(stream)
    for i in range(args.steps):
        step(args.warmup + i)
    ev1.record(stream)
    barrier()
    my_ms = max(ev0.elapsed_time(ev1), 1e-9)
    cnt = eng.counters()
    new_timed = eng.flow_info()["new_flow"] - new0
    # the classify (FlowFind) kernel alone: HIP-event dispatch timestamps of the same launches
    eng.timing(True)
    eng.timing_read(reset=True)
    for i in range(args.steps):
        if steer:  # the kernel timing runs this rank's own batches through its table, without the exchange
            bb, rr = calls[i % nbufs]
            fn(eng.ctx, C.byref(bb), C.byref(rr), C.byref(cfgs[args.warmup + args.steps + i]), sptr)
        else:
            step(args.warmup + args.steps + i)
    kern_ms, launches = eng.timing_read(reset=True)
    eng.timing(False)
    info = eng.flow_info()
    if dist is not None:
        t = torch.tensor([my_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        my_ms = float(t.item())
    mpps = n * args.steps * world / (my_ms / 1e3) / 1e6
    kern_avg_ms = kern_ms / max(launches, 1)
    bpp = flow_bytes(stride)
    achieved = bpp * n / (kern_avg_ms / 1e3) / 1e9

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        import pyoracle
        pk = bufs[0][4]
        o = pyoracle.Oracle(rules, default_action=abi.ACL_RULE_ACTION_FW, image=eng.image())
        ft = pyoracle.OracleFlow(o, capacity=2 * flows)
        ft.classify_batch(pk["hdr"], pk["len"], cfg=o.cfg(0, 1, NOW), use_tree=True)  # establish the flows
        reps, tc = 0, time.perf_counter()
        while time.perf_counter() - tc < args.cpu_seconds:
            ft.classify_batch(pk["hdr"], pk["len"], cfg=o.cfg(0, 1, NOW + 1 + reps), use_tree=True)
            reps += 1
        cpu_s = time.perf_counter() - tc
        ft.close()
        cpu = {"value": n * reps / cpu_s / 1e6, "unit": "Mpps", "cores": 1, "kind": "port",
               "sample": f"{reps} passes of one core's flow table (oracle FlowHandlePacket, tree-walk ACL) over the "
                         f"{n}-packet batch after the flows were established ({n * reps} packets, {cpu_s:.1f} s); the "
                         f"reference keeps one table per core, so cores scale it by flow-hash sharding"}

    if rank == 0:
        line = {
            "metric": FLOW_METRIC, "value": round(mpps, 2), "unit": "Mpps", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(my_ms / args.steps, 5), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic",
            "config": {"workload": f"{args.config}: {n} x 64B IPv4/UDP packets per GPU per batch over {flows} "
                                   f"bidirectional flows, {cfgd['rules']} five-tuple ACL rules, default FW",
                       "packets_per_gpu": n, "flows": flows, "rules": cfgd["rules"], "resident_batches": nbufs,
                       "parallelism": f"flow-sharded x{world}" + (" (all-to-all steering by flow hash)" if steer else "")},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": None,
                         "kernel": "ppe_classify_kernel<FLOW> (FlowFind + accounting; misses resolved by the flow "
                                   "kernels)",
                         "kernel_avg_us": round(kern_avg_ms * 1e3, 3), "bytes_per_pkt": bpp,
                         "batch_avg_us": round(my_ms / args.steps * 1e3, 3)},
            "cpu_baseline": cpu,
            "parity_sample_ok": parity,
            "flow_table": info,
            "new_flows_in_timed_region": new_timed,
            "counters": {k: cnt[k] for k in ("pkts", "acl_fw", "acl_drop", "flow_proc_ok", "flow_proc_fail",
                                             "flow_node_nomem")},
        }
        print(json.dumps(line), flush=True)
    eng.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
