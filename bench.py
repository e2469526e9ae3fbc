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
    if cfgd["kind"] == "frag":
        return run_defrag(args, cfgd, dev, world, rank, dist)
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


DEFRAG_METRIC = "Mfps device-resident IPv4 reassembly (Defrag: FCB find/create, chain, reassembled datagrams)"


def defrag_batch_variants(arena, off, lens, count):
    """`count` copies of one fragment batch whose datagrams are all distinct: copy v rewrites the top byte of every
    frame's IPv4 source address to v, so its FCB keys (sip, dip, ip_id) never meet another copy's.  Returns the byte
    offsets of that field and a function building copy v on the host."""
    l2 = np.where((arena[off + 12] == 0x81) & (arena[off + 13] == 0x00), 18, 14).astype(np.uint64)
    pos = (off + l2 + 12).astype(np.int64)

    def variant(v):
        a = arena.copy()
        a[pos] = v
        return a
    return pos, variant


def run_defrag(args, cfgd, dev, world, rank, dist):
    """--config D1: ppe_defrag batch after batch on one stream.  Every batch is the same
    65,536-fragment slice of a make_fragment_stream mix with a different source-address byte, so every batch
    creates fresh FCBs (none meets an earlier batch's datagrams); the warmup's FCBs are aged out before the timed
    region.  N > 1: each rank reassembles its own batches (fragments are steered to GPUs by (sip, dip, ip_id)
    upstream, as the reference's cores own their FCB tables), weak scaling with no data-path collective."""
    from ppe import Defrag
    n = args.n or cfgd["n"]
    hdr_stride = 128
    nvar = max(args.warmup, 1) + args.steps
    if nvar > 255:
        raise SystemExit("D1: warmup + steps must be <= 255 (one source-address byte per batch)")
    a_full, o_full, l_full = synth.make_fragment_stream(int(n / 3.1) + 64, seed=synth.SEED + 7 + 101 * rank)
    if len(l_full) < n:
        raise SystemExit(f"D1: fragment stream too short ({len(l_full)} < {n})")
    off, lens = o_full[:n].copy(), l_full[:n].copy()
    end = int(off[-1]) + int(lens[-1])
    arena = np.zeros(end + 64, np.uint8)
    arena[:end] = a_full[:end]
    pos, variant = defrag_batch_variants(arena, off, lens, nvar)

    eng = Engine(int(os.environ.get("LOCAL_RANK", "0")))
    stream = torch.cuda.current_stream(dev)
    t_off = torch.from_numpy(off.view(np.int64)).to(dev)
    t_len = torch.from_numpy(lens.view(np.int32)).to(dev)
    t_ids = torch.arange(n, dtype=torch.int64, device=dev)

    # parity sample: batch variant 1 through a fresh table and the oracle's sequential Defrag
    parity = None
    if rank == 0:
        import pyoracle
        g = Defrag(eng, fcb_max=1 << 16)
        o = pyoracle.OracleDefrag(fcb_max=1 << 16)
        a1 = variant(1)
        out = g.alloc_out(n, hdr_stride)
        g.run_torch(torch.from_numpy(a1).to(dev), t_off, t_len, out, NOW, ids=t_ids)
        ref = o.batch(a1, off, lens, NOW, ids=np.arange(n, dtype=np.uint64))
        torch.cuda.synchronize()
        nd = ref["n_dgram"]
        got_len = out["dgram_len"].cpu().numpy().view(np.uint32)
        ok = (np.array_equal(out["status"].cpu().numpy().view(np.uint32), ref["status"]) and
              int(out["n_dgram"].item()) == nd and np.array_equal(got_len, ref["dgram_len"]) and
              np.array_equal(out["dgram_of"].cpu().numpy().view(np.uint32), ref["dgram_of"]))
        gp = out["dgram_pkt"][:nd].cpu().numpy()
        for j in range(nd):
            m = int(ref["dgram_len"][j])
            ok = ok and np.array_equal(gp[j, :m], ref["dgram_pkt"][j, :m])
        parity = bool(ok)
        stats = {k: int(v) for k, v in o.stats().items()}
        del out, gp, ref
        g.close()
        o.close()

    d = Defrag(eng, fcb_max=cfgd["fcb_max"])
    base = torch.from_numpy(arena).to(dev)
    t_pos = torch.from_numpy(pos).to(dev)
    pkts = []
    for v in range(nvar):
        t = base.clone()
        t[t_pos] = v + 2   # variants 2.. (1 was the parity table's)
        pkts.append(t)
    out = d.alloc_out(n, hdr_stride)
    torch.cuda.synchronize()

    def step(i, now):
        d.run_torch(pkts[i], t_off, t_len, out, now, ids=t_ids, stream=stream)

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    nw = max(args.warmup, 1)
    for i in range(nw):
        step(i, NOW)
    torch.cuda.synchronize()
    d.age(NOW + 10**6, 20)   # free the warmup's FCBs (Frag_defrag_timeout), untimed
    info0 = d.info()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    barrier()
    ev0.record(stream)
    for i in range(args.steps):
        step(nw + i, NOW + 10**6)
    ev1.record(stream)
    barrier()
    my_ms = max(ev0.elapsed_time(ev1), 1e-9)
    info = d.info()
    n_dgram = int(out["n_dgram"].item())
    dlen = out["dgram_len"][:n_dgram].to(torch.int64).sum().item()
    st = out["status"].cpu().numpy().view(np.uint32) & 0xff
    held = int(np.isin(st, (0, 1, 2)).sum())
    if dist is not None:
        t = torch.tensor([my_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        my_ms = float(t.item())
    mfps = n * args.steps * world / (my_ms / 1e3) / 1e6
    call_ms = my_ms / args.steps
    # algorithmic bytes of one ppe_defrag call: every frame read once (parse reads its header
    # bytes, the stash or the assembly its data), the frames left held written to their FCB's store slots,
    # every datagram's bytes read (from the input or the store) and written out (whole frame + classify window), and the
    # per-fragment descriptors (offset 8, length 4, id 8 in; status 4, datagram index 4 out) and per-datagram
    # outputs (length 4, fragment ids 8 x cache_max)
    frame_bytes = float(lens.astype(np.int64).sum())
    # held fragments stay in the store unless their datagram completed in this same batch (those are assembled
    # straight from the input frames); every timed batch's datagrams are its own, so dgram_frags ids are batch indices
    fr_ids = out["dgram_frags"][:n_dgram].cpu().numpy().view(np.uint64).ravel()
    stored = np.isin(st, (0, 1, 2))
    stored[fr_ids[fr_ids < n].astype(np.int64)] = False
    held_bytes = float(lens[stored].astype(np.int64).sum())
    cm = d.info_["cache_max"]
    bytes_call = (frame_bytes + held_bytes + 2.0 * dlen + n_dgram * (hdr_stride + 4 + 8 * cm) + n * 28.0)
    stored_frags = int(stored.sum())
    achieved = bytes_call / (call_ms / 1e3) / 1e9

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        import pyoracle
        o = pyoracle.OracleDefrag(fcb_max=cfgd["fcb_max"])
        host = [variant(v + 2) for v in range(min(nvar, 16))]
        ids = np.arange(n, dtype=np.uint64)
        oo = dict(status=np.zeros(n, np.uint32), dgram_of=np.zeros(n, np.uint32), dgram_len=np.zeros(n, np.uint32),
                  dgram_frags=np.zeros((n, 8), np.uint64), dgram_pkt=np.zeros((n, 8168), np.uint8))
        reps, tc = 0, time.perf_counter()
        while time.perf_counter() - tc < args.cpu_seconds:
            a = host[reps % len(host)]
            o.lib.oracle_defrag_batch(o.h, a.ctypes.data, off.ctypes.data, lens.ctypes.data, ids.ctypes.data, n,
                                      NOW + reps, oo["status"].ctypes.data, oo["dgram_of"].ctypes.data,
                                      oo["dgram_pkt"].ctypes.data, oo["dgram_len"].ctypes.data,
                                      oo["dgram_frags"].ctypes.data)
            reps += 1
            if reps % len(host) == 0:
                o.age(NOW + 10**7 + reps, 20)   # the reference ages once a second; here once per variant cycle
        cpu_s = time.perf_counter() - tc
        o.close()
        cpu = {"value": n * reps / cpu_s / 1e6, "unit": "Mfps", "cores": 1, "kind": "port",
               "sample": f"{reps} passes of one core's Defrag (the oracle's sequential restatement, datagram bytes "
                         f"assembled) over the {n}-fragment batch ({n * reps} fragments, {cpu_s:.1f} s); the "
                         f"reference keeps one FCB table per core"}

    if rank == 0:
        line = {
            "metric": DEFRAG_METRIC, "value": round(mfps, 2), "unit": "Mfps", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(call_ms, 5), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic",
            "config": {"workload": f"{args.config}: {n} IPv4 fragments per GPU per batch (make_fragment_stream mix: "
                                   f"UDP/TCP/ICMP, reordered, duplicated, lost, overlapping, oversize), "
                                   f"fcb_max {cfgd['fcb_max']}, cache_max {cm}",
                       "fragments_per_gpu": n, "mean_frame_bytes": round(frame_bytes / n, 1),
                       "datagrams_per_batch": n_dgram, "parallelism": f"fcb-sharded x{world}"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": None,
                         "kernel": "one ppe_defrag call (parse..assemble, 17 stream-ordered kernels)",
                         "call_avg_us": round(call_ms * 1e3, 3), "bytes_per_call": bytes_call},
            "cpu_baseline": cpu,
            "parity_sample_ok": parity,
            "parity_sample_stats": stats if rank == 0 else None,
            "defrag_info": info,
            "held_fragments_per_batch": held, "stored_fragments_per_batch": stored_frags,
            "new_fcb_in_timed_region": int(info["new_fcb"] - info0["new_fcb"]),
            "fcb_full_in_timed_region": int(info["st_fcb_full"] - info0["st_fcb_full"]),
        }
        print(json.dumps(line), flush=True)
    d.close()
    eng.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
