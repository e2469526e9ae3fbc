#!/usr/bin/env python3
"""Benchmark: device-resident decode + 5-tuple ACL classify on MI355X (BASELINE.json metric).

A step = one pass of the hot path over one resident batch.  `value` is config C1 (1M x 64-B IPv4/UDP packets per
GPU, 256 five-tuple ACL rules, BASELINE configs[1]); the same JSON line carries C2 (IMIX 64/570/1500 B, Eth+VLAN,
TCP/UDP, 4k rules: the metric's 1500-B leg), C3 (64k rules, HBM/L2-resident classifier) and C4 (64 B, 4k rules:
BASELINE configs[4], the 1/2/4/8-GPU scaling config) under "configs", each timed and roofline-checked the same way.

The K timed batches of a config go through ONE ppe_classify_batches call, which the engine runs as one persistent
launch over the whole queue (device descriptor ring): as a dataplane draining a queue of resident batches would.
The batches rotate over >= 8 distinct resident buffers (> 600 MB, more than twice the 256 MiB Infinity Cache), so
every read is served by HBM.

Multi-GPU: one process per GPU.  `--gpus N` without WORLD_SIZE in the environment starts
`torch.distributed.run` with N ranks as a child process (before this process touches the GPU) and exits with its
code; with WORLD_SIZE set (the driver's own torchrun launch) the rank count must equal --gpus.  Every rank
classifies its own resident batches (batch-sharded, no data-path collective): weak scaling by default (1M packets
per GPU per step), `--scaling strong` splits a fixed 8M-packet step across the ranks.  `value` = all ranks'
packets / the slowest rank's time (barrier + synchronize around the timed region, MAX over ranks).  The RCCL
verdict gather a consumer would add is timed apart (`gather`).

`roofline`: the config's launch timed with its dispatch start/end timestamps (hipExtLaunchKernelGGL events on the
launch stream) inside the same timed region as `value`; achieved = SURVEY.md 8(d)'s algorithmic bytes per 64-B
packet (68 read + the verdict, flow hash and ACL hit written: 8 B in the default packed result layout, 12 B as three
4-B words with `--layout soa`; the kernel also writes a 1-B compacted-list entry (the compact partition list,
ppe_result_t.part8), counted in `written_bytes_per_pkt`) x packets in the launch / its duration; `read_frac` is the
68 read bytes alone against the peak (north_star's read-bandwidth target).  `traffic` = HBM bytes of the launch from the committed rocprofv3 FETCH_SIZE / WRITE_SIZE profile of the
same launch shape (per packet, scaled), when one exists.  `cpu_baseline` = the oracle's C restatement (tree-walk
ACL) timed on this host's cores as pinned run-to-completion pthreads (rank 0, N = 1).

`--dry-run`: the rank plumbing only (gloo, no GPU): spawn, rendezvous, MAX reduction, one JSON line.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import socket
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path[:0] = [str(ROOT / "packet-process-engine_amd"), str(ROOT / "oracle")]

import numpy as np  # noqa: E402
import torch  # noqa: E402  (load torch's HIP runtime before libppe_hip.so so both share it; no GPU call yet)

from ppe import Engine, synth  # noqa: E402

METRIC = "Mpps device-resident decode+ACL classify, 64B & 1500B pkts, 1/2/4/8 GPUs"
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
NOW = 1_700_000_000
STRONG_TOTAL = 8 << 20  # --scaling strong: packets per step over all ranks
EXTRA_CONFIGS = ("C2", "C3", "C4")


def algorithmic_bytes(stride_or_len: float) -> tuple[float, float]:
    """(read, write) bytes per packet of SURVEY.md 8(d): the header window (min(len, 64) B) + the 4-B length read,
    the 12-B verdict (status/action/flags, flow hash, ACL hit) written.  Payload bytes are never touched."""
    return float(min(stride_or_len, 64)) + 4.0, 12.0


def host_cores() -> list[int]:
    """The CPUs this process may run on, capped like `nproc` by OMP_NUM_THREADS (16 on the GPU box)."""
    cpus = sorted(os.sched_getaffinity(0))
    cap = os.environ.get("OMP_NUM_THREADS")
    if cap and cap.isdigit() and int(cap) > 0:
        cpus = cpus[:int(cap)]
    return cpus


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn(args_list: list[str], n: int) -> int:
    """Run this script under torch.distributed.run with n ranks (a child process: this one never touched the GPU)."""
    # torch.distributed.run's own parser would take `--n` as an ambiguous abbreviation of its options
    args_list = ["--packets" if a == "--n" else ("--packets=" + a[4:] if a.startswith("--n=") else a)
                 for a in args_list]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", str(Path(__file__).resolve())] + args_list
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.run(cmd, env=env).returncode


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=32)
    ap.add_argument("--warmup", type=int, default=4)
    ap.add_argument("--config", default="C1", choices=sorted(synth.CONFIGS))
    ap.add_argument("--configs", default=",".join(EXTRA_CONFIGS),
                    help="extra stateless configs measured after --config and nested in the line ('' = none)")
    ap.add_argument("--stateful", default="F1,D1",
                    help="stateful configs (flow table, reassembly) nested in the default line ('' = none)")
    ap.add_argument("--scaling", default="weak", choices=("weak", "strong"))
    ap.add_argument("--packets", "--n", dest="n", type=int, default=0,
                    help="packets per GPU per step (default: the config's; strong: 8M / ranks)")
    ap.add_argument("--stride", type=int, default=64)
    ap.add_argument("--layout", default="packed", choices=("packed", "soa"),
                    help="result layout of the stateless configs: packed = one 8-B word per packet (flow hash, status, "
                         "action, flags, ACL hit + 1: ppe_result_t.packed) + the 1-B compact partition list (9 B "
                         "written); soa = the 4-B verdict, flow hash and ACL hit words + the 1-B list (13 B)")
    ap.add_argument("--nbufs", type=int, default=0, help="distinct resident batches (default: >= 8, > 600 MB and >= "
                                                          "the batches of one launch)")
    ap.add_argument("--batches-per-launch", type=int, default=0,
                    help="0: the K batches in one persistent launch (default); B: launches of B batches "
                         "alternating over two streams")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-host-inclusive", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline sample length (all cores)")
    ap.add_argument("--nested-cpu-seconds", type=float, default=3.0,
                    help="CPU baseline sample length of each nested stateless config (all cores)")
    ap.add_argument("--no-c0", action="store_true", help="skip the C0 plumbing config (10k x 64 B, 16 rules)")
    ap.add_argument("--dry-run", action="store_true", help="rank plumbing only (gloo, no GPU)")
    ap.add_argument("--shared-gpu", action="store_true",
                    help="rehearsal of the N > 1 path on a one-GPU box: every rank on cuda:0, collectives over gloo "
                         "(the rates are not a scaling result; stateless configs only)")
    return ap.parse_args(argv)


def main():
    args = parse()
    if args.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn(sys.argv[1:], args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr, flush=True)
        sys.exit(2)
    if args.dry_run:
        return dry_run(args, world, rank)
    dist = None
    if args.shared_gpu:
        local = 0
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        if args.shared_gpu:
            dist.init_process_group("gloo", rank=rank, world_size=world)
        else:
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", local))
        if dist.get_world_size() != args.gpus:
            raise SystemExit(f"RCCL reports {dist.get_world_size()} ranks, expected {args.gpus}")
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    cfgd = synth.CONFIGS[args.config]
    if "flows" in cfgd:
        return run_flow(args, cfgd, dev, world, rank, dist)
    if cfgd["kind"] == "frag":
        return run_defrag(args, cfgd, dev, world, rank, dist)
    return run_stateless(args, dev, world, rank, dist)


def dry_run(args, world, rank):
    """Spawn + rendezvous + MAX-over-ranks plumbing on gloo (CPU only), one JSON line from rank 0."""
    import torch.distributed as dist
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    t = torch.tensor([1.0 + rank], dtype=torch.float64)
    if world > 1:
        dist.barrier()
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    ranks = dist.get_world_size() if world > 1 else 1
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": None, "unit": "Mpps", "n_gpus": world, "ranks_reported": ranks,
                          "max_over_ranks": float(t.item()), "scaling": args.scaling, "dry_run": True}), flush=True)
    if world > 1:
        dist.destroy_process_group()


class Resident:
    """`nbufs` distinct device batches of one config (2 generated batches, cloned / tiled on the device: every
    buffer is its own HBM allocation) with their output buffers and pre-built C argument blocks."""

    def __init__(self, name, n, stride, nbufs, rules, rank, dev, layout="packed"):
        from ppe import abi
        cfgd = synth.CONFIGS[name]
        self.n, self.stride, self.nbufs, self.layout = n, stride, nbufs, layout
        gen_n = min(n, 1 << 20)
        self.host = []
        for g in range(2):
            self.host.append(synth.make_packets(gen_n, rules, seed=synth.SEED + 1 + 7919 * (rank * 64 + g),
                                                kind=cfgd["kind"], stride=stride))
        self.bufs = []
        reps = (n + gen_n - 1) // gen_n
        for b in range(nbufs):
            pk = self.host[b % 2]
            hdr = torch.from_numpy(pk["hdr"]).to(dev)
            lens = torch.from_numpy(pk["len"].view(np.int32)).to(dev)
            if reps > 1:
                hdr = hdr.repeat(reps, 1)[:n].contiguous()
                lens = lens.repeat(reps)[:n].contiguous()
            if layout == "packed":  # one 8-B word per packet: include/ppe_hip.h PPE_PACKED_*
                out = {"packed": torch.empty(n, dtype=torch.int64, device=dev)}
            else:
                out = {k: torch.empty(n, dtype=torch.int32, device=dev) for k in ("verdict", "flow_hash", "acl_hit")}
            out["part8"] = torch.empty(n, dtype=torch.uint8, device=dev)
            bb = abi.Batch(hdr.data_ptr(), lens.data_ptr(), None, n, stride)
            # the compacted FW / PUNT / DROP lists in the compact partition layout (one byte per packet: its offset
            # in the tile and its action, include/ppe_hip.h ppe_result_t.part8)
            ptr = lambda k: out[k].data_ptr() if k in out else None  # noqa: E731
            rr = abi.Result(ptr("verdict"), ptr("flow_hash"), ptr("acl_hit"), None, None, None, None,
                            out["part8"].data_ptr(), ptr("packed"))
            self.bufs.append((hdr, lens, out, bb, rr))
        lens0 = self.host[0]["len"].astype(np.int64)
        self.read_bytes_per_pkt = float(np.minimum(lens0 & 0xFFFF, 64).mean() + 4.0) if stride == 64 else None
        # algorithmic result bytes (the verdict, flow hash and ACL hit: 12 B as three words, 8 B
        # packed) and the bytes the launch really writes per packet (+ the 1-B compact list entry)
        self.result_bytes = 8.0 if layout == "packed" else 12.0
        self.written_bytes = self.result_bytes + 1.0

    def results(self, b):
        """Buffer b's outputs as host arrays: verdict, flow_hash, acl_hit (unpacked from the packed words)."""
        from ppe import abi
        out = self.bufs[b][2]
        if self.layout == "packed":
            return abi.unpack(out["packed"].cpu().numpy())
        return {"verdict": out["verdict"].cpu().numpy().view(np.uint32),
                "flow_hash": out["flow_hash"].cpu().numpy().view(np.uint32), "acl_hit": out["acl_hit"].cpu().numpy()}

    def arrays(self, k):
        from ppe import abi
        ins = (abi.Batch * k)(*(self.bufs[i % self.nbufs][3] for i in range(k)))
        outs = (abi.Result * k)(*(self.bufs[i % self.nbufs][4] for i in range(k)))
        return ins, outs


def parity_sample(eng, res, rules, name):
    """Batch 0's outputs against the oracle on a sample: bit-exact verdict / flow hash / ACL hit (packets whose
    headers reach past the window must be WINDOW_PUNT) and the compact partition list of those tiles."""
    import pyoracle
    pk = res.host[0]
    m = min(res.n, 4096 if synth.CONFIGS[name]["rules"] > 10000 else 1 << 16)
    o = pyoracle.Oracle(rules, default_action=1)
    ref = o.classify_batch(pk["hdr"][:m], pk["len"][:m], cfg=o.cfg(now_seconds=NOW), nthreads=8)
    out = res.bufs[0][2]
    got = res.results(0)
    got_v, got_h, got_a = got["verdict"][:m], got["flow_hash"][:m], got["acl_hit"][:m]
    far = ref["reach"] > res.stride
    ok = ~far
    act = (got_v >> 8) & 0xFF
    order = np.argsort((np.arange(m) // 64) * 4 + np.array([0, 2, 1], np.int64)[act], kind="stable")
    want_part = ((order & 63) | (act[order] << 6)).astype(np.uint8)  # PPE_PART8_OFFSET / _ACTION
    got_p = out["part8"][:m].cpu().numpy()
    return bool(np.array_equal(got_v[ok], ref["verdict"][ok]) and np.array_equal(got_h[ok], ref["flow_hash"][ok])
                and np.array_equal(got_a[ok], ref["acl_hit"][ok]) and ((got_v[far] & 0xFF) == 18).all()
                and np.array_equal(got_p, want_part)), m


class _CalibBatch(ctypes.Structure):  # csrc/ppe_calib.hip ppe_calib_batch
    _fields_ = [("hdr", ctypes.c_void_p), ("len", ctypes.c_void_p), ("o0", ctypes.c_void_p), ("o1", ctypes.c_void_p),
                ("o2", ctypes.c_void_p), ("o3", ctypes.c_void_p), ("n", ctypes.c_uint32), ("pad", ctypes.c_uint32)]


class _CalibArgs(ctypes.Structure):  # ppe_calib_args
    _fields_ = [("b", _CalibBatch * 32), ("nb", ctypes.c_uint32), ("mode", ctypes.c_uint32), ("clk", ctypes.c_void_p)]


def sample_clocks(busy):
    """sclk / mclk (MHz) from rocm-smi, sampled while `busy()` keeps the GPU loaded (relaunched until rocm-smi has
    answered, at most a few seconds).  None where the tool is absent or says nothing parseable."""
    import re
    try:
        p = subprocess.Popen(["rocm-smi", "--showclocks", "--json"], stdout=subprocess.PIPE, stderr=subprocess.DEVNULL,
                             text=True)
    except OSError:
        return {}
    t0 = time.perf_counter()
    while p.poll() is None and time.perf_counter() - t0 < 8.0:
        busy()
    try:
        out, _ = p.communicate(timeout=5)
        card = next(iter(json.loads(out).values()))
    except Exception:
        return {}
    got = {}
    for k, v in card.items():
        m = re.search(r"(\d+)\s*Mhz", str(v), re.I)
        if m and k.lower().startswith(("sclk", "mclk", "fclk")):
            got[k.split()[0].lower() + "_mhz"] = int(m.group(1))
    return got


def ceiling(res, args, dev, kern_avg_ms, pk_launch, alg):
    """Same-run memory ceilings beside the classify launch: the kernel's own traffic with no decode / ACL
    work (skeleton: 52 + 4 B read and four 4-B results written per packet, one persistent launch over the same
    resident batches; real_GBps counts the 64-B lines the 52 B fetch, 68 + 16 B), the reads alone (read-only, 68 B),
    and a 16-B-per-lane copy of 1 GiB; each with the shader clock it
    ran at (in-kernel s_memtime over s_memrealtime), plus rocm-smi's sclk / mclk sampled under load."""
    import ctypes as C
    lib = C.CDLL(str(ROOT / "packet-process-engine_amd" / "libppe_calib.so"))
    lib.ppe_calib_stream_timed.argtypes = [C.POINTER(_CalibArgs), C.c_uint32, C.c_void_p, C.POINTER(C.c_double)]
    lib.ppe_calib_copy_timed.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_uint32, C.c_void_p, C.c_void_p,
                                         C.POINTER(C.c_double)]
    stream = torch.cuda.current_stream(dev)
    sptr = C.c_void_p(stream.cuda_stream)
    clk = torch.zeros(4, dtype=torch.int64, device=dev)
    nb = min(args.steps, 32, res.nbufs)
    a = _CalibArgs()
    packed = res.layout == "packed"
    for i in range(nb):
        hdr, lens, out = res.bufs[i][:3]
        if packed:  # (mode 4: the 8-B result goes to the packed buffer)
            a.b[i] = _CalibBatch(hdr.data_ptr(), lens.data_ptr(), out["packed"].data_ptr(), None, None,
                                 out["part8"].data_ptr(), res.n, 0)
        else:
            a.b[i] = _CalibBatch(hdr.data_ptr(), lens.data_ptr(), out["verdict"].data_ptr(),
                                 out["flow_hash"].data_ptr(), out["acl_hit"].data_ptr(), out["part8"].data_ptr(),
                                 res.n, 0)
    a.nb, a.clk = nb, clk.data_ptr()
    pk = res.n * nb

    def sclk():
        c = clk.cpu().tolist()
        return round((c[1] - c[0]) / max(c[3] - c[2], 1) * 100.0, 0)

    def stream_run(mode):  # (mode 2: the skeleton with the kernel's 1-B compact list entry; 4: packed 8 + 1 B)
        a.mode = mode
        ms, t = C.c_double(), []
        for _ in range(3):  # one warm launch, then the faster of two
            if lib.ppe_calib_stream_timed(C.byref(a), 0, sptr, C.byref(ms)) != 0:
                raise RuntimeError("ppe_calib_stream failed")
            t.append(ms.value)
        return min(t[1:]), sclk()

    skel_ms, skel_clk = stream_run(4 if packed else 2)
    ro_ms, ro_clk = stream_run(1)
    nbytes = 1 << 30
    src = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    dst = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    ms = C.c_double()
    cms = []
    for _ in range(3):
        if lib.ppe_calib_copy_timed(src.data_ptr(), dst.data_ptr(), nbytes, 0, clk.data_ptr(), sptr, C.byref(ms)):
            raise RuntimeError("ppe_calib_copy failed")
        cms.append(ms.value)
    copy_ms, copy_clk = min(cms[1:]), sclk()
    del src, dst
    clocks = sample_clocks(lambda: lib.ppe_calib_stream_timed(C.byref(a), 0, sptr, C.byref(ms)))
    torch.cuda.synchronize()
    us_1m = lambda t: round(t * 1e3 / (pk / (1 << 20)), 3)  # noqa: E731
    wb = res.written_bytes
    return {
        "skeleton": {"us_per_1M_packets": us_1m(skel_ms), "frac": round(alg * pk / (skel_ms / 1e3) / 1e9 / HBM_PEAK_GBPS, 4),
                     "real_GBps": round((68.0 + wb) * pk / (skel_ms / 1e3) / 1e9, 1), "sclk_mhz": skel_clk,
                     "bytes_per_pkt": f"52 + 4 read (68 B of HBM lines), {wb:g} written (the kernel's own traffic: "
                                      + ("one 8-B packed result" if packed else "three 4-B results")
                                      + " and the 1-B compact list entry)"},
        "read_only": {"us_per_1M_packets": us_1m(ro_ms), "real_GBps": round(68.0 * pk / (ro_ms / 1e3) / 1e9, 1),
                      "frac_at_68B": round(68.0 * pk / (ro_ms / 1e3) / 1e9 / HBM_PEAK_GBPS, 4), "sclk_mhz": ro_clk},
        "copy": {"GBps": round(2.0 * nbytes / (copy_ms / 1e3) / 1e9, 1), "bytes": nbytes, "sclk_mhz": copy_clk},
        "kernel_over_skeleton": round(skel_ms / (kern_avg_ms * nb * res.n / pk_launch), 4),
        "launch_packets": pk, "rocm_smi_under_load": clocks,
    }


def traffic_per_packet(name):
    """HBM bytes per packet of this config's launch from the committed rocprofv3 profile (tools/collect_traffic.py
    output: FETCH_SIZE doubled per the gfx950 note + WRITE_SIZE, calibrated), or None."""
    files = sorted((ROOT / "profiles").glob(f"r[0-9]*_traffic_{name}.json"))
    if not files:
        return None
    tj = json.load(open(files[-1]))
    if tj.get("n_packets"):
        return tj["traffic_bytes"] / tj["n_packets"]
    return None


WARM_SECONDS = 0.25


def warm_up(fn, seconds=WARM_SECONDS):
    """The W untimed warmup steps, repeated until the GPU has been busy for `seconds`: after the seconds of host-side
    input generation before every config the GPU idles at low clocks, and one short warmup launch (~0.1 ms) does
    not ramp them up before the timed region starts (a 24.5-us hole in C1's timed call only)."""
    t0 = time.perf_counter()
    while True:
        fn()
        torch.cuda.synchronize()
        if time.perf_counter() - t0 >= seconds:
            return


def gpu_busy(dev, seconds=WARM_SECONDS):
    """Filler work right before a stateful config's timed region whose warmup steps are not repeated (D1: every call
    creates FCBs): the same clock ramp as warm_up(), from a 6-MB working set, so the config's own state stays in the
    Infinity Cache (round 5 streamed 256 MB here, which evicted F1's 64-MB key array: its first timed batches ran
    at 142 / 91 / 68 / 50 µs against 39 in steady state, profiles/r6h_F1_timed_region.txt)."""
    a = torch.randn((1024, 1024), dtype=torch.bfloat16, device=dev)
    b = torch.randn((1024, 1024), dtype=torch.bfloat16, device=dev)
    warm_up(lambda: [torch.mm(a, b) for _ in range(8)], seconds)
    del a, b


def cpu_baseline(pk, rules, image, seconds, what):
    """The oracle's C restatement (the tree walk over the same classifier image: kind "port") on this host's cores:
    all of them (nproc, OMP_NUM_THREADS-capped) as pinned run-to-completion shards (mainloop, main.c:422-425) for
    `seconds` of passes over the batch, then one pinned thread for a quarter of that."""
    import pyoracle
    m = len(pk["len"])
    o = pyoracle.Oracle(rules, default_action=1, image=image)
    cores = host_cores()
    ocfg = o.cfg(now_seconds=NOW)
    o.pin(cores)
    o.classify_batch(pk["hdr"], pk["len"], cfg=ocfg, nthreads=len(cores), use_tree=True)
    reps, tc = 0, time.perf_counter()
    while time.perf_counter() - tc < seconds:
        o.classify_batch(pk["hdr"], pk["len"], cfg=ocfg, nthreads=len(cores), use_tree=True)
        reps += 1
    cpu_s = time.perf_counter() - tc
    o.pin(cores[:1])
    ones, t1 = 0, time.perf_counter()
    while time.perf_counter() - t1 < seconds / 4:
        o.classify_batch(pk["hdr"], pk["len"], cfg=ocfg, nthreads=1, use_tree=True)
        ones += 1
    one_s = (time.perf_counter() - t1) / ones
    o.pin([])
    return {"value": m * reps / cpu_s / 1e6, "unit": "Mpps", "cores": len(cores), "kind": "port",
            "sample": f"{reps} passes over a {m}-packet {what} batch ({m * reps} packets, {cpu_s:.1f} s), "
                      f"{len(cores)} pinned pthreads (nproc of this host) as run-to-completion shards "
                      f"(mainloop, main.c:422-425); 1 pinned thread: {m / one_s / 1e6:.2f} Mpps ({ones} passes)",
            "single_thread_mpps": m / one_s / 1e6}


def sharded_cpu(nshards, setup, run_pass, seconds):
    """Run-to-completion shards on this host's cores (mainloop, main.c:422-425): shard i in its own thread pinned to
    core i, `run_pass(state, rep)` over and over for `seconds` after one untimed `setup(i)` pass.  ctypes releases
    the GIL around the oracle's C calls, so the shards run in parallel.  Returns (units per second, passes); a pass
    returns the units it processed."""
    import threading
    cores = host_cores()[:nshards]
    done = [0] * len(cores)
    span = [0.0] * len(cores)
    states = [None] * len(cores)
    gate = threading.Barrier(len(cores) + 1)

    def worker(i):
        os.sched_setaffinity(0, {cores[i]})
        states[i] = setup(i)
        gate.wait()
        t0 = time.perf_counter()
        reps = 0
        while time.perf_counter() - t0 < seconds:
            done[i] += run_pass(states[i], reps)
            reps += 1
        span[i] = time.perf_counter() - t0

    th = [threading.Thread(target=worker, args=(i,)) for i in range(len(cores))]
    for t in th:
        t.start()
    gate.wait()
    for t in th:
        t.join()
    return sum(done) / max(span), len(cores)


def flow_cpu_baseline(pk, rules, image, flows, seconds):
    """F1's CPU baseline: the oracle's FlowHandlePacket (tree-walk ACL on misses) over the bench batch after its flows
    are established, on one core, and on every core with the batch sharded by flow hash, one flow table per core
    (the reference keeps flow_table[LOCAL_CPU_ID], dataplane/src/flow/flow.c:33,481-490, and the NIC steers a flow
    to one core, platform/oct-init.c:139-151)."""
    import pyoracle
    from ppe import abi
    n = len(pk["len"])
    o = pyoracle.Oracle(rules, default_action=abi.ACL_RULE_ACTION_FW, image=image)
    fh = o.classify_batch(pk["hdr"], pk["len"], cfg=o.cfg(0, 1, NOW), nthreads=8)["flow_hash"]
    ncores = len(host_cores())

    def make(shards):
        def setup(i):
            idx = np.nonzero(fh % shards == i)[0]
            h, ln = np.ascontiguousarray(pk["hdr"][idx]), np.ascontiguousarray(pk["len"][idx])
            ft = pyoracle.OracleFlow(o, capacity=2 * flows // shards + 4096)
            ft.classify_batch(h, ln, cfg=o.cfg(0, 1, NOW), use_tree=True)  # establish this core's flows
            return ft, h, ln

        def run_pass(st, rep):
            ft, h, ln = st
            ft.classify_batch(h, ln, cfg=o.cfg(0, 1, NOW + 1 + rep), use_tree=True)
            return len(ln)
        return setup, run_pass

    one, _ = sharded_cpu(1, *make(1), seconds / 4)
    allc, used = sharded_cpu(ncores, *make(ncores), seconds)
    return {"value": allc / 1e6, "unit": "Mpps", "cores": used, "kind": "port",
            "sample": f"passes of the {n}-packet batch after its flows were established, sharded by flow hash over "
                      f"{used} pinned threads with one flow table each (oracle FlowHandlePacket, tree-walk ACL on "
                      f"misses; {seconds:.1f} s); 1 pinned thread, the whole batch in one table: "
                      f"{one / 1e6:.2f} Mpps",
            "single_thread_mpps": one / 1e6}


def defrag_cpu_baseline(variant, off, lens, fcb_max, seconds):
    """D1's CPU baseline: the oracle's sequential Defrag (datagram bytes assembled) over fresh copies of the bench
    batch, on one core, and on every core with the fragments sharded by FCB key (sip, dip, ip_id: every fragment
    of a datagram on one core), one FCB table per core (dataplane/src/decode/decode-defrag.c keeps its tables per
    core).  The source-address byte that makes each copy's datagrams fresh is left out of the shard key."""
    import pyoracle
    n = len(lens)
    base = variant(2)
    l2 = np.where((base[off + 12] == 0x81) & (base[off + 13] == 0x00), 18, 14).astype(np.int64)
    ip = off.astype(np.int64) + l2
    b = lambda k: base[ip + k].astype(np.uint32)
    key = ((b(13) << 16) | (b(14) << 8) | b(15)) * 0x9E3779B1 ^ ((b(16) << 24) | (b(17) << 16) | (b(18) << 8) | b(19)) \
        ^ ((b(4) << 8) | b(5)) * 0x85EBCA6B
    key = key.astype(np.uint32)
    host = [variant(v + 2) for v in range(16)]
    ncores = len(host_cores())

    def make(shards):
        def setup(i):
            idx = np.nonzero(key % shards == i)[0]
            m = len(idx)
            o = pyoracle.OracleDefrag(fcb_max=max(1024, fcb_max // shards))
            so, sl = np.ascontiguousarray(off[idx]), np.ascontiguousarray(lens[idx])
            ids = idx.astype(np.uint64)
            oo = dict(status=np.zeros(m, np.uint32), dgram_of=np.zeros(m, np.uint32), dgram_len=np.zeros(m, np.uint32),
                      dgram_frags=np.zeros((m, 8), np.uint64), dgram_pkt=np.zeros((m, 8168), np.uint8))
            return o, so, sl, ids, oo

        def run_pass(st, rep):
            o, so, sl, ids, oo = st
            a = host[rep % len(host)]
            o.lib.oracle_defrag_batch(o.h, a.ctypes.data, so.ctypes.data, sl.ctypes.data, ids.ctypes.data, len(sl),
                                      NOW + rep, oo["status"].ctypes.data, oo["dgram_of"].ctypes.data,
                                      oo["dgram_pkt"].ctypes.data, oo["dgram_len"].ctypes.data,
                                      oo["dgram_frags"].ctypes.data)
            if (rep + 1) % len(host) == 0:
                o.age(NOW + 10**7 + rep, 20)   # the reference ages once a second; here once per variant cycle
            return len(sl)
        return setup, run_pass

    one, _ = sharded_cpu(1, *make(1), seconds / 4)
    allc, used = sharded_cpu(ncores, *make(ncores), seconds)
    return {"value": allc / 1e6, "unit": "Mfps", "cores": used, "kind": "port",
            "sample": f"passes of the {n}-fragment batch (fresh datagrams each pass), sharded by FCB key over {used} "
                      f"pinned threads with one FCB table each (the oracle's sequential Defrag, datagram bytes "
                      f"assembled; {seconds:.1f} s); 1 pinned thread, the whole batch in one table: "
                      f"{one / 1e6:.3f} Mfps",
            "single_thread_mfps": one / 1e6}


def measure_c0(args, dev):
    """C0 (BASELINE configs[0]): the reference's own plumbing case, 10k x 64-B IPv4/UDP packets and 16 rules on ONE
    CPU thread: the oracle restatement on one pinned core (the reported baseline), and beside it the same batch as
    one ppe_classify launch on the GPU (a 10k-packet launch is latency-bound: 157 tiles on 256 CUs), with the
    whole batch checked against the oracle."""
    import pyoracle
    cfgd = synth.CONFIGS["C0"]
    n = cfgd["n"]
    rules = synth.make_rules(cfgd["rules"])
    pk = synth.make_packets(n, rules, seed=synth.SEED + 3, kind=cfgd["kind"], stride=args.stride)
    eng = Engine(dev.index)
    try:
        eng.commit(rules, default_action=1)
        cfg = eng.cfg(now_seconds=NOW)
        hdr = torch.from_numpy(pk["hdr"]).to(dev)
        lens = torch.from_numpy(pk["len"].view(np.int32)).to(dev)
        out = {k: torch.empty(n, dtype=torch.int32, device=dev) for k in ("verdict", "flow_hash", "acl_hit")}
        stream = torch.cuda.current_stream(dev)
        warm_up(lambda: eng.classify_torch(hdr, lens, out, cfg=cfg))
        reps = 200
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        ev0.record(stream)
        for _ in range(reps):
            eng.classify_torch(hdr, lens, out, cfg=cfg)
        ev1.record(stream)
        torch.cuda.synchronize()
        gpu_ms = ev0.elapsed_time(ev1) / reps
        o = pyoracle.Oracle(rules, default_action=1)
        ref = o.classify_batch(pk["hdr"], pk["len"], cfg=o.cfg(now_seconds=NOW))
        got = {k: v.cpu().numpy().view(np.uint32 if k != "acl_hit" else np.int32) for k, v in out.items()}
        parity = all(np.array_equal(got[k], ref[k]) for k in got)
        cpu = None
        if not args.no_cpu_baseline:
            o.set_image(eng.image())
            cores = host_cores()
            o.pin(cores[:1])
            ocfg = o.cfg(now_seconds=NOW)
            o.classify_batch(pk["hdr"], pk["len"], cfg=ocfg, nthreads=1, use_tree=True)
            passes, t0 = 0, time.perf_counter()
            while time.perf_counter() - t0 < 2.0:
                o.classify_batch(pk["hdr"], pk["len"], cfg=ocfg, nthreads=1, use_tree=True)
                passes += 1
            cpu_s = time.perf_counter() - t0
            o.pin([])
            cpu = {"value": n * passes / cpu_s / 1e6, "unit": "Mpps", "cores": 1, "kind": "port",
                   "sample": f"{passes} passes over the {n}-packet C0 batch on one pinned thread ({cpu_s:.1f} s)"}
        return {"workload": f"C0: {n} x 64B IPv4/UDP packets, {cfgd['rules']} five-tuple ACL rules (the reference's "
                            f"CPU plumbing config)", "value": round(n / (gpu_ms / 1e3) / 1e6, 2), "unit": "Mpps",
                "ms_per_batch": round(gpu_ms, 5), "timing": f"GPU: {reps} back-to-back single-batch launches",
                "parity_ok": parity, "parity_packets": n, "cpu_baseline": cpu}
    finally:
        eng.close()


def acl_lookup_latency(eng, pk, rules, calls=300):
    """DP_Acl_Lookup's latency (flow.c:232: one call per flow miss on the reference's hot path): host-pointer lookups
    through the C ABI call DP_Acl_Lookup / DP_Acl_Lookup_Burst make (ppe_acl_lookup_host), 1 and 64 tuples per call,
    median and 99th percentile over `calls` back-to-back calls timed around the ctypes call (its ~1 us included);
    the 64 answers are checked against the oracle's linear first match."""
    import ctypes as C
    import pyoracle
    from ppe import abi
    o = pyoracle.Oracle(rules, default_action=1)
    ref = o.classify_batch(pk["hdr"][:64], pk["len"][:64], cfg=o.cfg(now_seconds=NOW))
    tup = np.ascontiguousarray(ref["tuple"][:64])
    tup[:, 3] &= 0xFF  # {sip, dip, sport | dport << 16, proto}
    hit = np.zeros(64, np.int32)
    act = np.zeros(64, np.uint32)
    out = {}
    for k in (1, 64):
        t = abi.Tuples(tup.ctypes.data, None, None, k)
        fn, cargs = eng.lib.ppe_acl_lookup_host, (eng.ctx, C.byref(t), hit.ctypes.data, act.ctypes.data, NOW)
        for _ in range(20):
            fn(*cargs)
        ts = []
        for _ in range(calls):
            t0 = time.perf_counter()
            rc = fn(*cargs)
            ts.append(time.perf_counter() - t0)
            if rc:
                raise RuntimeError(f"ppe_acl_lookup_host: {rc}")
        out[f"lookup_us_{k}"] = round(float(np.median(ts)) * 1e6, 2)
        out[f"lookup_us_{k}_p99"] = round(float(np.percentile(ts, 99)) * 1e6, 2)
    z = np.zeros(6, np.uint8)
    want = [o.lib.oracle_acl_linear(int(a), int(b), int(c) & 0xFFFF, int(c) >> 16, int(d), z.ctypes.data,
                                    z.ctypes.data, NOW, None) for a, b, c, d in tup]
    out["lookup_ok"] = bool(np.array_equal(hit, np.array(want, np.int32)))
    return out


def measure_config(name, args, dev, world, rank, dist, primary):
    """One stateless config: resident batches, K batches in one call, roofline launch, parity sample."""
    from ppe import abi
    import ctypes as C
    cfgd = synth.CONFIGS[name]
    if args.n:
        n = args.n
    elif args.scaling == "strong":
        n = STRONG_TOTAL // world
    else:
        n = cfgd["n"]
    stride = args.stride
    rules = synth.make_rules(cfgd["rules"])
    per_buf = n * (stride + 4 + 16)
    # distinct resident batches: more than twice the 256 MiB Infinity Cache, and at least as many as one launch takes
    # (a launch's batch groups run concurrently, so a buffer repeated inside one launch would be re-read from cache)
    nbufs = args.nbufs or max(8, int(np.ceil(600e6 / per_buf)), args.steps, max(args.warmup, 1))
    eng = Engine(dev.index)
    eng.tuning(batches_per_launch=args.batches_per_launch)
    acl = eng.commit(rules, default_action=1)
    cfg = eng.cfg(now_seconds=NOW)
    res = Resident(name, n, stride, nbufs, rules, rank, dev, layout=args.layout)
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream(dev)
    sptr = C.c_void_p(stream.cuda_stream)
    cfg_ref = C.byref(cfg)

    def run(arrs):
        ins, outs = arrs
        rc = eng.lib.ppe_classify_batches(eng.ctx, ins, outs, len(ins), cfg_ref, sptr)
        if rc:
            raise RuntimeError(f"ppe_classify_batches failed: {rc} {eng.lib.ppe_last_error(eng.ctx)}")

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    warm, timed = res.arrays(max(args.warmup, 1)), res.arrays(args.steps)
    run(warm)
    # (warmed up on the timed region's own descriptor set: a ring launch that reuses it uploads nothing)
    warm_up(lambda: run(timed))
    # timed region (value): K batches, barrier + synchronize on both sides.  The roofline's launch duration is this
    # SAME region's: HIP events on the launch stream around the call, which is one launch of all K
    # batches by default (bpl launches of B batches with --batches-per-launch B), so its time per launch can never
    # exceed ms_per_step x batches and includes the launch's submission (≈ 5 us).  Dispatch-timestamp events inside
    # the region would cost ≈ 11 us more per launch (profiles/r6_ab_runs.md r6c); they are taken in a second call
    # below, for the kernel alone (the rocprofv3 comparison and the same-run skeleton), never for `value` or `frac`.
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    barrier()
    ev0.record(stream)
    run(timed)
    ev1.record(stream)
    barrier()
    my_ms = max(ev0.elapsed_time(ev1), 1e-9)
    bpl = args.batches_per_launch or args.steps
    launches = -(-args.steps // bpl)
    kern_ms = my_ms
    # the kernel alone: the same call again with the dispatch's own start / end timestamps (hipExtLaunchKernelGGL)
    eng.timing(True)
    eng.timing_read(reset=True)
    barrier()
    run(timed)
    barrier()
    disp_ms, disp_launches = eng.timing_read(reset=True)
    eng.timing(False)
    if dist is not None:
        t = torch.tensor([my_ms, kern_ms, disp_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        my_ms, kern_ms, disp_ms = float(t[0].item()), float(t[1].item()), float(t[2].item())
    total_pkts = n * args.steps * world
    mpps = total_pkts / (my_ms / 1e3) / 1e6
    rd, wr = algorithmic_bytes(64)
    if res.read_bytes_per_pkt is not None:  # IMIX: min(len, 64) + 4 read per packet
        rd = res.read_bytes_per_pkt
    wr = res.result_bytes  # (12 B as three words, 8 B packed)
    alg = rd + wr
    pk_launch = n * args.steps / max(launches, 1)
    kern_avg_ms = kern_ms / max(launches, 1)
    disp_avg_ms = disp_ms / max(disp_launches, 1)
    achieved = alg * pk_launch / (kern_avg_ms / 1e3) / 1e9
    tpp = traffic_per_packet(name)
    parity, psample = parity_sample(eng, res, rules, name) if rank == 0 else (None, 0)
    out = {
        "value": round(mpps, 2), "unit": "Mpps", "ms_per_step": round(my_ms / args.steps, 5),
        "workload": f"{name}: {n} x {'64B IPv4/UDP' if cfgd['kind'] == 'udp64' else 'IMIX 64/570/1500B Eth+VLAN TCP/UDP'}"
                    f" packets per GPU, {cfgd['rules']} five-tuple ACL rules",
        "packets_per_gpu": n, "rules": cfgd["rules"], "resident_batches": nbufs,
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBPS, 4),
                     "traffic": round(tpp * pk_launch) if tpp else None,
                     "kernel": "ppe_classify_kernel", "kernel_avg_us": round(kern_avg_ms * 1e3, 3),
                     "launches_timed": launches, "packets_per_launch": int(pk_launch),
                     "timing": "the value region's own HIP events (launch stream) around its launch(es): the launch "
                               "duration with its submission",
                     "bytes_per_pkt": round(alg, 3), "read_bytes_per_pkt": round(rd, 3),
                     "written_bytes_per_pkt": res.written_bytes, "result_layout": args.layout,
                     "read_frac": round(rd * pk_launch / (kern_avg_ms / 1e3) / 1e9 / HBM_PEAK_GBPS, 4),
                     "us_per_1M_packets": round(kern_avg_ms * 1e3 / (pk_launch / (1 << 20)), 3),
                     "dispatch": {"kernel_avg_us": round(disp_avg_ms * 1e3, 3), "launches": disp_launches,
                                  "us_per_1M_packets": round(disp_avg_ms * 1e3 / (pk_launch / (1 << 20)), 3),
                                  "frac": round(alg * pk_launch / (disp_avg_ms / 1e3) / 1e9 / HBM_PEAK_GBPS, 4),
                                  "timing": "the same call again with the dispatch packet's start / end timestamps "
                                            "(hipExtLaunchKernelGGL events: what rocprofv3 reports): the kernel alone"}},
        "parity_sample_ok": parity, "parity_sample_packets": psample,
        "acl": {**{k: acl[k] for k in ("n_rules", "n_nodes", "max_depth", "blob_bytes", "lds_resident")},
                "build_ms": round(acl["build_ms"], 3)},
        "launch": eng.launch_info(),
    }
    if primary and rank == 0:
        try:
            out["roofline"]["ceiling"] = ceiling(res, args, dev, disp_avg_ms, pk_launch, alg)
        except Exception as e:  # the ceiling is context, never worth losing the line over
            out["roofline"]["ceiling"] = {"error": str(e)[:200]}
    if not primary and rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(res.host[0], rules, eng.image(), args.nested_cpu_seconds, name)
    ctx = dict(eng=eng, res=res, rules=rules, cfg=cfg, n=n, my_ms=my_ms)
    if not primary:
        eng.close()
        del res
        torch.cuda.empty_cache()
        return out, None
    return out, ctx


def run_stateless(args, dev, world, rank, dist):
    line_cfg, ctx = measure_config(args.config, args, dev, world, rank, dist, primary=True)
    eng, res, rules, cfg, n, my_ms = (ctx[k] for k in ("eng", "res", "rules", "cfg", "n", "my_ms"))

    # N > 1: the consumer-side verdict gather, timed apart from `value` (the classify path itself
    # exchanges nothing): all_gather over RCCL of one batch's verdict + flow hash + ACL hit (8 B per packet packed,
    # 12 B as three words)
    gather = None
    if dist is not None:
        try:
            out0 = res.bufs[0][2]
            src = (out0["packed"].view(1, -1) if res.layout == "packed"
                   else torch.stack([out0["verdict"], out0["flow_hash"], out0["acl_hit"]]))
            # the concatenated output form (rank r's 3 rows at [3r, 3r + 3)): RCCL and gloo both take it
            dst = torch.empty((world * src.shape[0],) + tuple(src.shape[1:]), dtype=src.dtype, device=dev)
            ts = []
            for _ in range(6):
                dist.barrier()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                dist.all_gather_into_tensor(dst, src)
                torch.cuda.synchronize()
                ts.append(time.perf_counter() - t0)
            gt = torch.tensor([float(np.median(ts[1:])) * 1e3], dtype=torch.float64, device=dev)
            dist.all_reduce(gt, op=dist.ReduceOp.MAX)
            g_ms = float(gt.item())
            gather = {"ms_per_batch": round(g_ms, 4), "bytes_per_rank": int(res.result_bytes) * n,
                      "collective": "all_gather (gloo, shared-GPU rehearsal)" if args.shared_gpu else "all_gather (RCCL)",
                      "value_with_gather": round(n * world / ((my_ms / args.steps + g_ms) / 1e3) / 1e6, 2)}
            # the per-reason counters summed over ranks (dp_show_pkt_stat's sum over cores, dp_cmd.c:844; SURVEY.md
            # 8(e)): ppe/dist.py allreduce_counters on the engine's 32 counters, device-resident on RCCL
            from ppe.dist import allreduce_counters
            from ppe.abi import COUNTERS
            cdict = eng.counters()
            cvec = np.array([cdict[k] for k in COUNTERS], np.int64)
            cdev = None if args.shared_gpu else dev
            cs = []
            for _ in range(6):
                dist.barrier()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                summed = allreduce_counters(dist, cvec, device=cdev)
                cs.append(time.perf_counter() - t0)
            ct = torch.tensor([float(np.median(cs[1:])) * 1e3], dtype=torch.float64, device=dev)
            dist.all_reduce(ct, op=dist.ReduceOp.MAX)
            gather["counters_allreduce"] = {
                "ms": round(float(ct.item()), 4), "words": int(len(cvec)),
                "pkts_all_ranks": int(summed[COUNTERS.index("pkts")]),
                "collective": "all_reduce (gloo)" if args.shared_gpu else "all_reduce (RCCL)"}
        except Exception as e:  # a failed side measurement must not lose the throughput line
            gather = {"error": str(e)[:200]}

    # live rule commit: host build + upload + publish of the same rule set between batches
    commit_ms = []
    for _ in range(3):
        tc0 = time.perf_counter()
        eng.commit(rules, default_action=1)
        commit_ms.append((time.perf_counter() - tc0) * 1e3)

    lookup = None
    if rank == 0:
        try:
            lookup = acl_lookup_latency(eng, res.host[0], rules)
        except Exception as e:
            lookup = {"error": str(e)[:200]}

    # host-inclusive rate (pinned host buffers: the kernel reads / writes them across PCIe), rank 0 at N = 1
    host_mpps = None
    if rank == 0 and world == 1 and not args.no_host_inclusive:
        import ctypes as C
        from ppe import abi
        pk = res.host[0]
        m = len(pk["len"])
        ph = torch.from_numpy(pk["hdr"]).pin_memory()
        pl = torch.from_numpy(pk["len"].view(np.int32)).pin_memory()
        b = abi.Batch(ph.data_ptr(), pl.data_ptr(), None, m, args.stride)
        if res.layout == "packed":
            hres = {"packed": torch.empty(m, dtype=torch.int64).pin_memory()}
            r = abi.Result(None, None, None, None, None, None, None, None, hres["packed"].data_ptr())
        else:
            hres = {k: torch.empty(m, dtype=torch.int32).pin_memory() for k in ("verdict", "flow_hash", "acl_hit")}
            r = abi.Result(hres["verdict"].data_ptr(), hres["flow_hash"].data_ptr(), hres["acl_hit"].data_ptr(),
                           None, None, None, None)
        eng.lib.ppe_classify_host(eng.ctx, C.byref(b), C.byref(r), C.byref(cfg), 1 << 18)
        reps = 5
        th = time.perf_counter()
        for _ in range(reps):
            if eng.lib.ppe_classify_host(eng.ctx, C.byref(b), C.byref(r), C.byref(cfg), 1 << 18) != 0:
                raise RuntimeError("ppe_classify_host failed")
        host_mpps = m * reps / (time.perf_counter() - th) / 1e6

    # CPU baseline: the oracle's C restatement (tree-walk ACL over the same classifier image), rank 0, N = 1: all of
    # this host's cores (nproc) as pinned run-to-completion shards, then one pinned thread
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(res.host[0], rules, eng.image(), args.cpu_seconds, args.config)

    eng.close()
    del res
    torch.cuda.empty_cache()
    extra = {}
    if rank == 0 and world == 1 and args.n == 0 and not args.no_c0:
        try:
            extra["C0"] = measure_c0(args, dev)
        except Exception as e:
            extra["C0"] = {"error": str(e)[:300]}
    names = [c for c in args.configs.split(",") if c and c != args.config] if args.n == 0 else []
    for name in names:
        try:
            extra[name], _ = measure_config(name, args, dev, world, rank, dist, primary=False)
        except Exception as e:  # one config failing must not lose the headline line
            import traceback
            print(f"bench.py rank {rank}: nested {name} failed:\n{traceback.format_exc()}", file=sys.stderr, flush=True)
            extra[name] = {"error": str(e)[:300]}
    # the stateful paths: the flow table (FlowHandlePacket) and IPv4 reassembly
    # (Defrag), each with its own roofline and parity sample
    for name in [c for c in args.stateful.split(",") if c] if args.n == 0 else []:
        fn = run_flow if "flows" in synth.CONFIGS[name] else run_defrag
        try:
            extra[name] = fn(args, synth.CONFIGS[name], dev, world, rank, dist, name=name, nested=True)
        except Exception as e:
            import traceback
            print(f"bench.py rank {rank}: nested {name} failed:\n{traceback.format_exc()}", file=sys.stderr, flush=True)
            extra[name] = {"error": str(e)[:300]}
        torch.cuda.empty_cache()

    if rank == 0:
        rf = line_cfg["roofline"]
        line = {
            "metric": METRIC, "value": line_cfg["value"], "unit": "Mpps", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": line_cfg["ms_per_step"], "higher_is_better": True,
            "scaling": args.scaling, "vs_baseline": None, "dtype": "u8", "data": "synthetic",
            "config": {"workload": line_cfg["workload"], "packets_per_gpu": line_cfg["packets_per_gpu"],
                       "global_batch": line_cfg["packets_per_gpu"] * world, "rules": line_cfg["rules"],
                       "window_bytes": args.stride, "resident_batches": line_cfg["resident_batches"],
                       "batches_per_launch": args.batches_per_launch or args.steps,
                       "result_layout": ("packed: 8-B flow hash | status | action | flags | ACL hit + 1, + 1-B "
                                         "compact partition list" if args.layout == "packed" else
                                         "soa: 4-B verdict, flow hash, ACL hit + 1-B compact partition list"),
                       "parallelism": f"batch-sharded x{world}"},
            "roofline": rf,
            "cpu_baseline": cpu,
            "host_inclusive_mpps": round(host_mpps, 2) if host_mpps else None,
            "parity_sample_ok": line_cfg["parity_sample_ok"],
            "ranks_reported": dist.get_world_size() if dist is not None else 1,
            "acl": {**line_cfg["acl"], "commit_ms": round(float(np.median(commit_ms)), 3), **(lookup or {})},
            "launch": line_cfg["launch"],
            "configs": extra,
        }
        if gather is not None:
            line["gather"] = gather
        if args.shared_gpu:
            line["shared_gpu_rehearsal"] = True
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


FLOW_METRIC = "Mpps device-resident decode+flow-table+ACL classify (stateful FlowHandlePacket)"


def flow_owner_update() -> bool:
    """The library's FlowUpdate mode (ppe_flow_create reads PPE_FLOW_OWNER the same way): owner-computed (default)
    or one atomic per found packet inside the classify kernel."""
    return os.environ.get("PPE_FLOW_OWNER", "1").strip() not in ("0", "")


def flow_bytes(stride: int, owner: bool = False) -> float:
    """Algorithmic bytes per packet of the flow-mode classify kernel on the hit path: the stateless kernel's 81 B
    (window + length read; verdict, hash, hit and the 1-B compact partition entry written: part8, round 6; 84 with
    round 5's 4-B partition list), the flow slot's 16-B key read and the 8-B
    tile mask per 64 packets, plus the FlowUpdate: in the kernel, the 16-B direction counters read and written (two
    8-B atomics) and the 8-B last-seen store; owner-computed, the 8-B bucket entry the kernel writes
    instead (the update kernel then touches each flow once per batch, outside this kernel's time)."""
    rd, wr = algorithmic_bytes(stride)
    return rd + wr + 1.0 + 16.0 + (8.0 if owner else 32.0 + 8.0) + 8.0 / 64.0


def run_flow(args, cfgd, dev, world, rank, dist, name=None, nested=False):
    """--config F1: ppe_classify_flow batch after batch (one stream: each batch sees the table the previous ones
    left) over a fixed population of bidirectional flows established during the warmup.  nested: measured after the
    stateless configs of the default line and returned as its configs.F1 entry (with a shorter CPU baseline; at N > 1
    every rank owns its flows, as the reference's cores do behind the NIC's flow steering: no exchange)."""
    import ctypes as C
    from ppe import abi
    name = name or args.config
    n = (0 if nested else args.n) or cfgd["n"]
    stride = args.stride
    rules = synth.make_rules(cfgd["rules"])
    flows = cfgd["flows"]
    nbufs = args.nbufs or 8
    eng = Engine(dev.index)  # (the rank's device: cuda:0 for every rank under --shared-gpu)
    acl = eng.commit(rules, default_action=abi.ACL_RULE_ACTION_FW)
    # N = 1: one flow population.  N > 1: the ranks share one population and every batch is steered by flow hash
    # to the owning GPU (ppe.dist.steered_classify_flow: all-to-all over RCCL), so flows span ranks as on a NIC that
    # does not steer by flow
    steer = world > 1 and not nested
    tseed = synth.SEED + 977 * (1 if steer else rank + 1)

    # parity sample first: a fresh table, four 64k batches, against the oracle's sequential flow table
    parity = None
    if rank == 0:
        try:  # (rank 0 only, no collectives: an error here must not leave the other ranks in a barrier)
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
        except Exception as e:
            import traceback
            print(f"bench.py: {name} parity sample failed:\n{traceback.format_exc()}", file=sys.stderr, flush=True)
            parity = False

    eng.flow_create(2 * flows, 2 * n if steer else n)  # a steered batch may exceed n (uneven owners)
    bufs = []
    for b in range(nbufs):
        pk = synth.make_flow_packets(n, rules, flows, seed=tseed + 7919 * (b + 1), template_seed=tseed, stride=stride)
        hdr = torch.from_numpy(pk["hdr"]).to(dev)
        lens = torch.from_numpy(pk["len"].view(np.int32)).to(dev)
        out = torch.empty((3, n), dtype=torch.int32, device=dev)
        part = torch.empty(n, dtype=torch.uint8, device=dev)  # the compact partition list (part8), as C1 - C4
        bufs.append((hdr, lens, out, part, pk if b == 0 else None))
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream(dev)
    sptr = C.c_void_p(stream.cuda_stream)
    calls = []
    for hdr, lens, out, part, _ in bufs:
        bb = abi.Batch(hdr.data_ptr(), lens.data_ptr(), None, n, stride)
        rr = abi.Result(out[0].data_ptr(), out[1].data_ptr(), out[2].data_ptr(), None, None, None, None,
                        part.data_ptr())
        calls.append((bb, rr))
    # (the timed batches' times follow every warm-up step's, NOW + warmup + extra < NOW + 1e6)
    cfgs = [eng.cfg(now_seconds=NOW + i if i < args.warmup else NOW + 10**6 + i) for i in range(args.warmup + 2 * args.steps + 1)]
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
    # then more steps over the same flows until the GPU has been busy for WARM_SECONDS: the clocks ramped and the
    # table's keys and records resident in the Infinity Cache, as in the steady state the timed batches measure
    # (filler work that streams other memory would evict them; round 5 did)
    nextra = [0]

    def extra():
        bb, rr = calls[nextra[0] % nbufs]
        cx = eng.cfg(now_seconds=NOW + args.warmup + nextra[0])
        nextra[0] += 1
        if steer:
            steered_classify_flow(sops, dist, bufs[nextra[0] % nbufs][0], bufs[nextra[0] % nbufs][1], cx, world, rank)
        elif fn(eng.ctx, C.byref(bb), C.byref(rr), C.byref(cx), sptr):
            raise RuntimeError("ppe_classify_flow failed (warm-up)")
    if steer:  # (the steered steps exchange batches: every rank runs the same count)
        for _ in range(8):
            extra()
        torch.cuda.synchronize()
    else:
        warm_up(extra)
    eng.clear_counters()
    new0 = eng.flow_info()["new_flow"]
    # value: the K timed batches with no dispatch events (a start / end event pair on every classify launch cost the
    # stream ≈ 6 us per batch, profiles/r6_ab_runs.md r6u)
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
    info = eng.flow_info()
    # the classify (FlowFind) kernel alone: the dispatch timestamps (hipExtLaunchKernelGGL events) of K more batches
    # over the same flows (their packet times follow the timed ones'); a steered rank's launches are its own share of
    # every batch
    eng.timing(True)
    eng.timing_read(reset=True)
    barrier()
    for i in range(args.steps):
        step(args.warmup + args.steps + i)
    barrier()
    kern_ms, launches = eng.timing_read(reset=True)
    eng.timing(False)
    if dist is not None:
        t = torch.tensor([my_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        my_ms = float(t.item())
    mpps = n * args.steps * world / (my_ms / 1e3) / 1e6
    kern_avg_ms = kern_ms / max(launches, 1)
    owner = flow_owner_update()
    bpp = flow_bytes(stride, owner)
    achieved = bpp * n / (kern_avg_ms / 1e3) / 1e9
    # the whole batch (classify, flow kernels, update) against the in-kernel definition's bytes: the batch roofline
    batch_achieved = flow_bytes(stride) * n / (my_ms / args.steps / 1e3) / 1e9

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = flow_cpu_baseline(bufs[0][4], rules, eng.image(), flows,
                                args.nested_cpu_seconds if nested else args.cpu_seconds)

    line = None
    if rank == 0:
        tpp = traffic_per_packet(name)
        line = {
            "metric": FLOW_METRIC, "value": round(mpps, 2), "unit": "Mpps", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(my_ms / args.steps, 5), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic",
            "config": {"workload": f"{name}: {n} x 64B IPv4/UDP packets per GPU per batch over {flows} "
                                   f"bidirectional flows, {cfgd['rules']} five-tuple ACL rules, default FW",
                       "packets_per_gpu": n, "flows": flows, "rules": cfgd["rules"], "resident_batches": nbufs,
                       "parallelism": f"flow-sharded x{world}" + (" (all-to-all steering by flow hash)" if steer else "")},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBPS, 4),
                         "traffic": round(tpp * n) if tpp else None,
                         "kernel": "ppe_classify_kernel<FLOW> (FlowFind; found flows' updates "
                                   + ("to the owners' buckets, applied beside finalize by ppe_flow_post_kernel" if owner else
                                      "by one atomic per packet") + "; misses resolved by the flow kernels)",
                         "kernel_avg_us": round(kern_avg_ms * 1e3, 3), "bytes_per_pkt": bpp,
                         "timing": "batch_avg_us and value: the timed region's HIP events around its K batches (no "
                                   "dispatch events inside); kernel_avg_us: the dispatch timestamps of the classify "
                                   "launches of K more batches over the same flows, run right after it",
                         "batch_avg_us": round(my_ms / args.steps * 1e3, 3),
                         "batch_bytes_per_pkt": flow_bytes(stride),
                         "batch_frac": round(batch_achieved / HBM_PEAK_GBPS, 4),
                         "flow_update": "owner" if owner else "atomic"},
            "cpu_baseline": cpu,
            "parity_sample_ok": parity,
            "flow_table": info,
            "new_flows_in_timed_region": new_timed,
            "counters": {k: cnt[k] for k in ("pkts", "acl_fw", "acl_drop", "flow_proc_ok", "flow_proc_fail",
                                             "flow_node_nomem")},
        }
        if not nested:
            print(json.dumps(line), flush=True)
    eng.close()
    if nested:
        return nested_line(line)
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


def nested_line(line):
    """A stateful config's own line, reduced to what a nested configs entry carries."""
    if line is None:
        return None
    out = {k: line[k] for k in ("metric", "value", "unit", "ms_per_step", "roofline", "parity_sample_ok",
                                "cpu_baseline") if k in line}
    out["workload"] = line["config"]["workload"]
    for k in ("flow_table", "new_flows_in_timed_region", "counters", "defrag_info", "held_fragments_per_batch",
              "new_fcb_in_timed_region", "fcb_full_in_timed_region"):
        if k in line:
            out[k] = line[k]
    return out


def run_defrag(args, cfgd, dev, world, rank, dist, name=None, nested=False):
    """--config D1: ppe_defrag batch after batch on one stream.  Every batch is the same
    65,536-fragment slice of a make_fragment_stream mix with a different source-address byte, so every batch
    creates fresh FCBs (none meets an earlier batch's datagrams); the warmup's FCBs are aged out before the timed
    region.  N > 1: each rank reassembles its own batches (fragments are steered to GPUs by (sip, dip, ip_id)
    upstream, as the reference's cores own their FCB tables), weak scaling with no data-path collective."""
    from ppe import Defrag
    name = name or args.config
    n = (0 if nested else args.n) or cfgd["n"]
    hdr_stride = 128
    # timed calls: at most 24, each creating ≈ 34k fresh FCBs, so the run stays below the config's fcb_max (2^20):
    # past it the batches would measure FCB_FULL handling, not reassembly (profiles/r6_ab_runs.md r6d)
    steps = min(args.steps, 24)
    nvar = max(args.warmup, 1) + steps
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

    eng = Engine(dev.index)  # (the rank's device: cuda:0 for every rank under --shared-gpu)
    stream = torch.cuda.current_stream(dev)
    t_off = torch.from_numpy(off.view(np.int64)).to(dev)
    t_len = torch.from_numpy(lens.view(np.int32)).to(dev)
    t_ids = torch.arange(n, dtype=torch.int64, device=dev)

    # parity sample: batch variant 1 through a fresh table and the oracle's sequential Defrag
    parity, stats = None, None
    if rank == 0:
        try:  # (rank 0 only, no collectives: an error here must not leave the other ranks in a barrier)
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
        except Exception as e:
            import traceback
            print(f"bench.py: D1 parity sample failed:\n{traceback.format_exc()}", file=sys.stderr, flush=True)
            parity = False

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
    gpu_busy(dev)
    info0 = d.info()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    barrier()
    ev0.record(stream)
    for i in range(steps):
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
    mfps = n * steps * world / (my_ms / 1e3) / 1e6
    call_ms = my_ms / steps
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
        cpu = defrag_cpu_baseline(variant, off, lens, cfgd["fcb_max"],
                                  args.nested_cpu_seconds if nested else args.cpu_seconds)

    line = None
    if rank == 0:
        line = {
            "metric": DEFRAG_METRIC, "value": round(mfps, 2), "unit": "Mfps", "n_gpus": world,
            "steps": steps, "warmup": args.warmup, "ms_per_step": round(call_ms, 5), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic",
            "config": {"workload": f"{name}: {n} IPv4 fragments per GPU per batch (make_fragment_stream mix: "
                                   f"UDP/TCP/ICMP, reordered, duplicated, lost, overlapping, oversize), "
                                   f"fcb_max {cfgd['fcb_max']}, cache_max {cm}",
                       "fragments_per_gpu": n, "mean_frame_bytes": round(frame_bytes / n, 1),
                       "datagrams_per_batch": n_dgram, "parallelism": f"fcb-sharded x{world}"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBPS, 4),
                         "traffic": round(traffic_per_packet(name) * n) if traffic_per_packet(name) else None,
                         "kernel": "one ppe_defrag call (parse..assemble, 10 stream-ordered kernels)",
                         "call_avg_us": round(call_ms * 1e3, 3), "bytes_per_call": bytes_call},
            "cpu_baseline": cpu,
            "parity_sample_ok": parity,
            "parity_sample_stats": stats if rank == 0 else None,
            "defrag_info": info,
            "held_fragments_per_batch": held, "stored_fragments_per_batch": stored_frags,
            "new_fcb_in_timed_region": int(info["new_fcb"] - info0["new_fcb"]),
            "fcb_full_in_timed_region": int(info["st_fcb_full"] - info0["st_fcb_full"]),
        }
        if not nested:
            print(json.dumps(line), flush=True)
    d.close()
    eng.close()
    if nested:
        return nested_line(line)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
