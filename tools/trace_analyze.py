#!/usr/bin/env python3
"""Per-wave phase timeline of the classify kernel (diagnostics).  Runs a library built with -DPPE_TRACE on the
config's batch (4 resident buffers, like bench.py), captures one launch's timestamps (s_memrealtime, 100 MHz) and
prints where the waves' time goes and how the phases overlap across the launch.

  make -C packet-process-engine_amd variant NAME=trace VFLAGS=-DPPE_TRACE=1
  python tools/trace_analyze.py --lib packet-process-engine_amd/libppe_hip_trace.so --config C1 [--tune k=v,...]
"""
import argparse
import ctypes as C
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "packet-process-engine_amd"), str(ROOT / "oracle")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from ppe import Engine, abi, synth  # noqa: E402

NOW = 1_700_000_000
TICK_US = 0.01  # s_memrealtime: 100 MHz


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=str(ROOT / "packet-process-engine_amd/libppe_hip_trace.so"))
    ap.add_argument("--config", default="C1")
    ap.add_argument("--nbufs", type=int, default=4)
    ap.add_argument("--tune", default="")
    ap.add_argument("--bins", type=float, default=1.0, help="timeline bin width, us")
    ap.add_argument("--batches", type=int, default=1,
                    help="batches in the traced launch (one ppe_classify_batches ring launch); build the library "
                         "with -DPPE_TRACE_SKIP=k to sample tile iterations k..k+3 (mid-launch steady state)")
    ap.add_argument("--skip", type=int, default=0, help="the library's PPE_TRACE_SKIP")
    a = ap.parse_args()
    c = synth.CONFIGS[a.config]
    n = c["n"]
    rules = synth.make_rules(c["rules"])
    dev = torch.device("cuda:0")
    lib = abi.load_variant(a.lib)
    eng = Engine(0, lib=lib)
    eng.commit(rules, default_action=1)
    if a.tune:
        eng.tuning(**{k: int(v) for k, v in (x.split("=") for x in a.tune.split(","))})
    li = eng.launch_info()
    waves = li["grid"] * li["block"] // 64
    trace = torch.zeros(waves * 32, dtype=torch.int64, device=dev)
    bufs = []
    for b in range(a.nbufs):
        pk = synth.make_packets(n, rules, seed=synth.SEED + 1 + 7919 * b, kind=c["kind"], stride=64)
        hdr = torch.from_numpy(pk["hdr"]).to(dev)
        lens = torch.from_numpy(pk["len"].view(np.int32)).to(dev)
        outs = [torch.empty(n, dtype=torch.int32, device=dev) for _ in range(5)] + \
               [torch.empty((n + 63) // 64, dtype=torch.int32, device=dev)]
        bufs.append((abi.Batch(hdr.data_ptr(), lens.data_ptr(), None, n, 64),
                     abi.Result(*(o.data_ptr() for o in outs), None), hdr, lens, outs))
    cfg = Engine.cfg(now_seconds=NOW)
    sp = C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    for i in range(8):  # warm up, then trace the 9th launch (buffer 0 of a rotating set: HBM, not cache, resident)
        bb, rr = bufs[i % a.nbufs][:2]
        assert lib.ppe_classify(eng.ctx, C.byref(bb), C.byref(rr), C.byref(cfg), sp) == 0
    torch.cuda.synchronize()
    assert lib.ppe_debug_trace(eng.ctx, C.c_void_p(trace.data_ptr())) == 0
    if a.batches > 1:
        ins = (abi.Batch * a.batches)(*(bufs[i % a.nbufs][0] for i in range(a.batches)))
        outs = (abi.Result * a.batches)(*(bufs[i % a.nbufs][1] for i in range(a.batches)))
        eng.tuning(batches_per_launch=0)
        assert lib.ppe_classify_batches(eng.ctx, ins, outs, a.batches, C.byref(cfg), sp) == 0
    else:
        bb, rr = bufs[8 % a.nbufs][:2]
        assert lib.ppe_classify(eng.ctx, C.byref(bb), C.byref(rr), C.byref(cfg), sp) == 0
    torch.cuda.synchronize()
    lib.ppe_debug_trace(eng.ctx, None)
    t = trace.cpu().numpy().reshape(waves, 32).astype(np.int64)
    iters = t[:, 31]
    t0 = t[:, 0][t[:, 0] > 0].min()
    us = lambda x: (x - t0) * TICK_US  # noqa: E731
    print(f"{a.config}: {waves} waves ({li}), tiles per wave {np.bincount(iters).nonzero()[0].tolist()}")
    end = us(t[:, 22]).max()
    print(f"span entry..last wave done: {end:.2f} us; entry spread {us(t[:, 0]).max():.2f} us; "
          f"staging {np.median(us(t[:, 1]) - us(t[:, 0])):.2f} us median")
    ep = us(t[:, 23]) - us(t[:, 22])
    print(f"epilogue (loop exit .. counters flushed): median {np.median(ep):.2f} p90 {np.percentile(ep, 90):.2f} us; "
          f"last flush at {us(t[:, 23]).max():.2f} us; last loop exit at {end:.2f} us")
    names = ["wait window", "decode+hash", "ACL", "outputs+counters", "to next top"]
    skip = int(a.skip)
    for i in range(int(iters.max()) - skip):
        if i >= 4:
            break
        m = iters > i + skip
        b = 2 + 5 * i
        seg = [us(t[m, b + k + 1]) - us(t[m, b + k]) for k in range(4)]
        start = us(t[m, b])
        print(f" tile {i}: top at {np.median(start):6.2f} us (p10 {np.percentile(start, 10):.2f}, "
              f"p90 {np.percentile(start, 90):.2f})  " +
              "  ".join(f"{nm} {np.median(x):.2f}/{np.percentile(x, 90):.2f}" for nm, x in zip(names, seg)))
    # timeline: how many waves are in each phase per time bin
    nb = int(np.ceil(end / a.bins)) + 1
    hist = np.zeros((nb, 5))
    for i in range(min(4, int(iters.max()) - skip)):
        m = iters > i + skip
        b = 2 + 5 * i
        for k in range(4):
            lo, hi = us(t[m, b + k]), us(t[m, b + k + 1])
            for j in range(nb):
                ov = np.clip(np.minimum(hi, (j + 1) * a.bins) - np.maximum(lo, j * a.bins), 0, None)
                hist[j, k] += ov.sum() / a.bins
    staged = us(t[:, 1])
    for j in range(nb):
        hist[j, 4] = ((staged > j * a.bins) & (us(t[:, 0]) < (j + 1) * a.bins)).sum()
    print(f" timeline (mean waves per phase, {a.bins} us bins): staging | {' | '.join(names[:4])}")
    for j in range(nb):
        print(f"  {j * a.bins:6.1f}  " + "  ".join(f"{hist[j, k]:7.0f}" for k in (4, 0, 1, 2, 3)))


if __name__ == "__main__":
    main()
