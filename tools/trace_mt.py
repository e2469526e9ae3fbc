#!/usr/bin/env python3
"""Diagnostic: per-round phase durations of the multi-tile round loop (split images: C3), from a library built with
-DPPE_MTTRACE=1 (make variant NAME=mttrace VFLAGS="-DPPE_MTTRACE=1 -DPPE_MTTRACE_SKIP=8").  One ring launch over
--batches distinct batches; rounds SKIP .. SKIP + 4 of every wave are stamped (s_memrealtime, 100 MHz).
Phases: load = round top -> decoded (the window loads' wait + decode), walk = decoded -> walked, finish = walked ->
records checked, results stored and drained; gap = previous round's end -> this round's top."""
import argparse
import ctypes as C
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "packet-process-engine_amd"), str(ROOT / "oracle")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from ppe import Engine, abi, synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", required=True)
    ap.add_argument("--config", default="C3")
    ap.add_argument("--batches", type=int, default=30)
    ap.add_argument("--tune", default="")
    args = ap.parse_args()
    c = synth.CONFIGS[args.config]
    n = c["n"]
    rules = synth.make_rules(c["rules"])
    dev = torch.device("cuda:0")
    eng = Engine(0, lib=abi.load_variant(str(Path(args.lib).resolve())))
    eng.commit(rules, default_action=1)
    if args.tune:
        eng.tuning(**{k: int(v) for k, v in (x.split("=") for x in args.tune.split(","))})
    pk = synth.make_packets(n, rules, seed=synth.SEED + 1, kind=c["kind"], stride=64)
    hdrs = [torch.from_numpy(pk["hdr"]).to(dev) for _ in range(args.batches)]
    lens = torch.from_numpy(pk["len"].view(np.int32)).to(dev)
    outs = [[torch.empty(n, dtype=torch.int32, device=dev) for _ in range(3)] for _ in range(args.batches)]
    p8 = [torch.empty(n, dtype=torch.uint8, device=dev) for _ in range(args.batches)]
    ins = (abi.Batch * args.batches)(*(abi.Batch(h.data_ptr(), lens.data_ptr(), None, n, 64) for h in hdrs))
    rs = (abi.Result * args.batches)(*(abi.Result(o[0].data_ptr(), o[1].data_ptr(), o[2].data_ptr(), None, None, None,
                                                  None, q.data_ptr()) for o, q in zip(outs, p8)))
    info = eng.launch_info()
    waves = info["grid"] * info["block"] // 64
    trace = torch.zeros(waves * 32, dtype=torch.int64, device=dev)
    cfg = eng.cfg(now_seconds=1_700_000_000)
    s = C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    for rep in range(3):
        trace.zero_()
        eng.lib.ppe_debug_trace(eng.ctx, C.c_void_p(trace.data_ptr()))
        eng.timing(True)
        eng.timing_read(reset=True)
        assert eng.lib.ppe_classify_batches(eng.ctx, ins, rs, args.batches, C.byref(cfg), s) == 0
        torch.cuda.synchronize()
        ms, _ = eng.timing_read(reset=True)
        t = trace.cpu().numpy().reshape(waves, 32)[:, 1:21].reshape(waves, 5, 4).astype(np.float64) * 0.01  # us
        ok = (t > 0).all(axis=2)
        ph = {"load+decode": t[:, :, 1] - t[:, :, 0], "walk": t[:, :, 2] - t[:, :, 1],
              "records+finish": t[:, :, 3] - t[:, :, 2]}
        gap = t[:, 1:, 0] - t[:, :-1, 3]
        gok = ok[:, 1:] & ok[:, :-1]
        print(f"rep {rep}: {ms * 1e3 / args.batches:.2f} us per batch, {ok.sum()} stamped rounds of {waves} waves "
              f"({info['image']}, {info['fetch']})")
        for k, v in ph.items():
            vv = v[ok]
            print(f"  {k:15s} mean {vv.mean():7.3f} us  p50 {np.median(vv):7.3f}  p90 {np.percentile(vv, 90):7.3f}")
        print(f"  {'gap':15s} mean {gap[gok].mean():7.3f} us")
        rt = (t[:, 4, 3] - t[:, 0, 0])[ok.all(axis=1)] / 5
        print(f"  round (5-round average) mean {rt.mean():.3f} us")
    eng.lib.ppe_debug_trace(eng.ctx, None)
    eng.close()


if __name__ == "__main__":
    main()
