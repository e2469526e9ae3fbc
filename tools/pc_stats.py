#!/usr/bin/env python3
"""Diagnostic: where the producer / consumer walk (PF_PC) waits.  Runs a config's ring launch on a library built with
-DPPE_PC_STATS=1 (make variant NAME=pcstats VFLAGS=-DPPE_PC_STATS=1) and prints, per role, the queue polls per tile
(each poll is an s_sleep of 128 cycles) and the tiles each role handled.

  python tools/pc_stats.py --lib packet-process-engine_amd/libppe_hip_pcstats.so --config C3
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", required=True)
    ap.add_argument("--config", default="C3")
    ap.add_argument("--batches", type=int, default=30)
    ap.add_argument("--tune", default="pipeline=6")
    args = ap.parse_args()
    c = synth.CONFIGS[args.config]
    n = c["n"]
    rules = synth.make_rules(c["rules"])
    dev = torch.device("cuda:0")
    eng = Engine(0, lib=abi.load_variant(str(Path(args.lib).resolve())))
    eng.commit(rules, default_action=1)
    eng.tuning(**{k: int(v) for k, v in (x.split("=") for x in args.tune.split(",") if x)})
    pk = synth.make_packets(n, rules, seed=synth.SEED + 1, kind=c["kind"], stride=64)
    hdrs = [torch.from_numpy(pk["hdr"]).to(dev) for _ in range(args.batches)]
    lens = torch.from_numpy(pk["len"].view(np.int32)).to(dev)
    outs = [{k: torch.empty(n, dtype=torch.int32, device=dev) for k in ("v", "h", "a")} for _ in range(args.batches)]
    p8 = [torch.empty(n, dtype=torch.uint8, device=dev) for _ in range(args.batches)]
    ins = (abi.Batch * args.batches)(*(abi.Batch(h.data_ptr(), lens.data_ptr(), None, n, 64) for h in hdrs))
    rs = (abi.Result * args.batches)(*(abi.Result(o["v"].data_ptr(), o["h"].data_ptr(), o["a"].data_ptr(), None, None,
                                                  None, None, q.data_ptr()) for o, q in zip(outs, p8)))
    trace = torch.zeros(64, dtype=torch.int64, device=dev)
    cfg = eng.cfg(now_seconds=1_700_000_000)
    s = C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    for rep in range(3):
        trace.zero_()
        eng.lib.ppe_debug_trace(eng.ctx, C.c_void_p(trace.data_ptr()))
        eng.timing(True)
        eng.timing_read(reset=True)
        assert eng.lib.ppe_classify_batches(eng.ctx, ins, rs, args.batches, C.byref(cfg), s) == 0
        torch.cuda.synchronize()
        ms, launches = eng.timing_read(reset=True)
        t = trace.cpu().numpy()
        for r, name in ((0, "producer"), (4, "consumer")):
            polls, tiles, waves = int(t[r]), int(t[r + 1]), int(t[r + 2])
            print(f"rep {rep} {name}: waves {waves} tiles {tiles} polls {polls} polls/tile {polls / max(tiles, 1):.2f}")
        print(f"rep {rep}: {ms * 1e3 / args.batches:.2f} us per batch ({launches} launches) {eng.launch_info()}")
    eng.lib.ppe_debug_trace(eng.ctx, None)
    eng.close()


if __name__ == "__main__":
    main()
