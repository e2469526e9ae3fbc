#!/usr/bin/env python3
"""In-process A/B timing of ppe_defrag builds (diagnostics): bench.py's D1 workload (65,536-fragment batches, every
call with fresh datagrams) through one Defrag table per library build, the builds interleaved round by round so clock
drift hits each alike.  Each round ages the table empty, then times --calls calls with events on one stream.  The
last call's outputs of every build are compared with the first build's (same inputs, same table history).

  python tools/ab_defrag.py --variant base=packet-process-engine_amd/libppe_hip.so \
      --variant asm4=packet-process-engine_amd/libppe_hip_asm4.so
"""
import argparse
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "packet-process-engine_amd"), str(ROOT / "oracle"), str(ROOT)]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from ppe import Defrag, Engine, abi, synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variant", action="append", required=True, help="name=path/to/lib.so")
    ap.add_argument("--calls", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    import bench
    cfgd = synth.CONFIGS["D1"]
    n = cfgd["n"]
    a_full, o_full, l_full = synth.make_fragment_stream(int(n / 3.1) + 64, seed=synth.SEED + 7)
    off, lens = o_full[:n].copy(), l_full[:n].copy()
    end = int(off[-1]) + int(lens[-1])
    arena = np.zeros(end + 64, np.uint8)
    arena[:end] = a_full[:end]
    pos, _ = bench.defrag_batch_variants(arena, off, lens, a.calls)
    dev = torch.device("cuda:0")
    stream = torch.cuda.current_stream(dev)
    t_off = torch.from_numpy(off.view(np.int64)).to(dev)
    t_len = torch.from_numpy(lens.view(np.int32)).to(dev)
    t_ids = torch.arange(n, dtype=torch.int64, device=dev)
    base = torch.from_numpy(arena).to(dev)
    t_pos = torch.from_numpy(pos).to(dev)
    pkts = []
    for v in range(a.calls):
        t = base.clone()
        t[t_pos] = v + 2
        pkts.append(t)
    vs = []
    for spec in a.variant:
        name, path = spec.split("=", 1)
        eng = Engine(0, lib=abi.load_variant(str(Path(path).resolve())))
        d = Defrag(eng, fcb_max=cfgd["fcb_max"])
        vs.append(dict(name=name, eng=eng, d=d, out=d.alloc_out(n, 128), us=[]))
    torch.cuda.synchronize()
    now = bench.NOW
    for r in range(a.rounds + 1):   # round 0: warmup
        for v in vs:
            v["d"].age(now + 10**6, 20)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record(stream)
            for i in range(a.calls):
                v["d"].run_torch(pkts[i], t_off, t_len, v["out"], now + 10**6, ids=t_ids, stream=stream)
            e1.record(stream)
            torch.cuda.synchronize()
            if r:
                v["us"].append(e0.elapsed_time(e1) * 1e3 / a.calls)
        now += 10**7
    ref = vs[0]["out"]
    for v in vs:
        same = all(torch.equal(v["out"][k], ref[k]) for k in ref if ref[k] is not None)
        med = statistics.median(v["us"])
        print(f"{v['name']:>8}: median {med:7.2f} us/call  min {min(v['us']):7.2f}  "
              f"{n / med:8.1f} Mfps  outputs {'== ' + vs[0]['name'] if same else 'DIFFER'}", flush=True)
    for v in vs:
        v["d"].close()
        v["eng"].close()


if __name__ == "__main__":
    main()
