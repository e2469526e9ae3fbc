#!/usr/bin/env python3
"""Profiling driver (diagnostics): `--launches` ring launches (ppe_classify_batches, batches_per_launch 0) of
`--batches` resident batches each, nothing else on the GPU, so rocprofv3 passes see only the steady-state kernel.

  python tools/ring_run.py --config C1 --batches 32 --launches 4 [--lib path.so] [--tune k=v,...]
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
    ap.add_argument("--config", default="C1")
    ap.add_argument("--batches", type=int, default=32)
    ap.add_argument("--launches", type=int, default=4)
    ap.add_argument("--nbufs", type=int, default=8)
    ap.add_argument("--lib", default=None)
    ap.add_argument("--tune", default="")
    ap.add_argument("--layout", default="packed", choices=("packed", "soa"), help="result layout (bench.py --layout)")
    a = ap.parse_args()
    a.nbufs = max(a.nbufs, a.batches)  # every batch of a launch distinct (its batch groups run concurrently)
    c = synth.CONFIGS[a.config]
    n = c["n"]
    rules = synth.make_rules(c["rules"])
    dev = torch.device("cuda:0")
    eng = Engine(0, lib=abi.load_variant(a.lib) if a.lib else None)
    eng.commit(rules, default_action=1)
    kv = {k: int(v) for k, v in (x.split("=") for x in a.tune.split(","))} if a.tune else {}
    eng.tuning(**{"batches_per_launch": 0, **kv})
    bufs = []
    gen = [synth.make_packets(n, rules, seed=synth.SEED + 1 + 7919 * g, kind=c["kind"], stride=64) for g in range(2)]
    for b in range(a.nbufs):  # 2 generated batches, each buffer its own device allocation (as bench.py)
        pk = gen[b % 2]
        hdr = torch.from_numpy(pk["hdr"]).to(dev)
        lens = torch.from_numpy(pk["len"].view(np.int32)).to(dev)
        outs = [torch.empty(n, dtype=torch.int32, device=dev) for _ in range(4)]
        if a.layout == "packed":  # the bench's default: 8-B packed results + the compact list
            pk8 = torch.empty(n, dtype=torch.int64, device=dev)
            outs.append(pk8)
            res = abi.Result(None, None, None, None, None, None, None, outs[3].data_ptr(), pk8.data_ptr())
        else:
            res = abi.Result(outs[0].data_ptr(), outs[1].data_ptr(), outs[2].data_ptr(), None, None, None, None,
                             outs[3].data_ptr())
        bufs.append((abi.Batch(hdr.data_ptr(), lens.data_ptr(), None, n, 64), res, hdr, lens, outs))
    cfg = Engine.cfg(now_seconds=1_700_000_000)
    sp = C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    ins = (abi.Batch * a.batches)(*(bufs[i % a.nbufs][0] for i in range(a.batches)))
    outs = (abi.Result * a.batches)(*(bufs[i % a.nbufs][1] for i in range(a.batches)))
    for _ in range(a.launches):
        assert eng.lib.ppe_classify_batches(eng.ctx, ins, outs, a.batches, C.byref(cfg), sp) == 0
    torch.cuda.synchronize()
    rd = float(np.minimum(gen[0]["len"].astype(np.int64) & 0xFFFF, 64).mean() + 4.0)
    print(f"{a.launches} ring launches x {a.batches} batches of {n} ({a.config}) {eng.launch_info()} "
          f"algorithmic_read_per_pkt {rd:.3f}")
    eng.close()


if __name__ == "__main__":
    main()
