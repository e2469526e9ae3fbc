#!/usr/bin/env python3
"""Diagnostics: where the time between the stream events around one ppe_classify_batches ring call goes
(event-to-event vs the kernel's dispatch timestamps), for K batches of C1."""
import ctypes as C
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "packet-process-engine_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from ppe import Engine, abi, synth  # noqa: E402


def main():
    n = 1 << 20
    rules = synth.make_rules(256)
    dev = torch.device("cuda:0")
    eng = Engine(0)
    eng.commit(rules, default_action=1)
    pk = synth.make_packets(n, rules)
    bufs = []
    for b in range(40):  # every batch of a launch distinct (batch groups run concurrently)
        hdr = torch.from_numpy(pk["hdr"]).to(dev)
        lens = torch.from_numpy(pk["len"].view(np.int32)).to(dev)
        outs = [torch.empty(n, dtype=torch.int32, device=dev) for _ in range(4)]
        bufs.append((abi.Batch(hdr.data_ptr(), lens.data_ptr(), None, n, 64),
                     abi.Result(outs[0].data_ptr(), outs[1].data_ptr(), outs[2].data_ptr(), outs[3].data_ptr(),
                                outs[3].data_ptr(), None, None), hdr, lens, outs))
    cfg = Engine.cfg(now_seconds=1_700_000_000)
    s = torch.cuda.current_stream(dev)
    sp = C.c_void_p(s.cuda_stream)
    for K in (1, 2, 8, 20, 32, 40):
        ins = (abi.Batch * K)(*(bufs[i % 40][0] for i in range(K)))
        outs = (abi.Result * K)(*(bufs[i % 40][1] for i in range(K)))
        for bpl in (0,):
            eng.tuning(batches_per_launch=bpl)
            res = []
            for it in range(6):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                eng.timing(True)
                eng.timing_read(reset=True)
                torch.cuda.synchronize()
                h0 = time.perf_counter()
                e0.record(s)
                assert eng.lib.ppe_classify_batches(eng.ctx, ins, outs, K, C.byref(cfg), sp) == 0
                e1.record(s)
                h1 = time.perf_counter()
                torch.cuda.synchronize()
                kms, nl = eng.timing_read(reset=True)
                eng.timing(False)
                res.append((e0.elapsed_time(e1) * 1e3, kms * 1e3, nl, (h1 - h0) * 1e6))
            r = np.median(np.array(res), axis=0)
            print(f"K={K:3d} bpl={bpl}: events {r[0]:9.1f} us  kernels {r[1]:9.1f} us ({int(r[2])} launches)  "
                  f"host call {r[3]:7.1f} us  per batch ev {r[0] / K:7.2f} kern {r[1] / K:7.2f}")
    # the same calls without per-launch timing events
    for K in (32,):
        ins = (abi.Batch * K)(*(bufs[i % 40][0] for i in range(K)))
        outs = (abi.Result * K)(*(bufs[i % 40][1] for i in range(K)))
        eng.tuning(batches_per_launch=0)
        for it in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record(s)
            assert eng.lib.ppe_classify_batches(eng.ctx, ins, outs, K, C.byref(cfg), sp) == 0
            e1.record(s)
            torch.cuda.synchronize()
            print(f"K={K} no timing events: {e0.elapsed_time(e1) * 1e3:.1f} us")
    eng.close()


if __name__ == "__main__":
    main()
