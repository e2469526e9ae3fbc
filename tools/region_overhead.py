#!/usr/bin/env python3
"""Diagnostic: what the value region of bench.py measures beyond the kernel.  For K batches of C1 in one
ppe_classify_batches call, interleaved over rounds: the region (torch events around the call, barrier + synchronize
on both sides) with the kernel's dispatch-timestamp events on and off, the host time of the call itself, and the
kernel time the dispatch events report.

  python tools/region_overhead.py --steps 32 128 --rounds 5
"""
import argparse
import ctypes as C
import statistics
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "packet-process-engine_amd"), str(ROOT / "oracle")]

import torch  # noqa: E402

import bench  # noqa: E402
from ppe import Engine, synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C1")
    ap.add_argument("--steps", type=int, nargs="+", default=[32, 128])
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--layout", default="packed")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    c = synth.CONFIGS[a.config]
    rules = synth.make_rules(c["rules"])
    eng = Engine(0)
    eng.tuning(batches_per_launch=0)
    eng.commit(rules, default_action=1)
    res = bench.Resident(a.config, c["n"], 64, max(a.steps), rules, 0, dev, layout=a.layout)
    cfg = eng.cfg(now_seconds=bench.NOW)
    stream = torch.cuda.current_stream(dev)
    sptr = C.c_void_p(stream.cuda_stream)

    def run(arrs):
        ins, outs = arrs
        assert eng.lib.ppe_classify_batches(eng.ctx, ins, outs, len(ins), C.byref(cfg), sptr) == 0

    out = {}
    arrs = {k: res.arrays(k) for k in a.steps}
    for k in a.steps:
        run(arrs[k])
    torch.cuda.synchronize()
    for _ in range(a.rounds):
        for k in a.steps:
            for timing in (False, True):
                eng.timing(timing)
                eng.timing_read(reset=True)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                e0.record(stream)
                t0 = time.perf_counter()
                run(arrs[k])
                host_us = (time.perf_counter() - t0) * 1e6
                e1.record(stream)
                torch.cuda.synchronize()
                reg = e0.elapsed_time(e1) * 1e3
                kern = eng.timing_read(reset=True)[0] * 1e3 if timing else float("nan")
                out.setdefault((k, timing), []).append((reg, host_us, kern))
    eng.timing(False)
    for (k, timing), v in sorted(out.items()):
        reg = statistics.median(x[0] for x in v)
        host = statistics.median(x[1] for x in v)
        kern = statistics.median(x[2] for x in v)
        print(f"steps {k:4d} timing {int(timing)}: region {reg:9.1f} us ({reg / k:7.3f} per step)  host call "
              f"{host:7.1f} us  kernel {kern:9.1f} us ({kern / k:7.3f} per step)  region - kernel {reg - kern:7.1f}")
    eng.close()


if __name__ == "__main__":
    main()
