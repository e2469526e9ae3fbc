#!/usr/bin/env python3
"""Host-resident batches, two ways (SURVEY.md §8(d) host-inclusive rate):
  copy       ppe_classify_host: H2D of the windows and lengths, classify, D2H of the results, chunked over 3 streams;
  zero-copy  ppe_classify on pinned host buffers directly: the kernel's loads and stores cross PCIe themselves
             (pinned host memory is device-addressable under ROCm's unified addressing).
Both bit-exact against each other; prints Mpps for each.  Usage: python tools/host_zero_copy.py [--n N] [--reps R]
"""
import argparse
import ctypes as C
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "packet-process-engine_amd"), str(ROOT / "oracle")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from ppe import Engine, abi, synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    rules = synth.make_rules(256)
    pk = synth.make_packets(a.n, rules, stride=64)
    eng = Engine(0)
    eng.commit(rules, default_action=1)
    cfg = eng.cfg(now_seconds=1_700_000_000)
    ph = torch.from_numpy(pk["hdr"]).pin_memory()
    pl = torch.from_numpy(pk["len"].view(np.int32)).pin_memory()
    names = ("verdict", "flow_hash", "acl_hit")
    outs = {k: torch.zeros(a.n, dtype=torch.int32).pin_memory() for k in names}
    ref = {k: torch.zeros(a.n, dtype=torch.int32).pin_memory() for k in names}
    b = abi.Batch(ph.data_ptr(), pl.data_ptr(), None, a.n, 64)
    r_copy = abi.Result(*(ref[k].data_ptr() for k in names), None, None, None, None)
    r_zc = abi.Result(*(outs[k].data_ptr() for k in names), None, None, None, None)
    lib = eng.lib
    res = {}
    for name in ("copy", "zero-copy", "copy", "zero-copy"):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.reps):
            if name == "copy":
                rc = lib.ppe_classify_host(eng.ctx, C.byref(b), C.byref(r_copy), C.byref(cfg), 1 << 18)
            else:
                rc = lib.ppe_classify(eng.ctx, C.byref(b), C.byref(r_zc), C.byref(cfg), None)
            assert rc == 0, lib.ppe_last_error(eng.ctx)
        torch.cuda.synchronize()
        res[name] = a.n * a.reps / (time.perf_counter() - t0) / 1e6
    same = all(torch.equal(outs[k], ref[k]) for k in names)
    print(json.dumps({"copy_mpps": round(res["copy"], 1), "zero_copy_mpps": round(res["zero-copy"], 1),
                      "identical": same, "n": a.n, "pcie_bytes_per_pkt": 68 + 12}))
    eng.close()


if __name__ == "__main__":
    main()
