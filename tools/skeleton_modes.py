#!/usr/bin/env python3
"""Memory-skeleton variants over the bench's resident C1 batches (tool, not product): what the classify kernel's
traffic costs with its four 4-B results (mode 0), with a 1-B partition entry instead of the 4-B one (mode 2), with no
partition entry (mode 3), and with the reads alone (mode 1).  Interleaved rounds of 32-batch persistent launches of
libppe_calib.so's calib_kernel, the same launch shape as bench.py's `ceiling`.

  python tools/skeleton_modes.py [--rounds 6] [--nbufs 32]
"""
import argparse
import ctypes as C
import json
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "packet-process-engine_amd")]

import bench  # noqa: E402
from ppe import synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--nbufs", type=int, default=32)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    n = 1 << 20
    rules = synth.make_rules(synth.CONFIGS["C1"]["rules"])
    res = bench.Resident("C1", n, 64, args.nbufs, rules, 0, dev)
    lib = C.CDLL(str(ROOT / "packet-process-engine_amd" / "libppe_calib.so"))
    lib.ppe_calib_stream_timed.argtypes = [C.POINTER(bench._CalibArgs), C.c_uint32, C.c_void_p, C.POINTER(C.c_double)]
    sptr = C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    a = bench._CalibArgs()
    nb = min(32, args.nbufs)
    lists = [torch.empty(n, dtype=torch.int32, device=dev) for _ in range(nb)]  # 4 B per packet: every mode fits
    for i in range(nb):
        hdr, lens, out = res.bufs[i][:3]
        a.b[i] = bench._CalibBatch(hdr.data_ptr(), lens.data_ptr(), out["verdict"].data_ptr(),
                                   out["flow_hash"].data_ptr(), out["acl_hit"].data_ptr(), lists[i].data_ptr(), n, 0)
    a.nb = nb
    names = {0: "skeleton 12+4 B written", 2: "skeleton 12+1 B written", 3: "skeleton 12 B written",
             1: "read-only"}
    t = {m: [] for m in names}
    ms = C.c_double()
    for r in range(args.rounds + 1):
        for m in names:
            a.mode = m
            if lib.ppe_calib_stream_timed(C.byref(a), 0, sptr, C.byref(ms)) != 0:
                raise SystemExit("ppe_calib_stream failed")
            if r:
                t[m].append(ms.value * 1e3 / nb)  # us per 1M-packet batch
    out = {}
    for m, v in t.items():
        out[names[m]] = {"us_per_1M_med": round(float(np.median(v)), 3), "us_per_1M_min": round(float(min(v)), 3)}
        print(f"{names[m]:28s} med {np.median(v):7.3f}  min {min(v):7.3f} us per 1M packets", flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
