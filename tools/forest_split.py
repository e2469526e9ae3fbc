#!/usr/bin/env python3
"""CPU analysis (tool, not product): what an EffiCuts-style partition of a config's rules into K forests would do to
the multi-tile kernel's block walk.  Rules are split by address-prefix "largeness": A = both
prefixes longer than /L, B = sip /L or shorter only, C = dip only, D = both.  For each group (and for unions of
groups) the product compiler builds its own image and the kernel's block walk (tools/walk_depth.py) runs the config's
packets through it: block reads per packet, the lockstep group's step count (the deepest of 256 lanes) and the block
count.

  python tools/forest_split.py --config C3 --L 8 10 12
"""
import argparse
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "packet-process-engine_amd"), str(ROOT / "oracle"), str(ROOT / "tools")]

from ppe import abi, synth  # noqa: E402
import pyoracle  # noqa: E402
from walk_depth import W_MAXBDEPTH, W_NBLOCKS, walk  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--n", type=int, default=65536)
    ap.add_argument("--L", type=int, nargs="+", default=[10])
    ap.add_argument("--group", type=int, default=256)
    args = ap.parse_args()
    c = synth.CONFIGS[args.config]
    rules = synth.make_rules(c["rules"])
    pk = synth.make_packets(args.n, rules, kind=c["kind"], stride=64)
    o = pyoracle.Oracle(rules, default_action=1)
    ref = o.classify_batch(pk["hdr"], pk["len"], cfg=o.cfg(0, 1, 0), nthreads=os.cpu_count() or 1)
    acl = ((ref["verdict"] >> 16) & 0x10) != 0
    t = ref["tuple"]
    keys = np.stack([t[:, 0], t[:, 1], t[:, 2] & 0xFFFF, t[:, 2] >> 16, t[:, 3] & 0xFF], 1).astype(np.uint32)
    g = args.group
    m = (len(keys) // g) * g

    def stats(sub, tag):
        img, _ = abi.build_image(sub, default_action=1, binth=0)
        path, _ = walk(img, keys)
        reads = (path >= 0).sum(1)
        reads[~acl] = 0
        steps = reads[:m].reshape(-1, g).max(1)
        print(f"{tag:>10}: rules {len(sub):6d} blocks {int(img[W_NBLOCKS]):6d} max depth {int(img[W_MAXBDEPTH]):2d} "
              f"reads/packet {reads[acl].mean():.2f} (>=5: {(reads[acl] >= 5).mean():.4f}) "
              f"group steps mean {steps.mean():.2f} max {steps.max()}", flush=True)

    stats(rules, "all")
    sp, dp = rules["sip_mask"].astype(int), rules["dip_mask"].astype(int)
    for L in args.L:
        a, b = sp <= L, dp <= L
        A, B, C, D = ~a & ~b, a & ~b, ~a & b, a & b
        for tag, msk in (("A", A), ("B", B), ("C", C), ("D", D), ("A+B", A | B), ("B+C+D", B | C | D)):
            stats(rules[msk], f"L={L} {tag}")


if __name__ == "__main__":
    main()
