#!/usr/bin/env python3
"""CPU analysis of the multi-tile kernel's block walk (tool, not product): for a config's rules and packets, how
many 2-level block reads each packet needs, how many of them fall outside the LDS-staged block prefix, and what a
lockstep group of 4 tiles (256 lanes, acl_walk_blocks_mt) waits for: the deepest lane sets the group's step count.

  python tools/walk_depth.py --config C3 [--n 65536] [--lds-blocks 4900] [--binth 1]

The walk is the kernel's (ppe_kernels.hip acl_walk_blocks_mt), vectorised with numpy over the image words built by
the product compiler (ppe_acl_build_image); the tuples come from the oracle's decode of the same packets.
"""
import argparse
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "packet-process-engine_amd"), str(ROOT / "oracle")]

from ppe import abi, synth  # noqa: E402
import pyoracle  # noqa: E402

W_JUMP, W_OFFBSEC, W_NBLOCKS, W_OFFBLOCKS, W_MAXBDEPTH = 14, 15, 16, 17, 18
BLK_LEAF = 0x80000000


def walk(img, keys):
    """keys: (n, 5) uint32 (sip, dip, sport, dport, proto).  Returns per-packet block indices visited (n, depth)."""
    n = len(keys)
    jump = int(img[W_JUMP])
    off_bsec, off_blocks, max_bd = int(img[W_OFFBSEC]), int(img[W_OFFBLOCKS]), int(img[W_MAXBDEPTH])
    blocks = img[off_blocks: off_blocks + 8 * int(img[W_NBLOCKS])].reshape(-1, 8)
    kx = np.concatenate([keys.astype(np.uint64), np.zeros((n, 11), np.uint64)], axis=1)  # slots >= 5 read key 0
    if jump:
        dim, shift = jump & 0xFF, (jump >> 8) & 0xFF
        blk = img[off_bsec + (keys[:, dim].astype(np.uint64) >> np.uint64(shift)).astype(np.int64)].astype(np.int64)
    else:
        blk = np.zeros(n, np.int64)
    path = np.full((n, max_bd), -1, np.int64)
    cnt = np.ones(n, np.int64)  # candidates of the leaf reached (leaf lists: count field of the exit)
    lists = int(img[12]) > 1
    live = np.ones(n, bool)
    rows = np.arange(n)
    for it in range(max_bd):
        if not live.any():
            break
        path[live, it] = blk[live]
        b = blocks[blk[live]].astype(np.uint64)
        k = kx[rows[live]]
        lw = b[:, 3]
        b0 = k[np.arange(len(k)), (lw & 15).astype(np.int64)] > b[:, 0]
        t1 = np.where(b0, b[:, 2], b[:, 1])
        k1 = ((lw >> np.where(b0, 8, 4).astype(np.uint64)) & 15).astype(np.int64)
        b1 = k[np.arange(len(k)), k1] > t1
        x = np.where(b0, np.where(b1, b[:, 7], b[:, 6]), np.where(b1, b[:, 5], b[:, 4])).astype(np.int64)
        leaf = (x & BLK_LEAF) != 0
        idx = rows[live]
        if lists:
            c = (x >> 23) & 0xFF
            esc = c == 255
            if esc.any():
                off_leaf = int(img[6])
                c[esc] = img[off_leaf + (x[esc] & 0x7FFFFF)]
            cnt[idx[leaf]] = np.maximum(c[leaf], 1)
        live[idx[leaf]] = False
        blk[idx[~leaf]] = x[~leaf]
    return path, cnt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--n", type=int, default=65536)
    ap.add_argument("--lds-blocks", type=int, default=4900, help="blocks [0, this) staged in LDS")
    ap.add_argument("--binth", type=int, default=0)
    ap.add_argument("--group", type=int, default=256, help="lanes walked in lockstep")
    args = ap.parse_args()
    c = synth.CONFIGS[args.config]
    rules = synth.make_rules(c["rules"])
    img, st = abi.build_image(rules, default_action=1, binth=args.binth)
    pk = synth.make_packets(args.n, rules, kind=c["kind"], stride=64)
    o = pyoracle.Oracle(rules, default_action=1)
    ref = o.classify_batch(pk["hdr"], pk["len"], cfg=o.cfg(0, 1, 0), nthreads=os.cpu_count() or 1)
    acl = ((ref["verdict"] >> 16) & 0x10) != 0  # PPE_F_ACL: packets that walk
    t = ref["tuple"]
    keys = np.stack([t[:, 0], t[:, 1], t[:, 2] & 0xFFFF, t[:, 2] >> 16, t[:, 3] & 0xFF], 1).astype(np.uint32)
    path, cnt = walk(img, keys)
    reads = (path >= 0).sum(1)
    l2 = ((path >= args.lds_blocks)).sum(1)
    reads[~acl] = 0
    l2[~acl] = 0
    print(f"{args.config}: blocks {int(img[W_NBLOCKS])}, max block depth {int(img[W_MAXBDEPTH])}, jump {int(img[W_JUMP]):#x},"
          f" LDS blocks {args.lds_blocks}, walking packets {acl.sum()} of {len(acl)}")
    print(f"block reads per walking packet: mean {reads[acl].mean():.2f}, from L2 {l2[acl].mean():.2f}")
    hist = np.bincount(reads[acl])
    print("reads histogram: " + ", ".join(f"{i}: {h / acl.sum():.3f}" for i, h in enumerate(hist) if h))
    g = args.group
    m = (len(reads) // g) * g
    steps = reads[:m].reshape(-1, g).max(1)
    l2steps = np.array([((path[i * g:(i + 1) * g] >= args.lds_blocks).any(0)).sum() for i in range(m // g)])
    print(f"lockstep groups of {g}: steps mean {steps.mean():.2f}, max {steps.max()}; steps with an L2 read mean "
          f"{l2steps.mean():.2f}")
    # dependent round trips of the whole lookup: block reads + one rule read per candidate scanned (serial leaf-list
    # loop; upper bound: every candidate of the leaf)
    cost = reads + np.where(acl, cnt, 0)
    cg = cost[:m].reshape(-1, g).max(1)
    print(f"leaf candidates: mean {cnt[acl].mean():.2f}, max {cnt[acl].max()}; walk + rule round trips per group "
          f"(deepest lane, candidates scanned serially): mean {cg.mean():.2f}, max {cg.max()}; image words {len(img)}")


if __name__ == "__main__":
    main()
