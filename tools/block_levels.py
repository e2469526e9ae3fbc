#!/usr/bin/env python3
"""CPU analysis (tool, not product): what k-level blocks would do to the multi-tile kernel's walk for a config.

For every packet that reaches the ACL, the node walk of the product image gives its root-to-leaf path (BFS node
indices).  A k-level block scheme groups the forest into blocks rooted at the nodes of depth 0, k, 2k, ...; a walk
to a leaf at depth D reads ceil(D / k) blocks.  Blocks are staged in LDS breadth-first (block roots in node order)
until `--lds-kb` is used up (k = 2: 32-B blocks, k = 3: 64-B blocks); the rest are L2 reads.  Reported per packet
and per lockstep group of 256 lanes (the deepest lane sets a group's step count).

  python tools/block_levels.py --config C3 [--n 65536] [--lds-kb 150]
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


def node_paths(img, keys):
    """(n, depth+1) node indices on each packet's path (-1 past its leaf), and its leaf depth."""
    n = len(keys)
    on, nn = int(img[5]), int(img[2])
    nodes = img[on:on + 4 * nn].reshape(nn, 4).astype(np.int64)
    kx = np.concatenate([keys.astype(np.int64), np.zeros((n, 3), np.int64)], axis=1)  # slot 5 = key 0
    jw = int(img[14])
    if jw:
        dim, shift = jw & 0xFF, (jw >> 8) & 0xFF
        e = img[32 + (keys[:, dim].astype(np.int64) >> shift)].astype(np.int64)
        cur, ks = ((e & 0xFFFFFF) // 4 - on) // 4, e >> 24
    else:
        cur, ks = np.zeros(n, np.int64), np.full(n, int(img[13]) >> 8, np.int64)
    maxd = int(img[10])
    path = np.full((n, maxd + 1), -1, np.int64)
    depth = np.zeros(n, np.int64)
    live = np.ones(n, bool)
    rows = np.arange(n)
    for d in range(maxd + 1):
        path[live, d] = cur[live]
        nd = nodes[cur]
        leaf = nd[:, 0] == 0xFFFFFFFF
        newly = live & leaf
        depth[newly] = d
        live &= ~leaf
        if not live.any():
            break
        gt = kx[rows, ks] > nd[:, 0]
        nxt = np.where(gt, nd[:, 2], nd[:, 1])
        nks = np.where(gt, nd[:, 3] >> 24, (nd[:, 3] >> 8) & 0xFF)
        cur = np.where(live, (nxt // 4 - on) // 4, cur)
        ks = np.where(live, nks, ks)
    return path, depth, nodes


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--n", type=int, default=65536)
    ap.add_argument("--lds-kb", type=float, default=150.0)
    ap.add_argument("--group", type=int, default=256)
    args = ap.parse_args()
    c = synth.CONFIGS[args.config]
    rules = synth.make_rules(c["rules"])
    img, st = abi.build_image(rules, default_action=1)
    pk = synth.make_packets(args.n, rules, kind=c["kind"], stride=64)
    o = pyoracle.Oracle(rules, default_action=1)
    ref = o.classify_batch(pk["hdr"], pk["len"], cfg=o.cfg(0, 1, 0), nthreads=os.cpu_count() or 1)
    acl = ((ref["verdict"] >> 16) & 0x10) != 0
    t = ref["tuple"]
    keys = np.stack([t[:, 0], t[:, 1], t[:, 2] & 0xFFFF, t[:, 2] >> 16, t[:, 3] & 0xFF], 1).astype(np.uint32)
    path, depth, nodes = node_paths(img, keys)
    nn = len(nodes)
    # node depths (BFS forest: children after parents)
    nd_depth = np.zeros(nn, np.int64)
    on = int(img[5])
    inner = nodes[:, 0] != 0xFFFFFFFF
    for k in np.nonzero(inner)[0]:
        for ch in ((nodes[k, 1] // 4 - on) // 4, (nodes[k, 2] // 4 - on) // 4):
            nd_depth[ch] = nd_depth[k] + 1
    jw = int(img[14])
    bjt = 4 * (1 << ((jw >> 16) & 0xFF)) if jw else 0
    print(f"{args.config}: nodes {nn}, max depth {int(img[10])}, walking packets {acl.sum()}, leaf depth mean "
          f"{depth[acl].mean():.2f}, jump table {bjt} B")
    g = args.group
    m = (args.n // g) * g
    for k, bbytes in ((2, 32), (3, 64), (4, 128)):
        roots = np.nonzero(inner & (nd_depth % k == 0))[0]  # block roots, in node (BFS) order
        cap = int((args.lds_kb * 1024 - bjt) // bbytes)
        rank = np.full(nn, -1, np.int64)
        rank[roots] = np.arange(len(roots))
        reads = np.where(acl, (depth + k - 1) // k, 0)
        # the block roots on each path: depths 0, k, 2k, ... < leaf depth
        cols = np.arange(0, path.shape[1], k)
        bp = path[:, cols]
        valid = (cols[None, :] < depth[:, None]) & acl[:, None]
        l2 = valid & (rank[np.maximum(bp, 0)] >= cap)
        steps = reads[:m].reshape(-1, g).max(1)
        l2steps = l2[:m].reshape(-1, g, l2.shape[1]).any(1).sum(1)
        print(f"  k={k} ({bbytes}-B blocks): blocks {len(roots)} ({len(roots) * bbytes / 1e6:.2f} MB), LDS holds {cap};"
              f" reads/pkt {reads[acl].mean():.2f}, L2 reads/pkt {l2.sum(1)[acl].mean():.2f}; group steps "
              f"{steps.mean():.2f} (max {steps.max()}), group steps with an L2 read {l2steps.mean():.2f}")


if __name__ == "__main__":
    main()
