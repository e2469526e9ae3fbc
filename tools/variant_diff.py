#!/usr/bin/env python3
"""Diagnostic (GPU): run one batch through the product library and a variant library with the same outputs layout and
report where verdict / flow hash / ACL hit differ, against the oracle as a third opinion.
  python tools/variant_diff.py packet-process-engine_amd/libppe_hip_x.so [--config C1] [--part]"""
import argparse
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "packet-process-engine_amd"), str(ROOT / "oracle")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from ppe import Engine, abi, synth  # noqa: E402
import pyoracle  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("variant")
ap.add_argument("--config", default="C1")
ap.add_argument("--n", type=int, default=1 << 16)
ap.add_argument("--part", action="store_true")
a = ap.parse_args()
cfgd = synth.CONFIGS[a.config]
rules = synth.make_rules(cfgd["rules"])
pk = synth.make_packets(a.n, rules, kind=cfgd["kind"])
dev = torch.device("cuda:0")
hdr = torch.from_numpy(pk["hdr"]).to(dev)
lens = torch.from_numpy(pk["len"].astype(np.int32)).to(dev)
res = {}
for name, lib in (("prod", None), ("variant", abi.load_variant(str(Path(a.variant).resolve())))):
    e = Engine(0, lib=lib) if lib else Engine(0)
    e.commit(rules, default_action=1)
    out = {k: torch.full((a.n,), -7, dtype=torch.int32, device=dev) for k in ("verdict", "flow_hash", "acl_hit")}
    lst = torch.zeros(a.n + 64, dtype=torch.int32, device=dev)
    if a.part:
        out["part_idx"] = lst
    else:
        out["fw_idx"] = lst
        out["drop_idx"] = torch.zeros(a.n + 64, dtype=torch.int32, device=dev)
        out["tile_cnt"] = torch.zeros((a.n + 63) // 64, dtype=torch.int32, device=dev)
    e.classify_torch(hdr, lens, out, e.cfg(0, 1, 1_700_000_000))
    torch.cuda.synchronize()
    res[name] = {k: v.cpu().numpy() for k, v in out.items() if k in ("verdict", "flow_hash", "acl_hit")}
    res[name]["list"] = lst.cpu().numpy()
    e.close()
o = pyoracle.Oracle(rules, default_action=1)
ref = o.classify_batch(pk["hdr"], pk["len"], cfg=o.cfg(0, 1, 1_700_000_000), nthreads=8)
for k in ("verdict", "flow_hash", "acl_hit"):
    p, v = res["prod"][k], res["variant"][k]
    r = ref[k].astype(p.dtype)
    bad = np.nonzero(p != v)[0]
    print(f"{k}: prod==oracle {np.array_equal(p, r)}  variant==oracle {np.array_equal(v, r)}  prod!=variant at {len(bad)}"
          f" packets, first {bad[:5].tolist()}  prod {p[bad[:5]].tolist()}  variant {v[bad[:5]].tolist()}  oracle {r[bad[:5]].tolist()}")
print("list equal:", np.array_equal(res["prod"]["list"], res["variant"]["list"]))
