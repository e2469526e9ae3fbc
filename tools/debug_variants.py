#!/usr/bin/env python3
"""Debug helper: classify one synthetic batch under each kernel variant and report mismatches vs the oracle."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "packet-process-engine_amd"), str(ROOT / "oracle")]
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

import pyoracle  # noqa: E402
from ppe import Engine, synth  # noqa: E402

NOW = 1_700_000_000
eng = Engine(0)
for resid in (0.0, 0.2):
    rules = synth.make_rules(200, seed=90, resid_frac=resid)
    pk = synth.make_packets(5000, rules, seed=91, kind="imix", stride=128, malformed_frac=0.1, with_ts=True)
    eng.commit(rules, default_action=1)
    o = pyoracle.Oracle(rules, default_action=1)
    for ts in (None, pk["ts"]):
        ref = o.classify_batch(pk["hdr"], pk["len"], ts=ts, cfg=o.cfg(0, 1, NOW))
        for tune in (dict(pipeline=1), dict(pipeline=4), dict(pipeline=1, lds_image=0)):
            eng.tuning(block=0, blocks_per_cu=0, pipeline=0, lds_image=1)
            eng.tuning(**tune)
            got = eng.classify_host(pk["hdr"], pk["len"], ts=ts, cfg=eng.cfg(0, 1, NOW))
            bad = np.nonzero((got["verdict"] != ref["verdict"]) | (got["acl_hit"] != ref["acl_hit"]))[0]
            print(f"resid={resid} ts={'y' if ts is not None else 'n'} {tune} launch={eng.launch_info()} bad={len(bad)}")
            for i in bad[:6]:
                print(f"   pkt {i} kind={pk['kinds'][i]} len={pk['len'][i]} got v={got['verdict'][i]:#x} hit={got['acl_hit'][i]}"
                      f" ref v={ref['verdict'][i]:#x} hit={ref['acl_hit'][i]}")
