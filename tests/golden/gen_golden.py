#!/usr/bin/env python3
"""Regenerate the committed parity fixtures (run in the build container: needs oracle/liboracle.so and, for the
reference-hash fixture, oracle/_ref/libref_tluhash.so built from /root/reference).

golden_v1.npz      packets + rules + the oracle's expected outputs under two configurations; frozen so later rounds
                   (and the GPU box, which has no reference tree) check against the same bytes.
ref_tluhash_v1.npz 5-tuples and the flow hash computed by the REFERENCE's own dataplane/src/flow/tluhash.h
                   (compiled unmodified by oracle/Makefile) — pins the flow hash to reference code.
"""
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
ROOT = HERE.parent.parent
sys.path[:0] = [str(ROOT / "packet-process-engine_amd"), str(ROOT / "oracle")]

import pyoracle  # noqa: E402
from ppe import synth  # noqa: E402
from ppe.abi import RULE_DTYPE  # noqa: E402

NOW = 1_700_000_000


def edge_rules():
    """Hand-written rules for the A11 edges: /0 /1 /31 /32 prefixes, port and protocol range endpoints, overlaps
    where the lower index must win, MAC and time constraints, an empty port range (never matches)."""
    r = np.zeros(16, RULE_DTYPE)
    def rule(i, sip=0, sm=0, dip=0, dm=0, sp=(0, 65535), dp=(0, 65535), pr=(0, 255), act=0, smac=None, dmac=None,
             t=(0, 0)):
        r[i]["sip"], r[i]["sip_mask"], r[i]["dip"], r[i]["dip_mask"] = sip, sm, dip, dm
        r[i]["sport_start"], r[i]["sport_end"] = sp
        r[i]["dport_start"], r[i]["dport_end"] = dp
        r[i]["protocol_start"], r[i]["protocol_end"] = pr
        r[i]["action"] = act
        if smac is not None:
            r[i]["smac"] = smac
        if dmac is not None:
            r[i]["dmac"] = dmac
        r[i]["time_start"], r[i]["time_end"] = t
    pool = synth._mac_pool(np.random.default_rng(synth.SEED ^ 0xA5A5))
    rule(0, sip=0x0A000001, sm=32, dp=(80, 80), pr=(17, 17), act=1)             # exact host, exact port
    rule(1, sip=0x0A000000, sm=31, dp=(79, 81), pr=(6, 17), act=0)              # /31 covering rule 0's host
    rule(2, dip=0x80000000, dm=1, sp=(1024, 65535), act=1)                      # /1 upper half
    rule(3, sip=0xC0A80000, sm=16, dip=0xC0A80000, dm=16, act=0)               # 192.168/16 both ways
    rule(4, sip=0xC0A80100, sm=24, act=1)                                       # shadowed by rule 3 for dip in /16
    rule(5, dp=(0, 0), act=1)                                                   # port 0 only
    rule(6, dp=(65535, 65535), act=1)                                           # port 65535 only
    rule(7, pr=(1, 5), act=1)                                                   # protocol range w/o TCP/UDP
    rule(8, smac=pool[3], act=1)                                                # MAC-constrained (residual)
    rule(9, dmac=pool[5], sp=(0, 32767), act=0)
    rule(10, t=(NOW - 100, NOW + 100), dip=0x40000000, dm=2, act=1)             # time window
    rule(11, t=(NOW + 10, NOW + 20), act=1)                                     # future-only window
    rule(12, sp=(500, 400), act=1)                                              # empty range: never matches
    rule(13, sip=0x0A000001, sm=32, dp=(80, 80), pr=(17, 17), act=0)            # duplicate 5-tuple, lower loses
    rule(14, sip=0x01020304, sm=8, act=1)                                       # host bits set beyond the prefix
    rule(15, sip=0xAC100000, sm=12, dip=0xAC100000, dm=12, dp=(1, 1023), act=0)
    return r


def main():
    rng = np.random.default_rng(20251015)
    rules = np.concatenate([edge_rules(), synth.make_rules(48, seed=77, resid_frac=0.3, any_ip_frac=0.1)])
    used = np.ones(len(rules), np.uint8)
    used[[20, 33]] = 0  # FREE entries are skipped
    parts = [
        synth.make_packets(1024, rules, seed=11, kind="udp64", stride=128, malformed_frac=0.15, with_ts=True),
        synth.make_packets(1024, rules, seed=12, kind="imix", stride=128, malformed_frac=0.15, with_ts=True),
        synth.make_packets(512, rules, seed=13, kind="imix", stride=128, malformed_frac=0.6, hit_frac=0.9,
                           with_ts=True),
    ]
    hdr = np.concatenate([p["hdr"] for p in parts])
    lens = np.concatenate([p["len"] for p in parts])
    ts = np.concatenate([p["ts"] for p in parts])
    # steer some packets onto the hand-written edge rules
    for i in rng.choice(len(lens), 200, replace=False):
        h = hdr[i]
        if h[12] != 0x08 or h[13] != 0x00 or h[14] != 0x45:
            continue
        k = rng.integers(0, 6)
        if k == 0:
            h[26:30] = [10, 0, 0, 1]; h[23] = 17
        elif k == 1:
            h[26:30] = [10, 0, 0, 0]
        elif k == 2:
            h[26:30] = [192, 168, 1, 2]; h[30:34] = [192, 168, 7, 7]
        elif k == 3:
            h[36:38] = [0, 0]
        elif k == 4:
            h[36:38] = [255, 255]
        else:
            h[6:12] = synth._mac_pool(np.random.default_rng(synth.SEED ^ 0xA5A5))[3]
    out = {"rules": rules, "used": used, "hdr": hdr, "len": lens, "ts": ts, "now": np.uint64(NOW)}
    o = pyoracle.Oracle(rules, used, default_action=1)
    for tag, cfg in (("a", o.cfg(0, 1, NOW)), ("b", o.cfg(1, 0, NOW))):
        r = o.classify_batch(hdr, lens, ts=ts, cfg=cfg)
        for k in ("verdict", "flow_hash", "acl_hit", "tuple", "reach", "counters"):
            out[f"{tag}_{k}"] = r[k]
    np.savez_compressed(HERE / "golden_v1.npz", **out)
    st = out["a_verdict"] & 0xFF
    print("golden_v1: %d packets, %d rules, statuses %s" % (len(lens), len(rules), np.unique(st).tolist()))

    ref = pyoracle.ref_hash_lib()
    if ref is None:
        print("reference tree absent: ref_tluhash_v1.npz not regenerated")
        return
    n = 20000
    tup = np.zeros((n, 4), np.uint32)
    tup[:, 0] = rng.integers(0, 1 << 32, n, dtype=np.uint64)
    tup[:, 1] = rng.integers(0, 1 << 32, n, dtype=np.uint64)
    tup[:, 2] = rng.integers(0, 1 << 32, n, dtype=np.uint64)
    tup[:, 3] = rng.choice([6, 17, 1, 0, 255], n)
    # SURVEY.md §8(a) A9 known answers, both directions
    tup[0] = [0x0A000001, 0x0A000002, 1234 | (80 << 16), 17]
    tup[1] = [0x0A000002, 0x0A000001, 80 | (1234 << 16), 17]
    tup[2] = [0xC0A80101, 0xC0A80102, 12345 | (443 << 16), 6]
    h = np.zeros(n, np.uint32)
    ref.ref_flow_hashfn_batch(tup.ctypes.data, n, h.ctypes.data)
    assert h[0] == 0x554D7C02 and h[1] == 0x554D7C02 and h[2] == 0xB1B70370, [hex(x) for x in h[:3]]
    np.savez_compressed(HERE / "ref_tluhash_v1.npz", tuple=tup, hash=h)
    print("ref_tluhash_v1: %d tuples hashed by the reference's tluhash.h" % n)


if __name__ == "__main__":
    main()
