"""The oracle reproduces the committed golden fixtures bit-exactly (guards the checker itself across rounds)."""
import numpy as np

import pyoracle


def test_oracle_vs_golden(golden):
    g = golden
    o = pyoracle.Oracle(g["rules"], g["used"], default_action=1)
    for tag, cfg in (("a", o.cfg(0, 1, int(g["now"]))), ("b", o.cfg(1, 0, int(g["now"])))):
        r = o.classify_batch(g["hdr"], g["len"], ts=g["ts"], cfg=cfg)
        for k in ("verdict", "flow_hash", "acl_hit", "tuple", "reach"):
            assert np.array_equal(r[k], g[f"{tag}_{k}"]), (tag, k)
        # the ABI 5 tuple differs from the frozen v1 one only in the fragments' Defrag fields (conftest.tuple_abi5)
        st = r["verdict"] & 0xFF
        fr = (st == 10) | (st == 11)
        assert fr.sum() > 20
        assert np.array_equal(g[f"{tag}_tuple"][~fr], g[f"{tag}_tuple_v1"][~fr])
        # per-reason counters as frozen; slot 31 (rx_bytes, added after the fixtures) is the sum of wire lengths
        assert np.array_equal(r["counters"][:31], g[f"{tag}_counters"][:31]), tag
        assert int(r["counters"][31]) == int(g["len"].astype(np.uint64).sum())


def test_golden_covers_every_decode_reason(golden):
    st = set((golden["a_verdict"] & 0xFF).tolist())
    assert set(range(18)) <= st  # every status except WINDOW_PUNT (stride-128 windows hold every header)
    assert (golden["a_acl_hit"] >= 0).sum() > 100
    assert len(np.unique(golden["a_acl_hit"][golden["a_acl_hit"] >= 0])) > 10


def test_oracle_threads_match_single(golden):
    g = golden
    o = pyoracle.Oracle(g["rules"], g["used"], default_action=1)
    a = o.classify_batch(g["hdr"], g["len"], ts=g["ts"], cfg=o.cfg(0, 1, int(g["now"])), nthreads=1)
    b = o.classify_batch(g["hdr"], g["len"], ts=g["ts"], cfg=o.cfg(0, 1, int(g["now"])), nthreads=5)
    for k in a:
        assert np.array_equal(a[k], b[k]), k
