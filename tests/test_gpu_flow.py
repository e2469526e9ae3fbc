"""GPU parity of the stateful flow table (ppe_classify_flow / ppe_flow_age / ppe_flow_dump) against the oracle's
sequential FlowHandlePacket (tests/test_oracle_flow.py pins the oracle to dataplane/src/flow/flow.c).

Bar: bit-exact per-packet verdict, flow hash, ACL hit, compacted lists and counters, and the same table (key,
per-direction packet / byte counters, last-seen time) after every batch and aging step."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

import torch  # noqa: E402

import pyoracle  # noqa: E402
from ppe import Engine, abi, synth  # noqa: E402
from test_gpu_parity import check_compaction, check_part8, check_partition  # noqa: E402

DEV = torch.device("cuda:0")
NOW = 1_000_000


def gpu_flow(eng, hdr, lens, now, syn_check=1, part=False):
    n = len(lens)
    th = torch.from_numpy(np.ascontiguousarray(hdr)).to(DEV)
    tl = torch.from_numpy(np.ascontiguousarray(lens, np.uint32).view(np.int32)).to(DEV)
    # part: False = separate FW / DROP lists + tile counts, True = the partition list, "8" = its compact form
    names = ("verdict", "flow_hash", "acl_hit") + (
        ("part8",) if part == "8" else ("part_idx",) if part else ("fw_idx", "drop_idx", "tile_cnt"))
    out = {k: torch.full(((n + 63) // 64,) if k == "tile_cnt" else (n,), -7, dtype=torch.int32, device=DEV)
           for k in names}
    if part == "8":
        out["part8"] = torch.full((n + 64,), 0xEE, dtype=torch.uint8, device=DEV)
    eng.classify_flow_torch(th, tl, out, cfg=eng.cfg(0, syn_check, now))
    torch.cuda.synchronize()
    return {k: (v.cpu().numpy() if k in ("acl_hit", "part8") else v.cpu().numpy().view(np.uint32))
            for k, v in out.items()}


def table(d):
    """order-independent view of a flow dump"""
    cols = ("sip", "dip", "sport", "dport", "protocol", "pktcnts2d", "pktcntd2s", "bytecnts2d", "bytecntd2s",
            "last_seen")
    rows = sorted(tuple(int(x) for x in r) for r in zip(*(d[c] for c in cols)))
    return rows


class Pair:
    """The HIP flow table and the oracle's, fed the same batches."""

    def __init__(self, eng, rules, capacity, max_batch, default_action=0):
        self.eng = eng
        eng.commit(rules, default_action=default_action)
        eng.flow_create(capacity, max_batch)
        eng.clear_counters()
        self.o = pyoracle.Oracle(rules, default_action=default_action)
        self.ft = pyoracle.OracleFlow(self.o, capacity=capacity)
        self.counters = np.zeros(32, np.uint64)

    def batch(self, hdr, lens, now, syn_check=1, part=False):
        got = gpu_flow(self.eng, hdr, lens, now, syn_check, part)
        ref = self.ft.classify_batch(hdr, lens, cfg=self.o.cfg(0, syn_check, now))
        for k in ("verdict", "flow_hash", "acl_hit"):
            if not np.array_equal(got[k], ref[k]):
                bad = np.nonzero(got[k] != ref[k])[0]
                raise AssertionError(f"{k}: {len(bad)} mismatches, first {bad[:5].tolist()}: "
                                     f"gpu={got[k][bad[:5]].tolist()} ref={ref[k][bad[:5]].tolist()}")
        if part == "8":
            check_part8(got, len(lens))
        elif part:
            check_partition(got, len(lens))
        else:
            check_compaction(got, len(lens))
        self.counters += ref["counters"]
        cnt = self.eng.counters()
        assert [cnt[c] for c in abi.COUNTERS] == self.counters[:len(abi.COUNTERS)].tolist()
        return got, ref

    def same_table(self):
        assert table(self.eng.flow_dump()) == table(self.ft.dump())
        info, st = self.eng.flow_info(), self.ft.stats()
        assert (info["live"], info["new_flow"], info["del_flow"]) == (st["live"], st["new_flow"], st["del_flow"])
        return info

    def close(self):
        self.eng.flow_destroy()
        self.ft.close()


@pytest.fixture(scope="module")
def eng():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    e = Engine(0)
    yield e
    e.close()


@pytest.mark.parametrize("kind,stride", [("udp64", 64), ("imix", 128)])
def test_flow_batches_parity(eng, kind, stride):
    """Several batches over a shared flow population: misses, in-batch creation, hits in both directions, syn_check,
    ACL drops, malformed packets; the table is compared after every batch."""
    rules = synth.make_rules(256, seed=21)
    p = Pair(eng, rules, capacity=100000, max_batch=1 << 16, default_action=0)
    try:
        for b in range(4):
            pk = synth.make_flow_packets(40000, rules, n_flows=6000, seed=100 + b if b < 2 else 100, kind=kind,
                                         stride=stride, malformed_frac=0.01)
            # batches 0 and 2 share the template seed, so batch 2 revisits batch 0's flows
            got, _ = p.batch(pk["hdr"], pk["len"], NOW + b, part=(False, True, False, "8")[b])
            p.same_table()
        v = got["verdict"]
        assert ((v >> 16) & abi.F_FLOW).any() and ((v >> 16) & abi.F_TOCLIENT).any()
    finally:
        p.close()


def test_flow_large_rule_set(eng):
    """A 4,096-rule image does not fit a workgroup's LDS: the stateless classify runs a multi-tile plan, but the
    flow-table classify kernel (node walk, per-lane key slots) must get its own single-tile plan (a prefix of the
    node forest in LDS, the rest from L2).  Misses walk that image; the table is compared after every batch."""
    rules = synth.make_rules(4096, seed=31)
    p = Pair(eng, rules, capacity=100000, max_batch=1 << 16, default_action=0)
    try:
        for b in range(3):
            pk = synth.make_flow_packets(30000, rules, n_flows=8000, seed=300 + b, template_seed=300, stride=64,
                                         malformed_frac=0.01)
            p.batch(pk["hdr"], pk["len"], NOW + b, part=(b == 1))
            p.same_table()
    finally:
        p.close()


def test_flow_large_table_global_buckets(eng):
    """A table of more than 2^23 slots (capacity 2^22): the owner update's bucket entries no longer fit 4 B (slot
    within the owner past 15 bits), so the classify kernel writes 8-B entries to global memory instead of staging
    them in LDS; results and the table stay equal to the oracle's."""
    rules = synth.make_rules(64, seed=27)
    p = Pair(eng, rules, capacity=1 << 22, max_batch=1 << 15, default_action=0)
    try:
        for b in range(3):
            pk = synth.make_flow_packets(20000, rules, n_flows=3000, seed=500 + b, template_seed=500, stride=64,
                                         malformed_frac=0.01)
            p.batch(pk["hdr"], pk["len"], NOW + b, part=(b == 1))
        p.same_table()
    finally:
        p.close()


def test_flow_pool_exhaustion(eng):
    """More new flows than the pool holds, within one batch and across batches: the creators past the free count
    (in packet order) fail with FLOW_NOMEM, exactly as one core running the batch in order."""
    rules = synth.make_rules(64, seed=22)
    p = Pair(eng, rules, capacity=700, max_batch=1 << 14, default_action=0)
    try:
        for b in range(3):
            pk = synth.make_flow_packets(12000, rules, n_flows=2000, seed=200 + b, syn_frac=0.8)
            got, ref = p.batch(pk["hdr"], pk["len"], NOW + b, part="8" if b == 1 else False)
            p.same_table()
        assert ((ref["verdict"] & 0xFF) == abi.ST["FLOW_NOMEM"]).any()
        assert p.eng.counters()["flow_node_nomem"] > 0
    finally:
        p.close()


def test_flow_aging_and_rehash(eng):
    """Age flows out batch after batch (ppe_flow_age vs FlowAgeTimeoutCB) until the tombstones force rehashes; the
    table stays equal to the oracle's throughout."""
    rules = synth.make_rules(32, seed=23)
    p = Pair(eng, rules, capacity=2000, max_batch=4096, default_action=0)
    try:
        now = NOW
        for b in range(12):
            pk = synth.make_flow_packets(4096, rules, n_flows=1500, seed=300 + b, syn_frac=0.9)
            p.batch(pk["hdr"], pk["len"], now)
            now += 15
            d_gpu = p.eng.flow_age(now, 20)
            d_ref = p.ft.age(now, 20)
            assert d_gpu == d_ref
            info = p.same_table()
        assert info["del_flow"] > 0 and info["rehashes"] >= 1
    finally:
        p.close()


@pytest.mark.parametrize("capacity,uhash", [(10000, 0), (1 << 17, 0), (10000, 1)])
def test_flow_counter_folding(monkeypatch, capacity, uhash):
    """The packed per-flow counters fold into the wide ones when a field passes its threshold (lowered here to a few
    packets / bytes so every flow folds many times); totals stay exact under concurrent folds.  The small pool makes
    every batch a possible overflow (finalize checks the exact counts), the large one never.  uhash: the update
    kernel's LDS hash cut to one entry, so every flow after the first of its owner takes the full-hash path (direct
    atomics)."""
    monkeypatch.setenv("PPE_FLOW_FOLD_PKTS", "3")
    monkeypatch.setenv("PPE_FLOW_FOLD_BYTES", "500")
    if uhash:
        monkeypatch.setenv("PPE_FLOW_UPD_HASH", str(uhash))
    e = Engine(0)
    rules = synth.make_rules(16, seed=24)
    p = Pair(e, rules, capacity=capacity, max_batch=1 << 15, default_action=0)
    try:
        for b in range(3):
            pk = synth.make_flow_packets(30000, rules, n_flows=300, seed=400 + b, template_seed=400, syn_frac=0.9)
            p.batch(pk["hdr"], pk["len"], NOW + b)
            p.same_table()
    finally:
        p.close()
        e.close()


def test_flow_known_answers(eng):
    """The oracle's known-answer sequences (test_oracle_flow.py) through the HIP path."""
    from pktbuild import tcp_packet, udp_packet
    from test_oracle_flow import batch, rule
    A, B = 0x0A000001, 0x0A000002
    rules = rule(action=1, sip=B, sip_mask=32, dip=A, dip_mask=32)
    p = Pair(eng, rules, capacity=2, max_batch=64, default_action=0)
    try:
        fwd = udp_packet(sip=A, dip=B, sport=1234, dport=80)
        rev = udp_packet(sip=B, dip=A, sport=80, dport=1234)
        seqs = [[rev, rev, fwd, rev, fwd], [tcp_packet(flags=0x10), tcp_packet(flags=0x02), tcp_packet(flags=0x10)],
                [udp_packet(sport=7, dport=7), udp_packet(sport=8), udp_packet(sport=9)]]
        for i, s in enumerate(seqs):
            h, l = batch(s)
            p.batch(h, l, NOW + i)
            p.same_table()
    finally:
        p.close()


def test_failed_post_launch_fails_fast(eng):
    """when a batch's post-classify launch fails (forced by the test hook, after the classify launch
    ran), that call and every later call on the table return PPE_EIO immediately instead of running against an
    un-finalized batch; ppe_flow_destroy + ppe_flow_create give a working table again."""
    import ctypes as C
    import time
    lib = eng.lib
    lib.ppe_flow_debug_fail_post.argtypes = [C.c_uint32]
    rules = synth.make_rules(64, seed=25)
    p = Pair(eng, rules, capacity=10000, max_batch=1 << 13, default_action=0)
    pk = [synth.make_flow_packets(8000, rules, n_flows=800, seed=600 + b, template_seed=600) for b in range(3)]
    try:
        p.batch(pk[0]["hdr"], pk[0]["len"], NOW)
        lib.ppe_flow_debug_fail_post(1)
        with pytest.raises(RuntimeError, match="-5"):
            gpu_flow(eng, pk[1]["hdr"], pk[1]["len"], NOW + 1)
        t0 = time.perf_counter()
        for _ in range(3):
            with pytest.raises(RuntimeError, match="-5"):
                gpu_flow(eng, pk[2]["hdr"], pk[2]["len"], NOW + 2)
        assert time.perf_counter() - t0 < 10.0
        info = abi.FlowInfo()
        assert lib.ppe_flow_info(eng.ctx, C.byref(info)) == -5
        assert lib.ppe_flow_age(eng.ctx, NOW + 3, 10, None) == -5
        assert lib.ppe_flow_clear_stat(eng.ctx) == -5
        n = C.c_uint32()
        assert lib.ppe_flow_dump(eng.ctx, None, 0, C.byref(n)) == -5
        assert b"unusable" in lib.ppe_last_error(eng.ctx)
    finally:
        lib.ppe_flow_debug_fail_post(0)
        p.close()
    # a fresh table works and matches the oracle again
    p = Pair(eng, rules, capacity=10000, max_batch=1 << 13, default_action=0)
    try:
        for b in range(2):
            p.batch(pk[b]["hdr"], pk[b]["len"], NOW + b)
            p.same_table()
    finally:
        p.close()


def test_flow_argument_errors(eng):
    import ctypes as C
    lib = eng.lib
    b = abi.Batch(None, None, None, 0, 64)
    r = abi.Result(None, None, None, None, None, None, None)
    eng.flow_destroy()
    assert lib.ppe_classify_flow(eng.ctx, C.byref(b), C.byref(r), C.byref(eng.cfg()), None) == -22  # no table
    eng.flow_create(100, 128)
    th = torch.zeros((256, 64), dtype=torch.uint8, device=DEV)
    tl = torch.full((256,), 64, dtype=torch.int32, device=DEV)
    v = torch.zeros(256, dtype=torch.int32, device=DEV)
    b = abi.Batch(th.data_ptr(), tl.data_ptr(), None, 256, 64)
    r = abi.Result(v.data_ptr(), None, None, None, None, None, None)
    assert lib.ppe_classify_flow(eng.ctx, C.byref(b), C.byref(r), C.byref(eng.cfg()), None) == -22  # n > max_batch
    r = abi.Result(None, None, None, None, None, None, None)
    b.n = 64
    assert lib.ppe_classify_flow(eng.ctx, C.byref(b), C.byref(r), C.byref(eng.cfg()), None) == -22  # no verdict
    eng.flow_destroy()
