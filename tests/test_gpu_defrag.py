"""GPU parity of IPv4 reassembly (ppe_defrag / ppe_defrag_age through the C ABI) against the oracle's sequential
Defrag (tests/test_oracle_defrag.py pins the oracle to dataplane/src/decode/decode-defrag.c).

Bar: bit-exact per-fragment status (with the teardrop bit), datagram index, datagram count, length, bytes, window and
fragment-id list, the same fragments dropped by every aging step, and identical counters; then the reassembled
datagrams classify exactly as the oracle classifies the oracle's datagrams."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

import torch  # noqa: E402

import pyoracle  # noqa: E402
from pktbuild import arena, ip_frag, udp  # noqa: E402
from ppe import Defrag, Engine, abi, synth  # noqa: E402
from test_gpu_parity import gpu_classify  # noqa: E402

DEV = torch.device("cuda:0")
NOW = 1_000_000


@pytest.fixture(scope="module")
def eng():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    e = Engine(0)
    yield e
    e.close()


class DfPair:
    """The HIP FCB table and the oracle's, fed the same fragment batches."""

    def __init__(self, eng, stride=128, **cfg):
        self.g = Defrag(eng, **cfg)
        o_cfg = dict(fcb_max=cfg.get("fcb_max", 0), cache_max=cfg.get("cache_max", 0),
                     frag_buf=cfg.get("frag_buf_bytes", 0), reasm_buf=cfg.get("reasm_buf_bytes", 0))
        self.o = pyoracle.OracleDefrag(**o_cfg)
        self.stride = stride
        self.cm = self.g.info_["cache_max"]
        self.rb = self.g.info_["reasm_buf_bytes"]

    def close(self):
        self.g.close()
        self.o.close()

    def batch(self, a, off, lens, now, ids=None):
        n = len(lens)
        ref = self.o.batch(a, off, lens, now, ids=ids)
        out = self.g.alloc_out(n, self.stride)
        for v in out.values():
            v.fill_(-7) if v.dtype != torch.uint8 else v.fill_(0xA5)
        ta = torch.from_numpy(np.ascontiguousarray(a)).to(DEV)
        to = torch.from_numpy(np.ascontiguousarray(off, np.uint64).view(np.int64)).to(DEV)
        tl = torch.from_numpy(np.ascontiguousarray(lens, np.uint32).view(np.int32)).to(DEV)
        ti = torch.from_numpy(np.ascontiguousarray(ids, np.uint64).view(np.int64)).to(DEV) if ids is not None else None
        self.g.run_torch(ta, to, tl, out, now, ids=ti)
        torch.cuda.synchronize()
        got = {k: v.cpu().numpy() for k, v in out.items()}
        nd = ref["n_dgram"]
        st = got["status"].view(np.uint32)
        if not np.array_equal(st, ref["status"]):
            bad = np.nonzero(st != ref["status"])[0]
            raise AssertionError(f"status: {len(bad)} mismatches, first {bad[:6].tolist()}: "
                                 f"gpu={st[bad[:6]].tolist()} ref={ref['status'][bad[:6]].tolist()}")
        assert int(got["n_dgram"][0]) == nd
        assert np.array_equal(got["dgram_of"].view(np.uint32), ref["dgram_of"])
        assert np.array_equal(got["dgram_len"].view(np.uint32), ref["dgram_len"])   # 0 past the count
        assert np.array_equal(got["dgram_frags"].view(np.uint64)[:nd], ref["dgram_frags"][:nd])
        for j in range(nd):
            m = int(ref["dgram_len"][j])
            assert np.array_equal(got["dgram_pkt"][j, :m], ref["dgram_pkt"][j, :m]), f"datagram {j} bytes"
            w = np.zeros(self.stride, np.uint8)
            w[:min(m, self.stride)] = ref["dgram_pkt"][j, :min(m, self.stride)]
            assert np.array_equal(got["dgram_hdr"][j], w), f"datagram {j} window"
        # rows past the count are not written (the 0xA5 fill stays): only their length 0 is part of the ABI
        assert (got["dgram_hdr"][nd:] == 0xA5).all() and (got["dgram_frags"].view(np.uint64)[nd:] != 0).all()
        return got, ref

    def age(self, now, timeout=20):
        gi, gf = self.g.age(now, timeout)
        oi, of = self.o.age(now, timeout)
        assert gf == of
        assert sorted(gi.tolist()) == sorted(oi.tolist())

    def check_stats(self):
        gi, os_ = self.g.info(), self.o.stats()
        for k, v in os_.items():
            assert gi[k] == v, (k, gi[k], v)


def replay(eng, a, o, l, bsz, now0=NOW, every_age=1, timeout=20, **cfg):
    p = DfPair(eng, **cfg)
    try:
        ids = (np.arange(len(l), dtype=np.uint64) * 3 + 11)
        for k, b in enumerate(range(0, len(l), bsz)):
            p.batch(a, o[b:b + bsz], l[b:b + bsz], now0 + k, ids=ids[b:b + bsz])
            if (k + 1) % every_age == 0:
                p.age(now0 + k, timeout)
        p.age(now0 + 10**6, timeout)
        p.check_stats()
    finally:
        p.close()


@pytest.mark.parametrize("seed,bsz", [(1, 4096), (2, 512), (3, 7), (4, 65536)])
def test_stream_vs_oracle(eng, seed, bsz):
    a, o, l = synth.make_fragment_stream(1500 if bsz > 7 else 200, seed=seed)
    replay(eng, a, o, l, bsz, every_age=3)


def test_unaligned_frames_and_pressure(eng):
    """Byte-aligned frames (the stash's byte path), a small FCB pool (FCB_FULL churn) and a short cache."""
    a, o, l = synth.make_fragment_stream(1200, seed=9, align=1)
    replay(eng, a, o, l, 1024, fcb_max=40, cache_max=3)


def test_cache_max_16_and_big_buffers(eng):
    a, o, l = synth.make_fragment_stream(800, seed=10, jumbo=0.1)
    replay(eng, a, o, l, 2048, cache_max=16, reasm_buf_bytes=16384, timeout=5)


@pytest.mark.parametrize("fcb_max", [1 << 20, 1000])
def test_large_batch_lookback(eng, fcb_max):
    """One 524,288-fragment batch: 2,048 admission workgroups, more than the GPU holds at once beside the other
    work, so the look-back ranking the creators crosses workgroups that start late.  With fcb_max 1000 the batch's
    ~170k creators overflow the pool and exactly the first 1,000 in index order may get FCBs: any rank error shows in
    the statuses.  Status, datagram index, count, lengths and fragment ids against the oracle (bytes: the other
    tests)."""
    import bench
    a1, o1, l1 = synth.make_fragment_stream(int(65536 / 3.1) + 64, seed=31)
    n1 = 65536
    off1, len1 = o1[:n1].copy(), l1[:n1].copy()
    end = int(off1[-1]) + int(len1[-1])
    base = np.zeros(end + 64, np.uint8)
    base[:end] = a1[:end]
    _, variant = bench.defrag_batch_variants(base, off1, len1, 8)
    copies = 8
    arena_all = np.concatenate([variant(v + 1) for v in range(copies)])
    off = np.concatenate([off1 + np.uint64(v * len(base)) for v in range(copies)])
    lens = np.tile(len1, copies)
    n = len(lens)
    ids = np.arange(n, dtype=np.uint64) * 5 + 3
    g = Defrag(eng, fcb_max=fcb_max, max_batch=n)
    o = pyoracle.OracleDefrag(fcb_max=fcb_max)
    try:
        ref = o.batch(arena_all, off, lens, NOW, ids=ids, full=False)
        out = g.alloc_out(n, 128, full=False)
        g.run_torch(torch.from_numpy(arena_all).to(DEV),
                    torch.from_numpy(off.view(np.int64)).to(DEV),
                    torch.from_numpy(lens.view(np.int32)).to(DEV), out, NOW,
                    ids=torch.from_numpy(ids.view(np.int64)).to(DEV))
        torch.cuda.synchronize()
        st = out["status"].cpu().numpy().view(np.uint32)
        bad = np.nonzero(st != ref["status"])[0]
        assert len(bad) == 0, f"status: {len(bad)} mismatches, first {bad[:6].tolist()}"
        nd = ref["n_dgram"]
        assert int(out["n_dgram"].item()) == nd
        assert np.array_equal(out["dgram_of"].cpu().numpy().view(np.uint32), ref["dgram_of"])
        assert np.array_equal(out["dgram_len"].cpu().numpy().view(np.uint32), ref["dgram_len"])
        assert np.array_equal(out["dgram_frags"].cpu().numpy().view(np.uint64)[:nd], ref["dgram_frags"][:nd])
        gi, os_ = g.info(), o.stats()
        for k, v in os_.items():
            assert gi[k] == v, (k, gi[k], v)
    finally:
        g.close()
        o.close()


def test_window_64(eng):
    a, o, l = synth.make_fragment_stream(600, seed=11)
    p = DfPair(eng, stride=64)
    try:
        p.batch(a, o, l, NOW)
    finally:
        p.close()


def test_datagrams_classify_like_the_oracle(eng):
    """Defrag → classify of the reassembled batch (DecodeTCP / DecodeUDP / flow hash / ACL on the datagram,
    decode-ipv4.c:241-290) equals the oracle classifying the oracle's datagrams."""
    from ppe import synth as s
    rules = s.make_rules(256)
    eng.commit(rules)
    orc = pyoracle.Oracle(rules)
    a, o, l = synth.make_fragment_stream(1500, seed=12)
    p = DfPair(eng, stride=128)
    try:
        got, ref = p.batch(a, o, l, NOW)
    finally:
        p.close()
    n = len(l)
    res = gpu_classify(eng, got["dgram_hdr"], got["dgram_len"].view(np.uint32), cfg=eng.cfg(now_seconds=NOW))
    nd = ref["n_dgram"]
    assert nd > 100
    win = np.zeros((n, 128), np.uint8)
    win[:nd] = ref["dgram_pkt"][:nd, :128]
    want = orc.classify_batch(win, ref["dgram_len"], cfg=orc.cfg(now_seconds=NOW))
    for k in ("verdict", "flow_hash", "acl_hit"):
        assert np.array_equal(res[k], want[k]), k
    st = res["verdict"][:nd] & 0xFF
    assert (st <= abi.ST["ACL_DROP"]).sum() > nd // 2          # most datagrams reach the ACL
    assert (res["verdict"][nd:] & 0xFF == abi.ST["L2_HEADER_ERR"]).all()   # padding entries (length 0)


def test_small_cases_and_errors(eng):
    S, D = 0x0A000001, 0x0A000002
    l4 = udp(1, 2, bytes(8))
    p = DfPair(eng)
    try:
        frames = [ip_frag(17, S, D, 1, 0, True, l4[:8]), ip_frag(17, S, D, 1, 8, False, l4[8:]),
                  ip_frag(17, S, D, 1, 0, True, l4[:8])]
        a, o, l = arena(frames)
        got, _ = p.batch(a, o, l, NOW)
        assert list(got["status"]) == [0, 1, 5]
        a, o, l = arena([frames[0]])
        p.batch(a, o, l, NOW)                              # n = 1: DELETED
        p.age(NOW + 1)
        p.batch(a, o, l, NOW + 2)                          # a fresh FCB after aging
        p.check_stats()
        # empty batch: nothing launched, nothing changes
        b = abi.FragBatch(None, None, None, None, 0, 0, NOW)
        oo = abi.DefragOut()
        assert p.g.lib.ppe_defrag(p.g.h, b, oo, None) == 0
        # too many fragments
        b = abi.FragBatch(1, 1, 1, None, p.g.info_["max_batch"] + 1, 0, NOW)
        assert p.g.lib.ppe_defrag(p.g.h, b, oo, None) == -22
    finally:
        p.close()


def test_groups_past_the_slots(eng):
    """FCBs with more fragments in one batch than the grouping's 15 slots per group (the rest go to the overflow
    list and the group's head steps them in index order): datagrams cut into 12 / 15 / 16 / 17 / 40 eight-byte
    fragments plus duplicates, shuffled together in one batch, with cache_max 8 (CACHE_FULL past it: the statuses
    depend on the order) and 16."""
    rng = np.random.default_rng(77)
    S, D = 0x0A000001, 0x0A0000FE
    frames = []
    for k, nf in enumerate([12, 15, 16, 17, 40]):
        l4 = udp(1000 + k, 53, rng.integers(0, 256, 8 * nf - 8, dtype=np.uint8).tobytes())
        frs = [ip_frag(17, S + k, D, 100 + k, 8 * f, f < nf - 1, l4[8 * f:8 * f + 8]) for f in range(nf)]
        frames += frs + [frs[f] for f in rng.choice(nf, 4)]
    frames = [frames[i] for i in rng.permutation(len(frames))]
    a, o, l = arena(frames)
    for cm in (8, 16):
        p = DfPair(eng, cache_max=cm)
        try:
            p.batch(a, o, l, NOW)
            p.check_stats()
        finally:
            p.close()


def test_one_key_flood_is_linear(eng):
    """one batch of 40,000 fragments of which 24,000 share one FCB key (duplicates of one datagram's
    fragments, as an attacker would send them), interleaved with 400 other datagrams that each pass their group's 15
    slots too.  Parity with the oracle, and the batch must finish in well under a second: the group heads enumerate
    their members in one pass over the batch, not one scan of a shared overflow list per member (which took
    ~10^9 serial loads here)."""
    import time
    rng = np.random.default_rng(78)
    S, D = 0x0B000001, 0x0B0000FE
    l4 = udp(4000, 53, rng.integers(0, 256, 8 * 5, dtype=np.uint8).tobytes())
    flood = [ip_frag(17, S, D, 7, 8 * f, f < 5, l4[8 * f:8 * f + 8]) for f in range(6)]
    frames = [flood[f] for f in rng.integers(0, 6, 24000)]
    for k in range(400):
        l4k = udp(5000 + k, 53, rng.integers(0, 256, 8 * 3, dtype=np.uint8).tobytes())
        frs = [ip_frag(17, S + 1 + k, D, 9, 8 * f, f < 3, l4k[8 * f:8 * f + 8]) for f in range(4)]
        frames += [frs[f] for f in rng.integers(0, 4, 40)]
    frames = [frames[i] for i in rng.permutation(len(frames))]
    a, o, l = arena(frames)
    p = DfPair(eng, max_batch=1 << 16)
    try:
        p.batch(a, o[:64], l[:64], NOW)   # (warm-up: module load, first-touch)
        t0 = time.perf_counter()
        p.g.run_torch(*(torch.from_numpy(x).to(DEV) for x in (a, o[64:].view(np.int64), l[64:].view(np.int32))),
                      p.g.alloc_out(len(l) - 64, 128), NOW + 1)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        assert dt < 1.0, f"defrag batch with a 24k-member group took {dt:.2f} s"
    finally:
        p.close()
    p = DfPair(eng, max_batch=1 << 16)
    try:
        p.batch(a, o, l, NOW)
        p.check_stats()
    finally:
        p.close()


def test_show_text_after_reassembly(eng):
    """`show packet statistic` / `show flow statistic` after defrag batches: the ip_frag_stat
    lines, new / del fcb and (monitor on) teardrop formatted from the GPU table's ppe_defrag_info equal the text
    formatted from the oracle's sequential Defrag counters for the same stream."""
    import ctypes as C
    a, o, l = synth.make_fragment_stream(3000, seed=21)
    p = DfPair(eng, fcb_max=1 << 12)
    try:
        for k, b in enumerate(range(0, len(l), 4096)):
            p.batch(a, o[b:b + 4096], l[b:b + 4096], NOW + k)
        p.age(NOW + 10**6)
        gi = abi.DefragInfo()
        assert eng.lib.ppe_defrag_info(p.g.h, C.byref(gi)) == 0
        os_ = p.o.stats()
        oi = abi.DefragInfo()
        for k, name in enumerate(abi.DF_NAME[i] for i in range(9)):
            oi.st[k] = os_["st_" + name.lower()]
        oi.teardrop, oi.new_fcb, oi.del_fcb = os_["teardrop"], os_["new_fcb"], os_["del_fcb"]
        assert oi.st[abi.DF["REASM"]] > 0 and oi.new_fcb > 0
        cnt = abi.Counters()
        fi = abi.FlowInfo()
        texts = []
        for info in (gi, oi):
            buf = C.create_string_buffer(8192)
            eng.lib.ppe_format_pkt_stat_ex(C.byref(cnt), C.byref(info), 1, buf, 8192)
            fbuf = C.create_string_buffer(512)
            eng.lib.ppe_format_flow_stat_ex(C.byref(fi), C.byref(info), fbuf, 512)
            texts.append((buf.value.decode(), fbuf.value.decode()))
        assert texts[0] == texts[1]
        assert f"reasm_ok: {oi.st[abi.DF['REASM']]}\n" in texts[0][0]
        assert f"new fcb is: {oi.new_fcb}\n" in texts[0][1]
    finally:
        p.close()


def test_failed_admission_lookback_is_reported(eng, monkeypatch):
    """A workgroup whose admission look-back fails (forced by the PPE_DF_LOOK_FAIL test hook) admits none of its
    creators and sets a pinned error word: the NEXT ppe_defrag call fails with PPE_EIO (once), ppe_defrag_info
    too, and the table keeps working afterwards (the failure must not stay silent).  The records its
    creators' ranks skipped go back onto the free stack: after aging everything out the running count is
    0 with new_fcb == del_fcb, and a batch with more new datagrams than fcb_max then matches a fresh oracle exactly
    (FCB_FULL at the same fragments: no record lost, none used twice)."""
    from ppe.engine import PPEError
    fcb_max = 1 << 12
    monkeypatch.setenv("PPE_DF_LOOK_FAIL", "3")
    p = DfPair(eng, fcb_max=fcb_max)
    monkeypatch.delenv("PPE_DF_LOOK_FAIL")
    g = p.g
    try:
        a, off, lens = synth.make_fragment_stream(4000, seed=4242)
        n = min(len(lens), 8192)   # >= 4 admission workgroups of 256 fragments
        off1, lens1 = off[:n].copy(), lens[:n].copy()
        out = g.alloc_out(n, 128)
        ta = torch.from_numpy(a).to(DEV)
        to = torch.from_numpy(off1.view(np.int64)).to(DEV)
        tl = torch.from_numpy(lens1.view(np.int32)).to(DEV)
        g.run_torch(ta, to, tl, out, NOW)   # (asynchronous: the failure is on the device)
        torch.cuda.synchronize()
        with pytest.raises(PPEError, match="look-back"):
            g.run_torch(ta, to, tl, out, NOW + 1)
        with pytest.raises(PPEError):
            g.info()   # the device counter of failed look-backs (then cleared)
        info = g.info()
        assert 0 < info["running"] <= fcb_max and info["new_fcb"] - info["del_fcb"] == info["running"]
        g.age(NOW + 10**6, 20)
        info = g.info()
        assert info["running"] == 0 and info["new_fcb"] == info["del_fcb"]
        # the whole free stack is back: a fresh oracle sees the same FCB_FULL boundary
        a2, off2, lens2 = synth.make_fragment_stream(9000, seed=4343)
        n2 = min(len(lens2), 20000)
        got, ref = p.batch(a2, off2[:n2], lens2[:n2], NOW + 2 * 10**6)
        assert ((ref["status"] & 0xFF) == abi.DF["FCB_FULL"]).any()
    finally:
        p.close()
