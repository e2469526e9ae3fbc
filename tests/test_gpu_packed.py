"""The packed result layout (ppe_result_t.packed, ABI 8): one 8-B word per packet with the flow hash, status, action,
flags and ACL hit + 1 (include/ppe_hip.h PPE_PACKED_*), the layout bench.py's throughput line writes (with part8:
9 B written per packet instead of 13).

Bar: every field decodes bit-exact to the three SoA words of the same launch and to the oracle (verdict, flow hash,
ACL hit; reference semantics: decode.c:19-28 → flow.c:204-237), over the exact bench workloads and the edges of the
layout (rule indices past 65,535 through the cut lists' 32-bit ids, the 2^19 - 1 rule-slot limit, argument errors)."""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

import torch  # noqa: E402

import pyoracle  # noqa: E402
from ppe import Engine, abi, synth  # noqa: E402
from test_gpu_parity import check_part8, part8_expected  # noqa: E402

DEV = torch.device("cuda:0")
NOW = 1_700_000_000
SAMPLE = {"C1": 1 << 16, "C2": 1 << 16, "C3": 1 << 14, "C4": 1 << 16}


@pytest.fixture(scope="module")
def eng():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    e = Engine(0)
    yield e
    e.close()


def packed_result(n, soa=False):
    o = {"packed": torch.full((n,), -7, dtype=torch.int64, device=DEV),
         "part8": torch.full((n,), 0xEE, dtype=torch.uint8, device=DEV)}
    if soa:
        o = {k: torch.full((n,), -7, dtype=torch.int32, device=DEV) for k in ("verdict", "flow_hash", "acl_hit")}
        o["part8"] = torch.full((n,), 0xEE, dtype=torch.uint8, device=DEV)
    r = abi.Result(*(o[k].data_ptr() if k in o else None
                     for k in ("verdict", "flow_hash", "acl_hit", "fw_idx", "drop_idx", "tile_cnt", "tuple", "part8",
                               "packed")))
    return o, r


@pytest.mark.parametrize("cfgname", ["C1", "C2", "C3", "C4"])
def test_packed_exact_workload(eng, cfgname):
    """bench.py's exact workload of each config (the two generated 1M-packet batches, 64-B windows) through
    ppe_classify_batches with 34 descriptors (the device descriptor ring): descriptors 0 / 1 write the SoA words,
    the rest the packed words + part8.  Over the WHOLE batch every packed field equals the SoA word of the same
    packet and every packed descriptor of a batch is bit-identical; the first SAMPLE packets plus a strided sample
    equal the oracle's linear first-match definition."""
    c = synth.CONFIGS[cfgname]
    n = c["n"]
    rules = synth.make_rules(c["rules"])
    eng.commit(rules, default_action=1)
    eng.tuning(batches_per_launch=0)
    host = [synth.make_packets(n, rules, seed=synth.SEED + 1 + 7919 * g, kind=c["kind"], stride=64) for g in range(2)]
    dev_in = [(torch.from_numpy(pk["hdr"]).to(DEV), torch.from_numpy(pk["len"].view(np.int32)).to(DEV)) for pk in host]
    ndesc = 34
    outs, bats, ress = [], [], []
    for d in range(ndesc):
        th, tl = dev_in[d % 2]
        o, r = packed_result(n, soa=d < 2)
        outs.append(o)
        bats.append(abi.Batch(th.data_ptr(), tl.data_ptr(), None, n, 64))
        ress.append(r)
    ins, rs = (abi.Batch * ndesc)(*bats), (abi.Result * ndesc)(*ress)
    cfg = eng.cfg(now_seconds=NOW)
    s = torch.cuda.current_stream(DEV)
    eng.clear_counters()
    assert eng.lib.ppe_classify_batches(eng.ctx, ins, rs, ndesc, C.byref(cfg), C.c_void_p(s.cuda_stream)) == 0
    torch.cuda.synchronize()
    assert eng.counters()["pkts"] == ndesc * n
    o = pyoracle.Oracle(rules, default_action=1)
    m = SAMPLE[cfgname]
    for g, pk in enumerate(host):
        soa = {k: outs[g][k].cpu().numpy() for k in ("verdict", "flow_hash", "acl_hit")}
        soa["verdict"], soa["flow_hash"] = soa["verdict"].view(np.uint32), soa["flow_hash"].view(np.uint32)
        for d in range(g + 2, ndesc, 2):
            assert torch.equal(outs[d]["packed"], outs[g + 2]["packed"]), (cfgname, d)
            assert torch.equal(outs[d]["part8"], outs[g]["part8"]), (cfgname, d)
        got = abi.unpack(outs[g + 2]["packed"].cpu().numpy())
        for k in ("verdict", "flow_hash", "acl_hit"):
            assert np.array_equal(got[k], soa[k]), (cfgname, g, k, np.nonzero(got[k] != soa[k])[0][:5])
        assert ((soa["verdict"] >> 16) < 64).all()   # the stateless path's flags fit the packed field
        assert np.array_equal(outs[g + 2]["part8"].cpu().numpy(), part8_expected(got["verdict"], n))
        idx = np.concatenate([np.arange(m), np.arange(m, n, max(1, (n - m) // m))])
        ref = o.classify_batch(pk["hdr"][idx], pk["len"][idx], cfg=o.cfg(0, 1, NOW), nthreads=16)
        far = ref["reach"] > 64
        for k in ("verdict", "flow_hash", "acl_hit"):
            gk = got[k][idx]
            assert np.array_equal(gk[~far], ref[k][~far]), (cfgname, g, k)
        assert (got["acl_hit"][idx] >= 0).sum() > len(idx) // 8


def test_packed_imix_malformed_and_ragged(eng):
    """Every status and flag combination the generator makes (IMIX, VLAN, TCP options, 5 % malformed, 128-B
    windows, ragged sizes) in the packed form equals the oracle, with and without part8."""
    rules = synth.make_rules(512, seed=71)
    eng.commit(rules, default_action=1)
    o = pyoracle.Oracle(rules, default_action=1)
    for n in (1, 63, 64, 65, 1000, 100_003):
        pk = synth.make_packets(n, rules, seed=72 + n, kind="imix", stride=128, malformed_frac=0.05)
        th, tl = torch.from_numpy(pk["hdr"]).to(DEV), torch.from_numpy(pk["len"].view(np.int32)).to(DEV)
        for with_part8 in (True, False):
            out = {"packed": torch.full((n,), -7, dtype=torch.int64, device=DEV)}
            if with_part8:
                out["part8"] = torch.full((n + 64,), 0xEE, dtype=torch.uint8, device=DEV)
            eng.classify_torch(th, tl, out, cfg=eng.cfg(now_seconds=NOW))
            torch.cuda.synchronize()
            got = abi.unpack(out["packed"].cpu().numpy())
            ref = o.classify_batch(pk["hdr"], pk["len"], cfg=o.cfg(0, 1, NOW), nthreads=16)
            for k in ("verdict", "flow_hash", "acl_hit"):
                assert np.array_equal(got[k], ref[k]), (n, k)
            if with_part8:
                check_part8({"verdict": got["verdict"], "part8": out["part8"].cpu().numpy()}, n)
    assert len(np.unique(ref["verdict"] & 0xFF)) >= 10


@pytest.mark.parametrize("cut_lines", ["0", "1"])
def test_packed_rule_ids_past_16_bits(eng, monkeypatch, cut_lines):
    """a classifier whose used rule indices reach past 65,535 (a sparse `used` array over 400,000 slots)
    takes the cut lists' 32-bit id layout; matches on those rules equal the oracle's linear definition, in the SoA
    and in the packed words (acl_hit + 1 needs 19 bits here), with the cut-list lines on and off."""
    monkeypatch.setenv("PPE_CUT_LINES", cut_lines)
    e = Engine(0)
    try:
        base = synth.make_rules(4096, seed=73)
        slots = 400_000
        rules = np.zeros(slots, abi.RULE_DTYPE)
        used = np.zeros(slots, np.uint8)
        pos = np.sort(np.random.default_rng(74).choice(np.arange(1, slots), len(base), replace=False))
        pos[-3:] = [65_536, 131_071, slots - 1]
        pos = np.unique(pos)
        rules[pos] = base[:len(pos)]
        used[pos] = 1
        st = e.commit(rules, used, default_action=1)
        o = pyoracle.Oracle(rules, used=used, default_action=1)
        pk = synth.make_packets(200_000, base[:len(pos)], seed=75, kind="udp64", stride=64, hit_frac=0.9)
        th, tl = torch.from_numpy(pk["hdr"]).to(DEV), torch.from_numpy(pk["len"].view(np.int32)).to(DEV)
        n = len(pk["len"])
        out = {"packed": torch.empty(n, dtype=torch.int64, device=DEV)}
        soa = {k: torch.empty(n, dtype=torch.int32, device=DEV) for k in ("verdict", "flow_hash", "acl_hit")}
        e.classify_torch(th, tl, out, cfg=e.cfg(now_seconds=NOW))
        e.classify_torch(th, tl, soa, cfg=e.cfg(now_seconds=NOW))
        torch.cuda.synchronize()
        got = abi.unpack(out["packed"].cpu().numpy())
        ref = o.classify_batch(pk["hdr"], pk["len"], cfg=o.cfg(0, 1, NOW), nthreads=16)
        assert np.array_equal(soa["acl_hit"].cpu().numpy(), ref["acl_hit"])
        for k in ("verdict", "flow_hash", "acl_hit"):
            assert np.array_equal(got[k], ref[k]), k
        assert (ref["acl_hit"] > 65_535).sum() > 100, "the sample must hit rules past 16-bit ids"
        assert st["n_rules"] == len(pos)
    finally:
        e.close()


def test_packed_argument_errors(eng):
    """packed replaces verdict / flow hash / ACL hit (both given: EINVAL); not in the flow-table path; refused for
    classifiers of more than PPE_PACKED_MAX_RULES rule slots (their indices would not fit)."""
    rules = synth.make_rules(16, seed=76)
    eng.commit(rules, default_action=1)
    n = 256
    th = torch.zeros((n, 64), dtype=torch.uint8, device=DEV)
    tl = torch.full((n,), 64, dtype=torch.int32, device=DEV)
    pkd = torch.empty(n, dtype=torch.int64, device=DEV)
    v = torch.empty(n, dtype=torch.int32, device=DEV)
    b = abi.Batch(th.data_ptr(), tl.data_ptr(), None, n, 64)
    cfg = eng.cfg()
    r = abi.Result(v.data_ptr(), None, None, None, None, None, None, None, pkd.data_ptr())
    assert eng.lib.ppe_classify(eng.ctx, C.byref(b), C.byref(r), C.byref(cfg), None) == -22
    r = abi.Result(None, None, None, None, None, None, None, None, pkd.data_ptr())
    assert eng.lib.ppe_classify(eng.ctx, C.byref(b), C.byref(r), C.byref(cfg), None) == 0
    eng.flow_create(1000, n)
    try:
        rf = abi.Result(v.data_ptr(), None, None, None, None, None, None, None, pkd.data_ptr())
        assert eng.lib.ppe_classify_flow(eng.ctx, C.byref(b), C.byref(rf), C.byref(cfg), None) == -22
    finally:
        eng.flow_destroy()
    big = np.zeros(abi.PACKED_MAX_RULES + 1, abi.RULE_DTYPE)
    used = np.zeros(len(big), np.uint8)
    big[:16] = rules
    used[:16] = 1
    eng.commit(big, used, default_action=1)
    assert eng.lib.ppe_classify(eng.ctx, C.byref(b), C.byref(r), C.byref(cfg), None) == -22
    assert b"rule slots" in eng.lib.ppe_last_error(eng.ctx)
    rs = abi.Result(v.data_ptr(), None, None, None, None, None, None, None, None)
    assert eng.lib.ppe_classify(eng.ctx, C.byref(b), C.byref(rs), C.byref(cfg), None) == 0   # the SoA form still runs
    torch.cuda.synchronize()
    eng.commit(rules, default_action=1)


@pytest.mark.parametrize("zerocopy", ["1", "0"])
def test_packed_host_buffers(eng, monkeypatch, zerocopy):
    """ppe_classify_host with the packed words in pinned host memory: zero-copy and the staged H2D / D2H path."""
    monkeypatch.setenv("PPE_HOST_ZEROCOPY", zerocopy)
    rules = synth.make_rules(256, seed=77)
    pk = synth.make_packets(70_001, rules, seed=78, kind="imix", stride=128, malformed_frac=0.02)
    eng.commit(rules, default_action=1)
    n = len(pk["len"])
    ph = torch.from_numpy(pk["hdr"]).pin_memory()
    pl = torch.from_numpy(pk["len"].view(np.int32)).pin_memory()
    pp = torch.full((n,), -7, dtype=torch.int64).pin_memory()
    p8 = torch.full((n,), 0xEE, dtype=torch.uint8).pin_memory()
    b = abi.Batch(ph.data_ptr(), pl.data_ptr(), None, n, 128)
    r = abi.Result(None, None, None, None, None, None, None, p8.data_ptr(), pp.data_ptr())
    cfg = eng.cfg(now_seconds=NOW)
    assert eng.lib.ppe_classify_host(eng.ctx, C.byref(b), C.byref(r), C.byref(cfg), 1 << 14) == 0
    o = pyoracle.Oracle(rules, default_action=1)
    ref = o.classify_batch(pk["hdr"], pk["len"], cfg=o.cfg(0, 1, NOW), nthreads=16)
    got = abi.unpack(pp.numpy())
    for k in ("verdict", "flow_hash", "acl_hit"):
        assert np.array_equal(got[k], ref[k]), k
    check_part8({"verdict": got["verdict"], "part8": p8.numpy()}, n)
