"""Decode() fills exactly the mbuf fields the reference's decoders write, on exactly the packets where they write
them, with the reference's values: ethh / MACs (decode-ethernet.c:57,71-72), vlanh / vlan_idx
(decode-vlan.c:41,46), network_header (decode-ipv4.c:42, after the version check), sip / dip / proto (:62-63,97),
a fragment's defrag_id / frag_offset / frag_len (:106-109, what Defrag keys and orders on), transport_header
(decode-udp.c:24, decode-tcp.c:146), sport / dport / payload / payload_len (decode-udp.c:38-45,
decode-tcp.c:179-187), tcpvars.ws (decode-tcp.c:61-70, options read to the end of the TCP header) and the flow
flags (flow.c:294-307).  Every other field keeps the value it had.

The oracle record (tests/test_oracle_mbuf.py) is computed on the WHOLE frame, i.e. what the reference reads; the GPU
path is Decode()'s 144-B header window.  Fields the reference does not write are checked unchanged against a fill
pattern.  The punted fragments then go through ppe_defrag, and the datagrams it builds group exactly the fragments
whose mbufs carry the same Defrag key (sip, dip, defrag_id; decode-defrag.c:108-111)."""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

import torch  # noqa: E402

import pyoracle  # noqa: E402
from mbuf_corpus import corpus, windows  # noqa: E402
from ppe import Defrag, Engine, abi, synth  # noqa: E402
from ppe.abi import ST  # noqa: E402
from pyoracle import M_ETH, M_FLOW, M_FRAG, M_IP, M_L3, M_L4, M_L4H, M_VLAN, M_WS  # noqa: E402

DEV = torch.device("cuda:0")
HOOK = C.CFUNCTYPE(None, C.POINTER(abi.Mbuf))
PAT8, PAT16, PAT32, PAT64 = 0xA5, 0xA5A5, 0xA5A5A5A5, 0xA5A5A5A5A5A5A5A5
PKT_TO_SERVER, PKT_HAS_FLOW = 1 << 4, 1 << 8


def new_mbufs(frames, bufs):
    """mbufs as oct_rx_process_work hands them over (pkt_ptr, pkt_totallen; vlan_idx 0, tcpvars.ws NULL, flags 0,
    which the decoders read), every other byte a fill pattern so an unwritten field is recognisable."""
    n = len(frames)
    mb = (abi.Mbuf * n)()
    C.memset(C.addressof(mb), PAT8, C.sizeof(mb))
    for i in range(n):
        mb[i].pkt_ptr = C.cast(bufs[i], C.c_void_p).value
        mb[i].pkt_totallen = len(frames[i])
        mb[i].vlan_idx = 0
        mb[i].tcpvars.ws = None
        mb[i].flags = 0
        mb[i].timestamp = 0
    return mb


def run_decode(lib, mb, n, burst=1000):
    """Decode + Decode_Flush; returns the indices each hook received, in delivery order."""
    base, sz = C.addressof(mb), C.sizeof(abi.Mbuf)
    got = {"fw": [], "drop": [], "punt": []}
    hooks = tuple(HOOK(lambda m, k=k: got[k].append((C.addressof(m.contents) - base) // sz))
                  for k in ("fw", "drop", "punt"))
    lib.ppe_set_output_hooks.argtypes = [HOOK, HOOK, HOOK]
    lib.ppe_set_output_hooks(*hooks)
    lib.Decode_Set_Burst(burst)
    for i in range(n):
        lib.Decode(C.byref(mb[i]))
    assert lib.Decode_Flush() >= 0
    lib.ppe_set_output_hooks(HOOK(), HOOK(), HOOK())
    return got


def check_mbuf(m, r, frame, base):
    """Every mbuf field against the oracle record r of the whole frame."""
    ms = r["mset"]
    ptr = lambda v: 0 if v is None else v  # noqa: E731
    if ms & M_ETH:
        assert ptr(m.ethh) == base and bytes(m.eth_dst) == frame[:6] and bytes(m.eth_src) == frame[6:12]
    else:
        assert m.ethh == PAT64 and bytes(m.eth_dst) == bytes([PAT8]) * 6 and bytes(m.eth_src) == bytes([PAT8]) * 6
    if ms & M_VLAN:
        assert (ptr(m.vlanh), m.vlan_idx) == (base + 14, 1)
    else:
        assert (m.vlanh, m.vlan_idx) == (PAT64, 0)
    assert m.network_header == (base + r["l3off"] if ms & M_L3 else PAT64)
    if ms & M_IP:
        assert (m.sip, m.dip, m.proto) == (r["sip"], r["dip"], r["proto"])
    else:
        assert (m.sip, m.dip, m.proto) == (PAT32, PAT32, PAT8)
    if ms & M_FRAG:
        assert (m.defrag_id, m.frag_offset, m.frag_len) == (r["frag_id"], r["frag_off"], r["frag_len"])
    else:
        assert (m.defrag_id, m.frag_offset, m.frag_len) == (PAT16, PAT16, PAT16)
    assert m.transport_header == (base + r["l4off"] if ms & M_L4H else PAT64)
    if ms & M_L4:
        assert (m.sport, m.dport, m.payload_len) == (r["sport"], r["dport"], r["paylen"])
        assert m.payload == base + r["payoff"]
    else:
        assert (m.sport, m.dport, m.payload_len, m.payload) == (PAT16, PAT16, PAT16, PAT64)
    if ms & M_WS:
        assert m.tcpvars.ws == C.addressof(m) + abi.Mbuf.tcpvars.offset  # &m->TCP_OPTS[0]
        o0 = m.tcpvars.tcp_opts[0]
        w = r["l4off"] + r["tcp_ws"]
        assert (o0.type, o0.len, o0.data) == (frame[w], frame[w + 1], base + w + 2) == (3, 3, base + w + 2)
    else:
        assert not m.tcpvars.ws
        assert (m.tcpvars.tcp_opts[0].type, m.tcpvars.tcp_opts[0].data) == (PAT8, PAT64)
    assert m.flags == ((PKT_TO_SERVER | PKT_HAS_FLOW) if ms & M_FLOW else 0)
    # untouched by every decoder
    assert (m.vlan_id, m.input_port, m.flow, m.fcb, m.tag) == (PAT16, PAT32, PAT64, PAT64, PAT32)


RULES = synth.make_rules(300, seed=44)
DEFAULT_FW = 0  # ACL_RULE_ACTION_FW: packets no rule drops create their flow (PKT_HAS_FLOW), rule DROPs do not


@pytest.fixture(scope="module")
def lib():
    """The compat layer's context with RULES committed through the rule store and a default action of FW."""
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    lb = abi.load()
    assert lb.DP_Acl_Rule_Init() == 0
    lb.ppe_rule_list_free()
    assert lb.ppe_rule_list_init() == 0
    for i in range(len(RULES)):
        rid = C.c_uint32()
        assert lb.Rule_add(RULES[i:i + 1].ctypes.data, C.byref(rid)) == 0
    dflt = C.c_uint32.in_dll(lb, "dp_acl_action_default")
    old = dflt.value
    dflt.value = DEFAULT_FW
    assert lb.DP_Acl_Rule_Commit() == 0
    yield lb
    dflt.value = old
    lb.ppe_rule_list_free()


def test_decode_fills_reference_mbuf_fields(lib):
    frames, kinds = corpus(6000, seed=41)
    n = len(frames)
    bufs = [C.create_string_buffer(f, max(len(f), 1)) for f in frames]
    mb = new_mbufs(frames, bufs)
    got = run_decode(lib, mb, n)
    assert sorted(got["fw"] + got["drop"] + got["punt"]) == list(range(n))
    o = pyoracle.Oracle(RULES, default_action=DEFAULT_FW)
    cfg = o.cfg(0, 1, 0)
    seen = 0
    for i in range(n):
        f = frames[i]
        buf = np.frombuffer(f, np.uint8).copy() if f else np.zeros(1, np.uint8)
        r = pyoracle.OResult()
        o.lib.oracle_classify(buf.ctypes.data, len(f), len(f), 0, C.byref(cfg), C.byref(r))
        r = {k: getattr(r, k) for k, _ in pyoracle.OResult._fields_}
        assert mb[i].ppe_verdict & 0xFF == r["status"], (i, kinds[i])
        try:
            check_mbuf(mb[i], r, f, C.cast(bufs[i], C.c_void_p).value)
        except AssertionError as e:
            raise AssertionError(f"packet {i} ({kinds[i]}, status {r['status']}, mset {r['mset']:#x})") from e
        seen |= r["mset"]
    assert seen == M_ETH | M_VLAN | M_L3 | M_IP | M_FRAG | M_L4H | M_L4 | M_WS | M_FLOW
    ws = [i for i in range(n) if kinds[i] == "tcp_linux_syn" and mb[i].tcpvars.ws]
    assert len(ws) > 300  # the Linux SYN's option at frame byte 71+ (VLAN / IPv4 options push it further)


def test_classify_tuple_vs_oracle_at_every_window(lib):
    """The batch API's tuple (ABI 5) against the oracle on the same window: 64 / 128 B windows report
    PPE_TUPLE_OPT_PAST where the option parse ran out of window; 144 B windows equal the whole-frame answer."""
    frames, kinds = corpus(20000, seed=43)
    rules = synth.make_rules(256, seed=5)
    o = pyoracle.Oracle(rules, default_action=1)
    full_hdr, full_len = windows(frames, 256)
    full = o.classify_batch(full_hdr, full_len, cfg=o.cfg(0, 1, 0), nthreads=8)
    eng = Engine(0)
    try:
        eng.commit(rules, default_action=1)
        for stride in (64, 128, 144, 256):
            hdr, lens = windows(frames, stride)
            n = len(lens)
            out = {k: torch.full((n,), -7, dtype=torch.int32, device=DEV) for k in ("verdict", "flow_hash", "acl_hit")}
            out["tuple"] = torch.full((n, 4), -7, dtype=torch.int32, device=DEV)
            eng.classify_torch(torch.from_numpy(hdr).to(DEV), torch.from_numpy(lens.view(np.int32)).to(DEV), out,
                               cfg=eng.cfg(now_seconds=0))
            torch.cuda.synchronize()
            got = {k: v.cpu().numpy().view(np.uint32 if k != "acl_hit" else np.int32) for k, v in out.items()}
            ref = o.classify_batch(hdr, lens, cfg=o.cfg(0, 1, 0), nthreads=8)
            ok = ref["reach"] <= stride  # the rest PUNT for their window (checked in test_gpu_tcpopt.py)
            for k in ("verdict", "flow_hash", "acl_hit", "tuple"):
                assert np.array_equal(got[k][ok], ref[k][ok]), (stride, k)
            past = (got["tuple"][:, 3] & abi.TUPLE_OPT_PAST) != 0
            if stride >= 144:
                assert ok.all() and not past.any()
                for k in ("verdict", "flow_hash", "acl_hit", "tuple"):
                    assert np.array_equal(got[k], full[k]), (stride, k)
            else:
                assert past.sum() > (50 if stride == 64 else 0), stride  # 128 B: only behind VLAN + IPv4 + TCP options
                # where the option did not need the missing bytes the answer is the whole frame's
                same = ok & ~past
                assert np.array_equal(got["tuple"][same], full["tuple"][same]), stride
            fr = ok & (((got["verdict"] & 0xFF) == ST["FRAG"]) | ((got["verdict"] & 0xFF) == ST["FRAG_LEN_ERR"]))
            assert fr.sum() > 1000
    finally:
        eng.close()


def test_punted_fragments_through_defrag(lib):
    """Fragments Decode() PUNTs carry the fields Defrag keys and orders on; ppe_defrag of the punted frames equals
    the oracle's Defrag, and each datagram's fragments share one (sip, dip, defrag_id) key in the mbufs, in
    ascending frag_offset order along the chain."""
    pkt, off, lens = synth.make_fragment_stream(600, seed=9)
    n = len(lens)
    arena = C.create_string_buffer(pkt.tobytes(), len(pkt))
    base = C.addressof(arena)
    frames = [pkt[int(off[i]):int(off[i]) + int(lens[i])].tobytes() for i in range(n)]
    mb = (abi.Mbuf * n)()
    C.memset(C.addressof(mb), PAT8, C.sizeof(mb))
    for i in range(n):
        mb[i].pkt_ptr = base + int(off[i])
        mb[i].pkt_totallen = int(lens[i])
        mb[i].vlan_idx, mb[i].tcpvars.ws, mb[i].flags = 0, None, 0
    got = run_decode(lib, mb, n, burst=n)
    punt = got["punt"]
    assert len(punt) > 0.9 * n and punt == sorted(punt)
    o = pyoracle.Oracle(RULES, default_action=DEFAULT_FW)
    cfg = o.cfg(0, 1, 0)
    for i in punt:
        f = frames[i]
        buf = np.frombuffer(f, np.uint8).copy()
        r = pyoracle.OResult()
        o.lib.oracle_classify(buf.ctypes.data, len(f), len(f), 0, C.byref(cfg), C.byref(r))
        assert r.status == ST["FRAG"] and r.mset & M_FRAG
        assert (mb[i].defrag_id, mb[i].frag_offset, mb[i].frag_len) == (r.frag_id, r.frag_off, r.frag_len)
        assert (mb[i].sip, mb[i].dip, mb[i].network_header) == (r.sip, r.dip, base + int(off[i]) + r.l3off)
    # the punted frames, in delivery order, through the GPU's Defrag and the oracle's
    poff = off[punt]
    plen = lens[punt]
    ids = np.array(punt, np.uint64)
    eng = Engine(0)
    try:
        d = Defrag(eng)
        od = pyoracle.OracleDefrag()
        ref = od.batch(pkt, poff, plen, 100, ids=ids)
        out = d.alloc_out(len(punt), 128)
        d.run_torch(torch.from_numpy(pkt).to(DEV), torch.from_numpy(poff.view(np.int64)).to(DEV),
                    torch.from_numpy(plen.view(np.int32)).to(DEV), out, 100,
                    ids=torch.from_numpy(ids.view(np.int64)).to(DEV))
        torch.cuda.synchronize()
        st = out["status"].cpu().numpy().view(np.uint32)
        assert np.array_equal(st, ref["status"])
        nd = int(out["n_dgram"].cpu()[0])
        assert nd == ref["n_dgram"] > 50
        fr = out["dgram_frags"].cpu().numpy().view(np.uint64)[:nd]
        assert np.array_equal(fr, ref["dgram_frags"][:nd])
        for j in range(nd):
            chain = [int(x) for x in fr[j] if x != np.uint64(2**64 - 1)]
            keys = {(mb[i].sip, mb[i].dip, mb[i].defrag_id) for i in chain}
            assert len(keys) == 1, j
            offs = [mb[i].frag_offset for i in chain]
            assert offs == sorted(offs), j
        d.close()
        od.close()
    finally:
        eng.close()
