"""Known answers for the oracle's record of the mbuf fields the reference's decoders write (oracle_result_t.mset and
the offsets / Defrag fields beside it), and for the window-bounded TCP option parse (opt_past).  Each expectation is
derived by hand from the cited reference lines; tests/test_gpu_mbuf.py then holds Decode() to this record."""
import numpy as np
import pytest

import pyoracle
from mbuf_corpus import LINUX_SYN_OPTS, corpus, windows
from pktbuild import eth, ip_frag, ipv4, tcp, udp, vlan
from pyoracle import M_ETH, M_FLOW, M_FRAG, M_IP, M_L3, M_L4, M_L4H, M_VLAN, M_WS
from ppe.abi import ST

CFG = pyoracle.Oracle.cfg(0, 1, 0)


@pytest.fixture(scope="module")
def o():
    return pyoracle.Oracle(None, default_action=0)  # no rules, default FW: ACL-passing packets create their flow


def one(o, f, avail=None, cfg=CFG):
    import ctypes as C
    buf = np.frombuffer(bytes(f), np.uint8).copy() if f else np.zeros(1, np.uint8)
    r = pyoracle.OResult()
    o.lib.oracle_classify(buf.ctypes.data, len(f) if avail is None else min(avail, len(f)), len(f), 0,
                          C.byref(cfg), C.byref(r))
    return {k: getattr(r, k) for k, _ in pyoracle.OResult._fields_}


def test_linux_syn_window_scale_at_byte_71(o):
    l4 = tcp(40000, 443, 0x02, off=10, opts=LINUX_SYN_OPTS)
    f = eth(0x0800) + ipv4(6, 0x0A000001, 0x0A000002, len(l4)) + l4
    r = one(o, f)
    assert r["status"] == ST["ACL_FW"]
    assert r["mset"] == M_ETH | M_L3 | M_IP | M_L4H | M_L4 | M_WS | M_FLOW
    assert (r["l3off"], r["l4off"], r["payoff"]) == (14, 34, 74)  # decode-ipv4.c:42, decode-tcp.c:146, :186
    assert r["tcp_ws"] == 37 and 14 + 20 + 37 == 71 and r["opt_past"] == 0  # decode-tcp.c:63-70
    # a 64-B header window ends inside the options before the window-scale option: the answer needs more bytes
    r64 = one(o, f, avail=64)
    assert (r64["tcp_ws"], r64["opt_past"]) == (0, 1)
    assert r64["status"] == r["status"] and r64["mset"] == r["mset"] & ~M_WS


def test_option_past_128_behind_vlan_and_ip_options(o):
    opts = b"\x01" * 37 + b"\x03\x03\x09"  # 40 option bytes, the window-scale option last (TCP bytes 57-59)
    l4 = tcp(1, 2, 0x02, off=15, opts=opts)
    f = eth(0x8100) + vlan(0x0800) + ipv4(6, 1, 2, len(l4), ihl=15) + l4
    r = one(o, f)
    assert r["mset"] & M_VLAN and (r["l3off"], r["l4off"]) == (18, 78) and r["tcp_ws"] == 57
    assert 78 + 57 == 135  # past a 128-B window
    r128 = one(o, f, avail=128)
    assert (r128["tcp_ws"], r128["opt_past"]) == (0, 1)
    r144 = one(o, f, avail=144)
    assert (r144["tcp_ws"], r144["opt_past"]) == (57, 0)
    # a window-scale option found before the edge is final (the first valid one counts): no opt_past
    opts2 = b"\x03\x03\x02" + b"\x01" * 37
    l4 = tcp(1, 2, 0x02, off=15, opts=opts2)
    f2 = eth(0x8100) + vlan(0x0800) + ipv4(6, 1, 2, len(l4), ihl=15) + l4
    r2 = one(o, f2, avail=100)
    assert (r2["tcp_ws"], r2["opt_past"]) == (20, 0)


def test_fragment_fields(o):
    # decode-ipv4.c:106-109: defrag_id = ip_id, frag_offset = (ip_off & 0x1fff) << 3, frag_len = len - ihl (len is
    # the buffer past L2, padding included)
    f = ip_frag(17, 0x0A000001, 0x0A000002, 0xBEEF, 1480, True, bytes(64), ihl=6, vlan_tag=True, pad=8)
    r = one(o, f)
    assert r["status"] == ST["FRAG"]
    assert r["mset"] == M_ETH | M_VLAN | M_L3 | M_IP | M_FRAG
    assert (r["frag_id"], r["frag_off"], r["frag_len"]) == (0xBEEF, 1480, 64 + 8)
    assert r["l3off"] == 18
    z = ip_frag(6, 1, 2, 7, 16, True, b"")  # no payload: FRAG_LEN_ERR, the fields are still written first
    r = one(o, z)
    assert r["status"] == ST["FRAG_LEN_ERR"] and r["mset"] & M_FRAG
    assert (r["frag_id"], r["frag_off"], r["frag_len"]) == (7, 16, 0)
    r = one(o, ip_frag(89, 1, 2, 7, 0, True, bytes(16)))  # OSPF: not a fragment for Defrag (:102)
    assert r["status"] == ST["IPV4_UNSUPPORT"] and not r["mset"] & M_FRAG


def test_which_layer_wrote_what(o):
    l4 = udp(1, 2, bytes(4))
    ok = eth(0x0800) + ipv4(17, 1, 2, len(l4)) + l4
    assert one(o, ok)["mset"] == M_ETH | M_L3 | M_IP | M_L4H | M_L4 | M_FLOW
    assert one(o, ok)["payoff"] == 14 + 20 + 8  # decode-udp.c:44
    # network_header is written after the version check, before the header-length check (decode-ipv4.c:36-44)
    bad_ihl = bytearray(ok)
    bad_ihl[14] = 0x44
    r = one(o, bytes(bad_ihl))
    assert r["status"] == ST["IPV4_HEADER_ERR"] and r["mset"] == M_ETH | M_L3
    r = one(o, eth(0x0800) + ipv4(17, 1, 2, 0)[:19])  # len < 20: before it
    assert r["status"] == ST["IPV4_HEADER_ERR"] and r["mset"] == M_ETH
    r = one(o, eth(0x0800) + ipv4(17, 1, 2, len(l4), ver=6) + l4)
    assert r["status"] == ST["IPV4_VERSION_ERR"] and r["mset"] == M_ETH
    r = one(o, eth(0x0800) + ipv4(17, 1, 2, len(l4), ip_len=200) + l4)
    assert r["status"] == ST["IPV4_LEN_ERR"] and r["mset"] == M_ETH | M_L3
    # transport_header after the first L4 length check only (decode-udp.c:18-24, decode-tcp.c:140-146)
    u = udp(1, 2, bytes(8), ulen=9)
    r = one(o, eth(0x0800) + ipv4(17, 1, 2, len(u)) + u)
    assert r["status"] == ST["UDP_LEN_ERR"] and r["mset"] == M_ETH | M_L3 | M_IP | M_L4H
    r = one(o, eth(0x0800) + ipv4(6, 1, 2, 12) + bytes(12))
    assert r["status"] == ST["TCP_HEADER_ERR"] and r["mset"] == M_ETH | M_L3 | M_IP
    t = tcp(1, 2, 0x02, off=4)
    r = one(o, eth(0x0800) + ipv4(6, 1, 2, len(t)) + t)
    assert r["status"] == ST["TCP_LEN_ERR"] and r["mset"] == M_ETH | M_L3 | M_IP | M_L4H
    # syn_check drop: ports and payload are written (decode-tcp.c:179-187), the flow is not (flow.c:204-214)
    t = tcp(1, 2, 0x10)
    r = one(o, eth(0x0800) + ipv4(6, 1, 2, len(t)) + t)
    assert r["status"] == ST["FLOW_TCP_NO_SYN_FIRST"] and r["mset"] == M_ETH | M_L3 | M_IP | M_L4H | M_L4
    # L2: zero MAC writes nothing; an unsupported type after the MACs; VLAN fields once the tag's checks pass
    assert one(o, eth(0x0800, dmac=bytes(6)) + ipv4(17, 1, 2, len(l4)) + l4)["mset"] == 0
    assert one(o, eth(0x86DD) + bytes(40))["mset"] == M_ETH
    assert one(o, eth(0x8100) + bytes(3))["mset"] == M_ETH  # VLAN len < 4
    assert one(o, eth(0x8100) + vlan(0x86DD) + bytes(20))["mset"] == M_ETH | M_VLAN
    r = one(o, eth(0x8100) + vlan(0x8100) + vlan(0x0800) + bytes(40))  # the second tag: LAYER_EXCEED
    assert r["status"] == ST["VLAN_LAYER_EXCEED"] and r["mset"] == M_ETH | M_VLAN


def test_tuple_carries_fragment_fields_and_option_bit(o):
    frames, kinds = corpus(3000, seed=3)
    for stride in (64, 128, 144):
        hdr, lens = windows(frames, stride)
        b = o.classify_batch(hdr, lens, cfg=CFG)
        for i in range(len(frames)):
            r = one(o, frames[i], avail=stride)
            t = b["tuple"][i]
            if r["mset"] & M_FRAG:
                assert t[2] == r["frag_id"] | (r["frag_off"] << 16) and t[3] >> 16 == r["frag_len"]
            assert bool(t[3] & (1 << 15)) == bool(r["opt_past"]) and (t[3] >> 9) & 63 == r["tcp_ws"]
    # with 144 bytes every option lies inside the window; at 64 some do not
    hdr, lens = windows(frames, 144)
    assert not (o.classify_batch(hdr, lens, cfg=CFG)["tuple"][:, 3] & (1 << 15)).any()
    hdr, lens = windows(frames, 64)
    assert (o.classify_batch(hdr, lens, cfg=CFG)["tuple"][:, 3] & (1 << 15)).sum() > 100
