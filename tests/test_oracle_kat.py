"""Known-answer packets, one per decode/flow/ACL reason, checked against the CPU oracle.

Each case cites the reference line whose behaviour it pins (the reference decoders cannot be compiled here without
stand-ins for the Cavium SDK headers, so these hand-derived answers are the decode pin)."""
import numpy as np
import pytest

import pyoracle
from ppe.abi import ST, RULE_DTYPE
from pktbuild import DMAC, SMAC, eth, ipv4, tcp, tcp_packet, udp, udp_packet, vlan

C = {name: i for i, name in enumerate(__import__("ppe").COUNTERS)}


def bits(*names):
    return sum(1 << C[n] for n in names)


@pytest.fixture(scope="module")
def orc():
    return pyoracle.Oracle(np.zeros(0, RULE_DTYPE), default_action=0)  # no rules, default FW


def run(orc, pkt, length=None, cfg=None):
    return orc.classify_one(pkt, length, cfg=cfg)


def test_udp_ok_and_hash_known_answer(orc):
    r = run(orc, udp_packet())
    assert r["status"] == ST["ACL_FW"] and r["action"] == 0
    assert (r["sip"], r["dip"], r["sport"], r["dport"], r["proto"]) == (0x0A000001, 0x0A000002, 1234, 80, 17)
    assert r["flow_hash"] == 0x554D7C02  # SURVEY.md §8(a) A9, tluhash.h:26-35
    assert r["paylen"] == 22  # decode-udp.c:45
    assert r["counters"] == bits("pkts", "l2_rx_ok", "ipv4_rx_ok", "udp_rx_ok", "acl_fw", "flow_proc_ok", "out_fw")


def test_hash_is_symmetric(orc):
    a = run(orc, udp_packet(sip=0x0A000001, dip=0x0A000002, sport=1234, dport=80))
    b = run(orc, udp_packet(sip=0x0A000002, dip=0x0A000001, sport=80, dport=1234))
    assert a["flow_hash"] == b["flow_hash"] == 0x554D7C02


def test_tcp_syn_ok_known_hash(orc):
    r = run(orc, tcp_packet())
    assert r["status"] == ST["ACL_FW"] and r["flow_hash"] == 0xB1B70370
    assert r["flags"] & 0x4 and r["flags"] & 0x8


def test_vlan_udp(orc):
    r = run(orc, udp_packet(vlan_tag=True))
    assert r["status"] == ST["ACL_FW"] and r["flags"] & 0x1  # decode-vlan.c:46
    assert r["counters"] & bits("vlan_rx_ok")


@pytest.mark.parametrize("length", [0, 1, 13])
def test_l2_short(orc, length):  # decode-ethernet.c:29-34
    r = run(orc, udp_packet(), length=length)
    assert r["status"] == ST["L2_HEADER_ERR"] and r["action"] == 1
    assert r["counters"] == bits("pkts", "l2_headerlen_err", "out_drop")


def test_l2_zero_macs(orc):  # decode-ethernet.c:38-54 (dst OR src all-zero)
    p = bytearray(udp_packet())
    p[0:6] = b"\0" * 6
    assert run(orc, bytes(p))["status"] == ST["L2_HEADER_ERR"]
    p = bytearray(udp_packet())
    p[6:12] = b"\0" * 6
    assert run(orc, bytes(p))["status"] == ST["L2_HEADER_ERR"]
    p = bytearray(udp_packet())
    p[0:5] = b"\0" * 5  # one non-zero byte left → fine
    assert run(orc, bytes(p))["status"] == ST["ACL_FW"]


@pytest.mark.parametrize("etype", [0x86DD, 0x0806, 0x88A8, 0x0000])
def test_l2_unsupported(orc, etype):  # decode-ethernet.c:102-111; 0x88a8 is not decoded
    p = eth(etype) + b"\0" * 50
    r = run(orc, p)
    assert r["status"] == ST["L2_UNSUPPORT"] and r["action"] == 1  # unsupport_proto_action 0 = drop
    r = run(orc, p, cfg=orc.cfg(unsupport_proto_action=1))
    assert r["action"] == 0  # decode.c:33-36


def test_vlan_errors(orc):
    assert run(orc, eth(0x8100) + b"\0\0\0")["status"] == ST["VLAN_HEADER_ERR"]  # decode-vlan.c:28-33
    r = run(orc, eth(0x8100) + vlan(0x8100) + vlan(0x0800) + b"\0" * 40)
    assert r["status"] == ST["VLAN_LAYER_EXCEED"]  # decode-vlan.c:35-39 (recursion)
    assert r["counters"] & bits("vlan_rx_ok")  # the outer tag was accepted first (:73)
    r = run(orc, eth(0x9100) + vlan(0x9100) + b"\0\0")  # second tag with < 4 bytes left
    assert r["status"] == ST["VLAN_HEADER_ERR"]
    assert run(orc, eth(0x8100) + vlan(0x0806) + b"\0" * 40)["status"] == ST["VLAN_UNSUPPORT"]


def test_ipv4_errors(orc):
    assert run(orc, eth(0x0800) + b"\x45" + b"\0" * 18)["status"] == ST["IPV4_HEADER_ERR"]  # len < 20
    p = eth(0x0800) + ipv4(17, 1, 2, 8, ver=6) + udp(1, 2)
    assert run(orc, p)["status"] == ST["IPV4_VERSION_ERR"]  # decode-ipv4.c:36-40
    p = eth(0x0800) + ipv4(17, 1, 2, 8, ihl=4)[:16] + b"\0" * 4 + udp(1, 2)
    assert run(orc, p)["status"] == ST["IPV4_HEADER_ERR"]  # ihl*4 < 20, :44-48
    p = eth(0x0800) + ipv4(17, 1, 2, 8, ip_len=19) + udp(1, 2)
    assert run(orc, p)["status"] == ST["IPV4_LEN_ERR"]  # ip_len < hlen, :50-54
    p = eth(0x0800) + ipv4(17, 1, 2, 8, ip_len=100) + udp(1, 2)
    assert run(orc, p)["status"] == ST["IPV4_LEN_ERR"]  # len < ip_len, :56-60


def test_fragments(orc):
    p = eth(0x0800) + ipv4(17, 1, 2, 8, off=0x2000) + udp(1, 2)
    r = run(orc, p)
    assert r["status"] == ST["FRAG"] and r["action"] == 2  # MF → Defrag → punt, :102-125
    p = eth(0x0800) + ipv4(17, 1, 2, 8, off=0x0003) + udp(1, 2)
    assert run(orc, p)["status"] == ST["FRAG"]
    p = eth(0x0800) + ipv4(17, 1, 2, 0, off=0x0001)
    assert run(orc, p)["status"] == ST["FRAG_LEN_ERR"]  # frag_len == 0, :109-114
    p = eth(0x0800) + ipv4(17, 1, 2, 8, off=0x4000) + udp(1, 2)  # DF only: not a fragment
    assert run(orc, p)["status"] == ST["ACL_FW"]
    p = eth(0x0800) + ipv4(89, 1, 2, 8, off=0x2000) + b"\0" * 8  # OSPF fragments are not defragmented
    assert run(orc, p)["status"] == ST["IPV4_UNSUPPORT"]


def test_ipv4_unsupported(orc):  # decode-ipv4.c:233-243 (ROUTE_PROC_ENABLE off)
    r = run(orc, eth(0x0800) + ipv4(1, 1, 2, 8) + b"\0" * 8)
    assert r["status"] == ST["IPV4_UNSUPPORT"] and r["sip"] == 1 and r["proto"] == 1


def test_udp_errors(orc):
    p = eth(0x0800) + ipv4(17, 1, 2, 7) + b"\0" * 7
    assert run(orc, p)["status"] == ST["UDP_HEADER_ERR"]  # l4len < 8, decode-udp.c:18-22
    p = eth(0x0800) + ipv4(17, 1, 2, 12) + udp(1, 2, b"\0" * 4, ulen=13)
    assert run(orc, p)["status"] == ST["UDP_LEN_ERR"]  # l4len < uh_len, :26-30
    p = eth(0x0800) + ipv4(17, 1, 2, 12) + udp(1, 2, b"\0" * 4, ulen=11)
    assert run(orc, p)["status"] == ST["UDP_LEN_ERR"]  # l4len != uh_len, :32-36
    p = eth(0x0800) + ipv4(17, 1, 2, 12) + udp(1, 2, b"\0" * 4) + b"\0" * 10  # ethernet padding is fine
    assert run(orc, p)["status"] == ST["ACL_FW"]


def test_tcp_errors(orc):
    p = eth(0x0800) + ipv4(6, 1, 2, 19) + b"\0" * 19
    assert run(orc, p)["status"] == ST["TCP_HEADER_ERR"]  # decode-tcp.c:140-144
    for off in (0, 1, 4):  # (uint8)(hlen - 20) > 40, :155-160
        p = eth(0x0800) + ipv4(6, 1, 2, 20) + tcp(1, 2, off=off)
        assert run(orc, p)["status"] == ST["TCP_LEN_ERR"], off
    p = eth(0x0800) + ipv4(6, 1, 2, 24) + tcp(1, 2, off=7) + b"\0" * 4  # hlen 28 > l4len 24, :149-153
    assert run(orc, p)["status"] == ST["TCP_LEN_ERR"]
    p = eth(0x0800) + ipv4(6, 1, 2, 60) + tcp(1, 2, off=15, opts=b"\x01" * 40)  # max options
    assert run(orc, p)["status"] == ST["ACL_FW"]


def test_tcp_options_window_scale_no_verdict_effect(orc):
    opts = b"\x01\x03\x03\x07"  # NOP + WS(7)
    p = eth(0x0800) + ipv4(6, 1, 2, 24) + tcp(1, 2, off=6, opts=opts)
    r = run(orc, p)
    # m->tcpvars.ws = the option at TCP header byte 21 (decode-tcp.c:61-70); the tuple carries it in bits 9-15
    assert r["status"] == ST["ACL_FW"] and r["tcp_ws"] == 21
    bad = b"\x03\x09\x00\x00"  # option length past the option space: DecodeTCPOptions returns -1, ignored
    r = run(orc, eth(0x0800) + ipv4(6, 1, 2, 24) + tcp(1, 2, off=6, opts=bad))
    assert r["status"] == ST["ACL_FW"] and r["tcp_ws"] == 0
    cases = [
        (b"\x02\x04\x05\xb4" + b"\x03\x03\x02" + b"\x01", 24),      # MSS, then WS at 24
        (b"\x03\x03\x01" + b"\x03\x03\x09" + b"\x00\x00", 20),      # duplicate WS: the first is kept (:63-66)
        (b"\x03\x04\x01\x01" + b"\x03\x03\x09\x00", 24),           # WS of length 4 is not recorded (:60-62)
        (b"\x03\x03\x01" + b"\x08\x0a" + b"\x00" * 3, 20),            # recorded, then an invalid length (:43-47)
        (b"\x00" + b"\x03\x03\x01" + b"\x00" * 4, 0),                  # EOL first: nothing after it is parsed
        (b"\x01" * 7 + b"\x03", 0),                                     # a kind byte with no length byte left
    ]
    for opts, want in cases:
        r = run(orc, eth(0x0800) + ipv4(6, 1, 2, 28) + tcp(1, 2, off=7, opts=opts))
        assert r["status"] == ST["ACL_FW"] and r["tcp_ws"] == want, (opts, r["tcp_ws"])


def test_syn_check(orc):  # flow.c:204-214
    r = run(orc, tcp_packet(flags=0x10))
    assert r["status"] == ST["FLOW_TCP_NO_SYN_FIRST"] and r["action"] == 1
    assert r["counters"] & bits("flow_proc_fail") and r["flags"] & 0x2
    assert run(orc, tcp_packet(flags=0x10), cfg=orc.cfg(syn_check=0))["status"] == ST["ACL_FW"]


def test_len_truncated_to_16_bits(orc):  # decode.c:22 passes (uint16_t)pkt_totallen
    p = udp_packet()
    assert run(orc, p, length=65536 + len(p))["status"] == ST["ACL_FW"]
    assert run(orc, p, length=65536 + 5)["status"] == ST["L2_HEADER_ERR"]


def test_ip_options_shift_l4(orc):
    l4 = udp(7, 9, b"\0" * 4)
    p = eth(0x0800) + ipv4(17, 5, 6, len(l4), ihl=8) + l4
    r = run(orc, p)
    assert r["status"] == ST["ACL_FW"] and (r["sport"], r["dport"]) == (7, 9)
    assert r["reach"] == 14 + 32 + 6


def rules_of(*specs):
    r = np.zeros(len(specs), RULE_DTYPE)
    for i, s in enumerate(specs):
        r[i]["sport_end"] = r[i]["dport_end"] = 65535
        r[i]["protocol_end"] = 255
        for k, v in s.items():
            r[i][k] = v
    return r


def test_acl_first_match_lowest_index():
    rules = rules_of(dict(dip=0x0A000002, dip_mask=32, action=1), dict(dport_start=80, dport_end=80, action=0))
    o = pyoracle.Oracle(rules, default_action=0)
    r = o.classify_one(udp_packet())
    assert r["acl_hit"] == 0 and r["status"] == ST["ACL_DROP"]
    rules = rules[::-1].copy()
    o = pyoracle.Oracle(rules, default_action=1)
    r = o.classify_one(udp_packet())
    assert r["acl_hit"] == 0 and r["status"] == ST["ACL_FW"]


@pytest.mark.parametrize("plen,ip,hit", [(0, 0, True), (1, 0x00000000, True), (1, 0x80000000, False),
                                          (31, 0x0A000000, True), (31, 0x0A000002, False), (32, 0x0A000001, True),
                                          (32, 0x0A000003, False), (8, 0x0AFFFFFF, True)])
def test_acl_prefix_boundaries(plen, ip, hit):
    o = pyoracle.Oracle(rules_of(dict(sip=ip, sip_mask=plen, action=1)), default_action=0)
    r = o.classify_one(udp_packet(sip=0x0A000001))
    assert (r["acl_hit"] == 0) == hit


def test_acl_ranges_mac_time_default():
    base = dict(action=1)
    o = pyoracle.Oracle(rules_of(dict(base, dport_start=80, dport_end=80)), default_action=0)
    assert o.classify_one(udp_packet(dport=80))["acl_hit"] == 0
    assert o.classify_one(udp_packet(dport=81))["acl_hit"] == -1
    o = pyoracle.Oracle(rules_of(dict(base, protocol_start=6, protocol_end=6)), default_action=1)
    r = o.classify_one(udp_packet())
    assert r["acl_hit"] == -1 and r["status"] == ST["ACL_DROP"]  # default action DROP
    o = pyoracle.Oracle(rules_of(dict(base, smac=np.frombuffer(SMAC, np.uint8))), default_action=0)
    assert o.classify_one(udp_packet())["acl_hit"] == 0
    o = pyoracle.Oracle(rules_of(dict(base, dmac=np.frombuffer(SMAC, np.uint8))), default_action=0)
    assert o.classify_one(udp_packet())["acl_hit"] == -1
    o = pyoracle.Oracle(rules_of(dict(base, time_start=100, time_end=200)), default_action=0)
    assert o.classify_one(udp_packet(), ts=150)["acl_hit"] == 0
    assert o.classify_one(udp_packet(), ts=201)["acl_hit"] == -1
    assert o.classify_one(udp_packet(), ts=100)["acl_hit"] == 0
    o = pyoracle.Oracle(rules_of(dict(base, sport_start=9, sport_end=3)), default_action=0)
    assert o.classify_one(udp_packet(sport=5))["acl_hit"] == -1  # empty range never matches
    used = np.array([0], np.uint8)
    o = pyoracle.Oracle(rules_of(dict(base)), used=used, default_action=0)
    assert o.classify_one(udp_packet())["acl_hit"] == -1  # FREE entries are skipped
