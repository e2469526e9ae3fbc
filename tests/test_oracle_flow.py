"""Known answers for the oracle's flow table (dataplane/src/flow/flow.c), derived from the cited reference lines.

The flow table is the first §8(f) row: a packet whose flow exists is forwarded without an ACL lookup and updates
the flow's counters; a miss goes through syn_check and the ACL and, on FW, creates the flow (FlowAdd), or fails
when the pool is empty.  These cases pin the oracle that tests/test_gpu_flow.py holds the HIP path to."""
import numpy as np
import pytest

import pyoracle
from ppe import abi
from ppe.abi import ST, F_ACL, F_FLOW, F_NEWFLOW, F_TOCLIENT
from pktbuild import tcp_packet, udp_packet

C = {name: i for i, name in enumerate(abi.COUNTERS)}
A, B = 0x0A000001, 0x0A000002
NOW = 1_700_000_000


def rule(action=0, sip=0, sip_mask=0, dip=0, dip_mask=0, sport=(0, 65535), dport=(0, 65535), proto=(0, 255)):
    r = np.zeros(1, abi.RULE_DTYPE)
    r["sip"], r["sip_mask"], r["dip"], r["dip_mask"] = sip, sip_mask, dip, dip_mask
    r["sport_start"], r["sport_end"] = sport
    r["dport_start"], r["dport_end"] = dport
    r["protocol_start"], r["protocol_end"] = proto
    r["action"] = action
    return r


def batch(pkts, stride=64):
    hdr = np.zeros((len(pkts), stride), np.uint8)
    lens = np.zeros(len(pkts), np.uint32)
    for i, p in enumerate(pkts):
        b = bytes(p)
        hdr[i, :min(len(b), stride)] = np.frombuffer(b[:stride], np.uint8)
        lens[i] = len(b)
    return hdr, lens


def run(ft, pkts, now=NOW, syn_check=1):
    hdr, lens = batch(pkts)
    return ft.classify_batch(hdr, lens, cfg=pyoracle.Oracle.cfg(0, syn_check, now))


def fields(v):
    return v & 0xFF, (v >> 8) & 0xFF, v >> 16


@pytest.fixture
def fw_all():
    """No rule matches anything; default FW"""
    o = pyoracle.Oracle(np.zeros(0, abi.RULE_DTYPE), default_action=abi.ACL_RULE_ACTION_FW)
    ft = pyoracle.OracleFlow(o, capacity=100)
    yield o, ft
    ft.close()


def test_first_packet_creates_later_packets_hit(fw_all):
    _, ft = fw_all
    fwd = udp_packet(sip=A, dip=B, sport=1234, dport=80)
    rev = udp_packet(sip=B, dip=A, sport=80, dport=1234)
    r = run(ft, [fwd, fwd, rev])
    st, act, fl = fields(r["verdict"])
    assert (st == ST["ACL_FW"]).all() and (act == 0).all()
    # packet 0: miss → ACL (flow.c:232) → FlowAdd (flow.c:243), to-server; packets 1-2: FlowFind hit, no ACL
    assert fl[0] & F_ACL and fl[0] & F_NEWFLOW and fl[0] & F_FLOW and not fl[0] & F_TOCLIENT
    assert not fl[1] & (F_ACL | F_NEWFLOW) and fl[1] & F_FLOW and not fl[1] & F_TOCLIENT
    assert not fl[2] & F_ACL and fl[2] & F_TOCLIENT  # FlowGetPacketDirection, flow.c:248-269
    assert r["acl_hit"].tolist() == [-1, -1, -1]  # no rule matched on the miss, not consulted on hits
    assert r["counters"][C["acl_fw"]] == 3 and r["counters"][C["flow_proc_ok"]] == 3  # flow.c:199,240,309
    d = ft.dump()
    assert len(d) == 1 and (d["sip"][0], d["dip"][0], d["sport"][0], d["dport"][0], d["protocol"][0]) == (A, B, 1234, 80, 17)
    # FlowUpdate, flow.c:163-178: by sport equality, bytes = pkt_totallen
    assert (d["pktcnts2d"][0], d["pktcntd2s"][0]) == (2, 1)
    assert (d["bytecnts2d"][0], d["bytecntd2s"][0]) == (2 * len(fwd), len(rev))
    assert d["last_seen"][0] == NOW
    assert ft.stats() == dict(live=1, new_flow=1, del_flow=0)


def test_syn_check_only_first_packet(fw_all):
    _, ft = fw_all
    ack = tcp_packet(flags=0x10)
    syn = tcp_packet(flags=0x02)
    r = run(ft, [ack, syn, ack])
    st, act, fl = fields(r["verdict"])
    # flow.c:204-214: a TCP miss without SYN is dropped and creates nothing; after the SYN created the flow, the
    # same ACK finds it
    assert st.tolist() == [ST["FLOW_TCP_NO_SYN_FIRST"], ST["ACL_FW"], ST["ACL_FW"]]
    assert act.tolist() == [1, 0, 0]
    assert fl[1] & F_NEWFLOW and fl[2] & F_FLOW and not fl[2] & F_NEWFLOW
    assert r["counters"][C["flow_tcp_no_syn_first"]] == 1 and r["counters"][C["flow_proc_fail"]] == 1


def test_acl_drop_creates_no_flow_reverse_direction_hits():
    # the rule drops B → A only; A → B creates the flow and B → A then finds it (ACL consulted on misses only)
    rules = rule(action=1, sip=B, sip_mask=32, dip=A, dip_mask=32)
    o = pyoracle.Oracle(rules, default_action=abi.ACL_RULE_ACTION_FW)
    ft = pyoracle.OracleFlow(o, capacity=10)
    rev = udp_packet(sip=B, dip=A, sport=80, dport=1234)
    fwd = udp_packet(sip=A, dip=B, sport=1234, dport=80)
    r = run(ft, [rev, rev, fwd, rev])
    st, act, fl = fields(r["verdict"])
    assert st.tolist() == [ST["ACL_DROP"], ST["ACL_DROP"], ST["ACL_FW"], ST["ACL_FW"]]
    assert r["acl_hit"].tolist() == [0, 0, -1, -1]
    assert fl[3] & F_TOCLIENT and not fl[3] & F_ACL
    assert r["counters"][C["acl_drop"]] == 2 and r["counters"][C["acl_fw"]] == 2
    ft.close()


def test_pool_exhausted_nomem():
    o = pyoracle.Oracle(np.zeros(0, abi.RULE_DTYPE), default_action=abi.ACL_RULE_ACTION_FW)
    ft = pyoracle.OracleFlow(o, capacity=2)
    pk = [udp_packet(sport=1000 + i) for i in range(3)] + [udp_packet(sport=1002), udp_packet(sport=1000)]
    r = run(ft, pk)
    st, act, fl = fields(r["verdict"])
    # flow.c:124-129: STAT_FLOW_NODE_NOMEM after STAT_ACL_FW, FlowHandlePacket drops (flow.c:278-284)
    assert st.tolist() == [ST["ACL_FW"], ST["ACL_FW"], ST["FLOW_NOMEM"], ST["FLOW_NOMEM"], ST["ACL_FW"]]
    assert act.tolist() == [0, 0, 1, 1, 0]
    c = r["counters"]
    assert c[C["flow_node_nomem"]] == 2 and c[C["acl_fw"]] == 5 and c[C["flow_proc_fail"]] == 2
    assert c[C["out_drop"]] == 2 and c[C["flow_proc_ok"]] == 3
    assert ft.stats()["live"] == 2
    ft.close()


def test_aging_strictly_greater(fw_all):
    _, ft = fw_all
    run(ft, [udp_packet(sport=1)], now=100)
    run(ft, [udp_packet(sport=2)], now=110)
    # FlowTimeOut, flow.c:391-410: removed iff now > cycle and now - cycle > timeout
    assert ft.age(120, 20) == 0
    assert ft.age(121, 20) == 1
    assert ft.stats() == dict(live=1, new_flow=2, del_flow=1)
    r = run(ft, [udp_packet(sport=1), udp_packet(sport=2)], now=125)
    st, _, fl = fields(r["verdict"])
    assert fl[0] & F_NEWFLOW and not fl[1] & F_NEWFLOW
    d = ft.dump()
    assert sorted(d["last_seen"].tolist()) == [125, 125]


def test_equal_ports_direction_by_address(fw_all):
    _, ft = fw_all
    # sport == dport: FlowGetPacketDirection compares addresses (flow.c:259-265); FlowUpdate still compares
    # sport only, so both directions count as s2d (flow.c:166-177)
    p = udp_packet(sip=A, dip=B, sport=53, dport=53)
    q = udp_packet(sip=B, dip=A, sport=53, dport=53)
    r = run(ft, [p, q])
    _, _, fl = fields(r["verdict"])
    assert not fl[0] & F_TOCLIENT and fl[1] & F_TOCLIENT
    d = ft.dump()
    assert (d["pktcnts2d"][0], d["pktcntd2s"][0]) == (2, 0)


def test_stateless_equivalence_unique_flows():
    """With every flow distinct, the table changes nothing but the flow flags."""
    from ppe import synth
    rules = synth.make_rules(64, seed=3)
    pk = synth.make_packets(4000, rules, seed=11, kind="imix", stride=128)
    o = pyoracle.Oracle(rules, default_action=1)
    ft = pyoracle.OracleFlow(o, capacity=100000)
    cfg = o.cfg(0, 1, NOW)
    a = o.classify_batch(pk["hdr"], pk["len"], pk.get("ts"), cfg=cfg)
    b = ft.classify_batch(pk["hdr"], pk["len"], pk.get("ts"), cfg=cfg)
    # unique tuples ⇒ every packet misses: identical verdicts except the FLOW/NEWFLOW/TOCLIENT flags
    tup = a["tuple"][:, :3]
    key = np.minimum(tup[:, 0], tup[:, 1]).astype(np.uint64) << 32 | np.maximum(tup[:, 0], tup[:, 1])
    _, first = np.unique(np.stack([key, tup[:, 2] & 0xFFFF, tup[:, 2] >> 16, a["tuple"][:, 3] & 0xFF], 1), axis=0,
                         return_index=True)
    uniq = np.zeros(len(key), bool)
    uniq[first] = True
    l4 = (a["verdict"] >> 16) & abi.F_L4 != 0
    dup = l4 & ~uniq
    m = ~dup
    mask = ~np.uint32((F_FLOW | F_NEWFLOW | F_TOCLIENT) << 16)
    assert np.array_equal(a["verdict"][m], b["verdict"][m] & mask)
    assert np.array_equal(a["acl_hit"][m], b["acl_hit"][m])
    assert np.array_equal(a["flow_hash"], b["flow_hash"])
    ft.close()
