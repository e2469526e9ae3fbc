"""The PPE-compatible surface (include/ppe_acl.h, include/ppe_decode.h) end to end on the GPU: rule store →
DP_Acl_Rule_Commit → Decode() bursts delivered through the output hooks, DP_Log_Func on the logged drop reasons,
DP_Acl_Lookup(mbuf)."""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

import torch  # noqa: E402,F401

import pyoracle  # noqa: E402
from ppe import abi, synth  # noqa: E402
from ppe.abi import ST  # noqa: E402


Mbuf = abi.Mbuf


HOOK = C.CFUNCTYPE(None, C.POINTER(Mbuf))
ALERT = C.CFUNCTYPE(C.c_int, C.c_void_p)
LOGGED = {ST[k] for k in ("L2_HEADER_ERR", "VLAN_HEADER_ERR", "IPV4_HEADER_ERR", "IPV4_VERSION_ERR", "IPV4_LEN_ERR",
                          "FRAG_LEN_ERR", "UDP_HEADER_ERR", "UDP_LEN_ERR", "TCP_HEADER_ERR", "TCP_LEN_ERR",
                          "ACL_DROP")}


def test_rule_store_commit_decode_hooks():
    lib = abi.load()
    lib.ppe_set_output_hooks.argtypes = [HOOK, HOOK, HOOK]
    lib.reg_fw_alert.argtypes = [ALERT]
    assert lib.DP_Acl_Rule_Init() == 0
    lib.ppe_rule_list_free()
    assert lib.ppe_rule_list_init() == 0
    rules = synth.make_rules(200, seed=90, resid_frac=0.2)
    ids = []
    for i in range(len(rules)):
        rid = C.c_uint32()
        assert lib.Rule_add(rules[i:i + 1].ctypes.data, C.byref(rid)) == 0
        ids.append(rid.value)
    assert ids == list(range(200))
    assert lib.Rule_del_by_id(17) == 0  # a FREE hole
    assert lib.DP_Acl_Rule_Commit() == 0
    used = np.ones(200, np.uint8)
    used[17] = 0

    pk = synth.make_packets(5000, rules, seed=91, kind="imix", stride=128, malformed_frac=0.1, with_ts=True)
    n = len(pk["len"])
    frames = [bytes(pk["hdr"][i][: min(int(pk["len"][i]) & 0xFFFF, 128)]) for i in range(n)]
    bufs = [C.create_string_buffer(f, max(len(f), 1)) for f in frames]
    mbufs = (Mbuf * n)()
    for i in range(n):
        mbufs[i].pkt_ptr = C.cast(bufs[i], C.c_void_p)
        mbufs[i].pkt_totallen = int(pk["len"][i])
        mbufs[i].timestamp = int(pk["ts"][i])
    base = C.addressof(mbufs)
    got = {"fw": [], "drop": [], "punt": [], "log": 0}

    def mk(key):
        return HOOK(lambda m: got[key].append((C.addressof(m.contents) - base) // C.sizeof(Mbuf)))

    def alert(p):
        got["log"] += 1
        return 0

    hooks = (mk("fw"), mk("drop"), mk("punt"), ALERT(alert))
    lib.ppe_set_output_hooks(hooks[0], hooks[1], hooks[2])
    lib.reg_fw_alert(hooks[3])
    lib.Decode_Set_Burst(1024)
    for i in range(n):
        lib.Decode(C.byref(mbufs[i]))
    assert lib.Decode_Flush() >= 0

    o = pyoracle.Oracle(rules, used, default_action=1)
    ref = o.classify_batch(pk["hdr"], pk["len"], ts=pk["ts"], cfg=o.cfg(0, 1, 0))
    act = (ref["verdict"] >> 8) & 0xFF
    assert sorted(got["fw"]) == np.nonzero(act == 0)[0].tolist()
    assert sorted(got["drop"]) == np.nonzero(act == 1)[0].tolist()
    assert sorted(got["punt"]) == np.nonzero(act == 2)[0].tolist()
    assert got["log"] == int(np.isin(ref["verdict"] & 0xFF, list(LOGGED)).sum())
    v = np.array([mbufs[i].ppe_verdict for i in range(n)], np.uint32)
    h = np.array([mbufs[i].ppe_acl_hit for i in range(n)], np.int32)
    assert np.array_equal(v, ref["verdict"]) and np.array_equal(h, ref["acl_hit"])
    l4 = np.nonzero((ref["verdict"] >> 16) & 0x10)[0]  # PPE_F_ACL
    for i in l4[:200]:
        assert (mbufs[i].sip, mbufs[i].dip, mbufs[i].sport, mbufs[i].dport) == tuple(int(x) for x in (
            ref["tuple"][i][0], ref["tuple"][i][1], ref["tuple"][i][2] & 0xFFFF, ref["tuple"][i][2] >> 16))

    # DP_Acl_Lookup on decoded mbufs (flow.c:232 contract: DROP iff the rule/default action is DROP)
    lib.DP_Acl_Lookup.argtypes = [C.POINTER(Mbuf)]
    for i in l4[:100]:
        a = lib.DP_Acl_Lookup(C.byref(mbufs[i]))
        assert a == (1 if ref["verdict"][i] & 0xFF == ST["ACL_DROP"] else 0)
        assert mbufs[i].ppe_acl_hit == ref["acl_hit"][i]
    assert C.c_int.in_dll(lib, "gNumTreeNode").value > 0
    lib.ppe_rule_list_free()
    lib.DP_Acl_Rule_Release()
