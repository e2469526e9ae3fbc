"""TCP options (DecodeTCPOptions, dataplane/src/decode/decode-tcp.c:18-131, recorded at :175-177) and the compat
layer under concurrent use, on the GPU.

The reference records only the window-scale option (m->tcpvars.ws, :61-70: the first one of length 3; a duplicate is
ignored; an invalid option length ends the parse and keeps what was recorded).  It has no verdict effect.  The
kernel reports its byte offset from the TCP header in bits 9-15 of the tuple output; Decode() turns that into the
mbuf's tcpvars.ws.  Bit-exact against the oracle's restatement (oracle/ppe_oracle.c decode_tcp_options)."""
import ctypes as C
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

import torch  # noqa: E402

import pyoracle  # noqa: E402
from ppe import Engine, abi, synth  # noqa: E402
from ppe.abi import ST  # noqa: E402
from pktbuild import eth, ipv4, tcp, vlan  # noqa: E402

NOW = 1_700_000_000
DEV = torch.device("cuda:0")
OPTS = [b"\x01", b"\x00", b"\x02\x04\x05\xb4", b"\x03\x03\x07", b"\x04\x02", b"\x08\x0a" + b"\x11" * 8,
        b"\x03\x04\x01\x01", b"\x05\x0a" + b"\x22" * 8, b"\x03\x03\x0e"]


def random_tcp_packets(n, seed):
    """TCP packets whose option space (data offset 6..15) holds random sequences of NOP / EOL / MSS / WS / SACK-OK /
    TS / SACK options, window-scale options of the wrong length, duplicates, and random junk bytes (invalid lengths
    among them); some behind a VLAN tag or IPv4 options; SYN and non-SYN."""
    rng = np.random.default_rng(seed)
    frames = []
    for i in range(n):
        off = int(rng.integers(6, 16))
        space = 4 * (off - 5)
        if rng.random() < 0.15:
            opts = bytes(rng.integers(0, 256, space, dtype=np.uint8))
        else:
            opts = b""
            while len(opts) < space:
                opts += OPTS[int(rng.integers(0, len(OPTS)))]
            opts = opts[:space]
        ihl = 5 if rng.random() < 0.8 else int(rng.integers(6, 9))
        flags = 0x02 if rng.random() < 0.7 else 0x10
        l4 = tcp(int(rng.integers(1, 65536)), int(rng.integers(1, 65536)), flags=flags, off=off, opts=opts)
        l3 = ipv4(6, int(rng.integers(1, 1 << 32)), int(rng.integers(1, 1 << 32)), len(l4), ihl=ihl) + l4
        l2 = eth(0x8100) + vlan(0x0800) if rng.random() < 0.3 else eth(0x0800)
        frames.append(l2 + l3)
    return frames


def windows(frames, stride):
    hdr = np.zeros((len(frames), stride), np.uint8)
    lens = np.zeros(len(frames), np.uint32)
    for i, f in enumerate(frames):
        c = min(len(f), stride)
        hdr[i, :c] = np.frombuffer(f[:c], np.uint8)
        lens[i] = len(f)
    return hdr, lens


@pytest.mark.parametrize("stride", [128, 64])
def test_tcp_option_parse_vs_oracle(stride):
    frames = random_tcp_packets(20_000, seed=stride)
    hdr, lens = windows(frames, stride)
    rules = synth.make_rules(256, seed=5)
    eng = Engine(0)
    try:
        eng.commit(rules, default_action=1)
        n = len(lens)
        th = torch.from_numpy(hdr).to(DEV)
        tl = torch.from_numpy(lens.view(np.int32)).to(DEV)
        out = {k: torch.full((n,), -7, dtype=torch.int32, device=DEV) for k in ("verdict", "flow_hash", "acl_hit")}
        out["tuple"] = torch.full((n, 4), -7, dtype=torch.int32, device=DEV)
        eng.classify_torch(th, tl, out, cfg=eng.cfg(now_seconds=NOW))
        torch.cuda.synchronize()
    finally:
        eng.close()
    o = pyoracle.Oracle(rules, default_action=1)
    ref = o.classify_batch(hdr, lens, cfg=o.cfg(0, 1, NOW), nthreads=8)
    far = ref["reach"] > stride
    ok = ~far
    got = {k: v.cpu().numpy() for k, v in out.items()}
    assert np.array_equal(got["verdict"].view(np.uint32)[ok], ref["verdict"][ok])
    assert np.array_equal(got["tuple"].view(np.uint32)[ok], ref["tuple"][ok])
    ws = (ref["tuple"][:, 3] >> 9) & 0x3F
    past = (ref["tuple"][:, 3] & abi.TUPLE_OPT_PAST) != 0
    st = ref["verdict"] & 0xFF
    assert (ws[ok] > 0).sum() > 2000 and (ws[ok] == 0).sum() > 2000  # both outcomes well covered
    # a 64-B window cuts many option spaces short before their window-scale option (128 B holds these packets' options
    # whole: IPv4 options here reach ihl 8 only; tests/test_gpu_mbuf.py covers 128-B windows cut short)
    assert past[ok].sum() > 1000 if stride == 64 else not past.any()
    assert ((st[ok] == ST["ACL_FW"]) | (st[ok] == ST["ACL_DROP"]) | (st[ok] == ST["FLOW_TCP_NO_SYN_FIRST"])).mean() > 0.9
    assert ((got["verdict"].view(np.uint32)[far] & 0xFF) == ST["WINDOW_PUNT"]).all()


HOOK = C.CFUNCTYPE(None, C.POINTER(abi.Mbuf))


def test_decode_records_window_scale_option():
    """Decode(mbuf) fills m->tcpvars.ws as DecodeTCPOptions does (decode-tcp.c:66-69): the option's type, length and
    a data pointer into the packet two bytes past the option start; network / transport header pointers as
    DecodeIPV4 / DecodeTCP set them (decode-ipv4.c:42, :131-140)."""
    lib = abi.load()
    lib.ppe_set_output_hooks.argtypes = [HOOK, HOOK, HOOK]
    assert lib.DP_Acl_Rule_Init() == 0
    frames = random_tcp_packets(3000, seed=7)
    n = len(frames)
    bufs = [C.create_string_buffer(f, len(f)) for f in frames]
    mbufs = (abi.Mbuf * n)()
    for i in range(n):
        mbufs[i].pkt_ptr = C.cast(bufs[i], C.c_void_p)
        mbufs[i].pkt_totallen = len(frames[i])
    seen = []
    hooks = tuple(HOOK(lambda m: seen.append(1)) for _ in range(3))
    lib.ppe_set_output_hooks(*hooks)
    lib.Decode_Set_Burst(1000)
    for i in range(n):
        lib.Decode(C.byref(mbufs[i]))
    assert lib.Decode_Flush() >= 0
    lib.ppe_set_output_hooks(HOOK(), HOOK(), HOOK())
    assert len(seen) == n
    hdr, lens = windows(frames, 256)  # the whole frames: what the reference reads
    o = pyoracle.Oracle(np.zeros(0, abi.RULE_DTYPE), default_action=1)
    ref = o.classify_batch(hdr, lens, cfg=o.cfg(0, 1, 0))
    assert not (ref["tuple"][:, 3] & abi.TUPLE_OPT_PAST).any()
    found = 0
    for i in range(n):
        m = mbufs[i]
        flags = ref["verdict"][i] >> 16
        want = int((ref["tuple"][i][3] >> 9) & 0x3F)
        base = C.cast(bufs[i], C.c_void_p).value
        if flags & 0x2:  # PPE_F_L4: the header pointers
            l3 = 14 + (4 if m.vlan_idx else 0)
            assert m.network_header == base + l3
            assert m.transport_header == base + l3 + (frames[i][l3] & 0xF) * 4
        if want:
            found += 1
            assert m.tcpvars.ws == C.addressof(m) + abi.Mbuf.tcpvars.offset  # &m->TCP_OPTS[0]
            o0 = m.tcpvars.tcp_opts[0]
            assert (o0.type, o0.len) == (3, 3)
            assert o0.data == m.transport_header + want + 2
        else:
            assert not m.tcpvars.ws
    assert found > 500


def test_lookup_and_commit_while_threads_decode():
    """DP_Acl_Rule_Commit and DP_Acl_Lookup_Burst on the process's one engine context while 4 threads run
    Decode bursts.  Every call that uses the context takes its lock, so nothing corrupts: every mbuf reaches exactly
    one hook, every lookup answers with one of the two rule sets' results, every commit succeeds."""
    lib = abi.load()
    lib.ppe_set_output_hooks.argtypes = [HOOK, HOOK, HOOK]
    lib.DP_Acl_Lookup_Burst.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p]
    assert lib.DP_Acl_Rule_Init() == 0
    lib.ppe_rule_list_free()
    assert lib.ppe_rule_list_init() == 0
    sets = [synth.make_rules(300, seed=s) for s in (11, 12)]
    for i in range(300):
        rid = C.c_uint32()
        assert lib.Rule_add(sets[0][i:i + 1].ctypes.data, C.byref(rid)) == 0
    assert lib.DP_Acl_Rule_Commit() == 0
    pk = synth.make_packets(8000, sets[0], seed=13, kind="imix", stride=128, hit_frac=0.9)
    n = len(pk["len"])
    frames = [bytes(pk["hdr"][i][: min(int(pk["len"][i]) & 0xFFFF, 128)]) for i in range(n)]
    bufs = [C.create_string_buffer(f, max(len(f), 144)) for f in frames]  # (Decode reads up to 144 B)
    mbufs = (abi.Mbuf * n)()
    for i in range(n):
        mbufs[i].pkt_ptr = C.cast(bufs[i], C.c_void_p)
        mbufs[i].pkt_totallen = int(pk["len"][i])
    lock = threading.Lock()
    hits = np.zeros(n, np.int32)
    base = C.addressof(mbufs)

    def hook(m):
        with lock:
            hits[(C.addressof(m.contents) - base) // C.sizeof(abi.Mbuf)] += 1
    hooks = tuple(HOOK(hook) for _ in range(3))
    lib.ppe_set_output_hooks(*hooks)
    lib.Decode_Set_Burst(200)
    errors = []

    def decoder(t):
        try:
            for i in range(t, n, 4):
                lib.Decode(C.byref(mbufs[i]))
            if lib.Decode_Flush() < 0:
                errors.append("flush")
        except Exception as e:  # pragma: no cover
            errors.append(repr(e))

    # lookups on a separate mbuf copy of some decoded packets' tuples
    probe = (abi.Mbuf * 64)()
    for j in range(64):
        probe[j].sip, probe[j].dip = int(pk["hdr"][j][26:30].view(">u4")[0]), int(pk["hdr"][j][30:34].view(">u4")[0])
        probe[j].sport, probe[j].dport, probe[j].proto = 1000 + j, 2000 + j, 17
    ptrs = (C.c_void_p * 64)(*(C.addressof(probe[j]) for j in range(64)))
    acts = (C.c_int * 64)()
    stop = threading.Event()
    commits, lookups = [], []

    def control():
        k = 0
        while not stop.is_set():
            lookups.append(lib.DP_Acl_Lookup_Burst(ptrs, 64, acts))
            if k % 4 == 0:
                assert lib.Rule_del_all() == 0
                for i in range(300):
                    rid = C.c_uint32()
                    lib.Rule_add(sets[(k // 4) % 2][i:i + 1].ctypes.data, C.byref(rid))
                commits.append(lib.DP_Acl_Rule_Commit())
            k += 1
    ths = [threading.Thread(target=decoder, args=(t,)) for t in range(4)]
    ctl = threading.Thread(target=control)
    ctl.start()
    for t in ths:
        t.start()
    for t in ths:
        t.join(120)
    stop.set()
    ctl.join(60)
    lib.ppe_set_output_hooks(HOOK(), HOOK(), HOOK())
    assert not errors and not any(t.is_alive() for t in ths) and not ctl.is_alive()
    assert (hits == 1).all()
    assert lookups and all(r == 0 for r in lookups) and commits and all(r == 0 for r in commits)
    refs = []
    zmac = np.zeros(6, np.uint8)
    for rs in sets:
        o = pyoracle.Oracle(rs, default_action=1)
        refs.append([o.lib.oracle_acl_linear(probe[j].sip, probe[j].dip, probe[j].sport, probe[j].dport, 17,
                                             zmac.ctypes.data, zmac.ctypes.data, 0, None) for j in range(64)])
    got = [probe[j].ppe_acl_hit for j in range(64)]
    assert got in refs
    lib.ppe_rule_list_free()
