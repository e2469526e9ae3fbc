"""Deterministic synthetic rule sets and packet batches for the benchmark configs (seed 0x5EED).

C0  10k × 64 B IPv4/UDP, 16 rules            C1  1M × 64 B IPv4/UDP, 256 rules
C2  IMIX 64/570/1500 (7:4:1), 50 % VLAN, TCP(SYN):UDP 1:1, 4096 rules
C3  64 B IPv4/UDP, 65,536 rules              C4  64 B, 4096 rules, 1M packets per GPU

Rules: random prefixes /8–/32; ports 25 % exact / 50 % range / 25 % any; protocol 6 / 17 / any; actions 50/50;
default DROP.  Packets: 50 % draw sip/dip (and usually ports/proto) from a random rule so hits land at varied
indices, 50 % uniform; ~1 % malformed, spread over every drop reason of the decoder.
"""
from __future__ import annotations

import numpy as np

from .abi import RULE_DTYPE

SEED = 0x5EED

CONFIGS = {
    "C0": dict(n=10_000, rules=16, kind="udp64"),
    "C1": dict(n=1 << 20, rules=256, kind="udp64"),
    "C2": dict(n=1 << 20, rules=4096, kind="imix"),
    "C3": dict(n=1 << 20, rules=65536, kind="udp64"),
    "C4": dict(n=1 << 20, rules=4096, kind="udp64"),
    # stateful flow table: 1M-packet batches over 256k bidirectional UDP flows, default FW
    "F1": dict(n=1 << 20, rules=256, kind="udp64", flows=1 << 18),
    # IPv4 reassembly: 65,536-fragment batches (ppe_defrag's default max_batch) of a
    # make_fragment_stream mix, every batch over fresh datagrams; an FCB pool large enough that no batch hits FCB_FULL
    "D1": dict(n=1 << 16, rules=256, kind="frag", fcb_max=1 << 20),
}

MAC_POOL = 16
N_MALFORMED_KINDS = 24


def _mac_pool(rng):
    pool = rng.integers(0, 256, size=(MAC_POOL, 6), dtype=np.uint8)
    pool[:, 0] = (pool[:, 0] | 0x02) & 0xFE  # locally administered unicast, never all-zero
    return pool


def make_rules(n_rules: int, seed: int = SEED, resid_frac: float = 0.0, any_ip_frac: float = 0.0,
               now: int = 1_700_000_000) -> np.ndarray:
    rng = np.random.default_rng(seed)
    r = np.zeros(n_rules, RULE_DTYPE)
    if n_rules == 0:
        return r
    for f in ("sip", "dip"):
        plen = rng.integers(8, 33, n_rules)
        r[f] = rng.integers(0, 1 << 32, n_rules, dtype=np.uint64).astype(np.uint32)
        r[f + "_mask"] = plen
        if any_ip_frac:
            anyip = rng.random(n_rules) < any_ip_frac
            r[f][anyip] = 0
            r[f + "_mask"][anyip] = 0
    for f in ("sport", "dport"):
        kind = rng.choice(3, n_rules, p=[0.25, 0.5, 0.25])  # exact / range / any
        a = rng.integers(0, 65536, n_rules)
        b = rng.integers(0, 65536, n_rules)
        lo, hi = np.minimum(a, b), np.maximum(a, b)
        lo = np.where(kind == 0, a, np.where(kind == 1, lo, 0))
        hi = np.where(kind == 0, a, np.where(kind == 1, hi, 65535))
        r[f + "_start"] = lo
        r[f + "_end"] = hi
    pk = rng.integers(0, 3, n_rules)
    r["protocol_start"] = np.where(pk == 0, 6, np.where(pk == 1, 17, 0))
    r["protocol_end"] = np.where(pk == 0, 6, np.where(pk == 1, 17, 255))
    r["action"] = rng.integers(0, 2, n_rules)
    r["logable"] = rng.integers(0, 2, n_rules)
    if resid_frac:
        pool = _mac_pool(np.random.default_rng(seed ^ 0xA5A5))
        sel = np.nonzero(rng.random(n_rules) < resid_frac)[0]
        for i in sel:
            k = rng.integers(0, 4)
            if k in (0, 3):
                r["smac"][i] = pool[rng.integers(0, MAC_POOL)]
            if k in (1, 3):
                r["dmac"][i] = pool[rng.integers(0, MAC_POOL)]
            if k in (2, 3):
                t0 = now + int(rng.integers(-1000, 1000))
                r["time_start"][i] = t0
                r["time_end"][i] = t0 + int(rng.integers(0, 2000))
    return r


def _prefix_draw(rng, ip, plen):
    """Random address inside each prefix (ip/plen arrays)."""
    plen = plen.astype(np.uint64)
    host_bits = np.where(plen >= 32, 0, 32 - plen)
    mask = ((np.uint64(1) << host_bits) - np.uint64(1)).astype(np.uint64)
    rnd = rng.integers(0, 1 << 32, len(ip), dtype=np.uint64)
    base = ip.astype(np.uint64) & ~mask & np.uint64(0xFFFFFFFF)
    return (base | (rnd & mask)).astype(np.uint32)


def _put16(hdr, rows, off, val):
    val = np.asarray(val, dtype=np.uint32)
    hdr[rows, off] = (val >> 8) & 0xFF
    hdr[rows, off + 1] = val & 0xFF


def _put32(hdr, rows, off, val):
    val = np.asarray(val, dtype=np.uint64)
    for k in range(4):
        hdr[rows, off + k] = (val >> np.uint64(24 - 8 * k)) & np.uint64(0xFF)


def make_packets(n: int, rules: np.ndarray, seed: int = SEED + 1, kind: str = "udp64", stride: int = 64,
                 malformed_frac: float = 0.01, hit_frac: float = 0.5, vlan_frac: float | None = None,
                 tcp_frac: float | None = None, now: int = 1_700_000_000, with_ts: bool = False):
    """Returns dict(hdr=(n, stride) uint8, len=(n,) uint32, ts=(n,) uint64 or None, kinds=(n,) int16)."""
    rng = np.random.default_rng(seed)
    if kind == "imix":
        lens = rng.choice(np.array([64, 570, 1500], np.uint32), n, p=[7 / 12, 4 / 12, 1 / 12])
        vlan_frac = 0.5 if vlan_frac is None else vlan_frac
        tcp_frac = 0.5 if tcp_frac is None else tcp_frac
    else:
        lens = np.full(n, 64, np.uint32)
        vlan_frac = 0.0 if vlan_frac is None else vlan_frac
        tcp_frac = 0.0 if tcp_frac is None else tcp_frac
    vlan = rng.random(n) < vlan_frac
    tcp = rng.random(n) < tcp_frac
    pool = _mac_pool(np.random.default_rng(SEED ^ 0xA5A5))
    dmac = pool[rng.integers(0, MAC_POOL, n)]
    smac = pool[rng.integers(0, MAC_POOL, n)]

    sip = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
    dip = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
    sport = rng.integers(0, 65536, n).astype(np.uint32)
    dport = rng.integers(0, 65536, n).astype(np.uint32)
    if len(rules) and hit_frac > 0:
        hit = np.nonzero(rng.random(n) < hit_frac)[0]
        ri = rng.integers(0, len(rules), len(hit))
        sip[hit] = _prefix_draw(rng, rules["sip"][ri], rules["sip_mask"][ri])
        dip[hit] = _prefix_draw(rng, rules["dip"][ri], rules["dip_mask"][ri])
        inport = rng.random(len(hit)) < 0.8  # most of them also inside the rule's port ranges
        for f, arr in (("sport", sport), ("dport", dport)):
            lo = rules[f + "_start"][ri].astype(np.int64)
            hi = rules[f + "_end"][ri].astype(np.int64)
            v = lo + (rng.random(len(hit)) * (hi - lo + 1)).astype(np.int64)
            arr[hit[inport]] = np.minimum(v, hi)[inport].astype(np.uint32)
        p_lo = rules["protocol_start"][ri]
        tcp[hit] = np.where(p_lo == 6, True, np.where(p_lo == 17, False, tcp[hit]))
    proto = np.where(tcp, 6, 17).astype(np.uint32)

    hdr = np.zeros((n, stride), np.uint8)
    rows = np.arange(n)
    w = min(stride, 64)
    hdr[:, 0:6] = dmac
    hdr[:, 6:12] = smac
    l3 = np.where(vlan, 18, 14)
    _put16(hdr, rows, 12, np.where(vlan, 0x8100, 0x0800))
    vr = rows[vlan]
    _put16(hdr, vr, 14, rng.integers(0, 4096, len(vr)))
    _put16(hdr, vr, 16, 0x0800)
    ip_len = lens - l3
    hdr[rows, l3] = 0x45
    _put16(hdr, rows, l3 + 2, ip_len)
    _put16(hdr, rows, l3 + 4, rng.integers(0, 65536, n))
    _put16(hdr, rows, l3 + 6, np.where(rng.random(n) < 0.5, 0x4000, 0))  # DF or nothing
    hdr[rows, l3 + 8] = 64
    hdr[rows, l3 + 9] = proto
    _put16(hdr, rows, l3 + 10, rng.integers(0, 65536, n))
    _put32(hdr, rows, l3 + 12, sip)
    _put32(hdr, rows, l3 + 16, dip)
    l4 = l3 + 20
    _put16(hdr, rows, l4, sport)
    _put16(hdr, rows, l4 + 2, dport)
    u = rows[~tcp]
    _put16(hdr, u, l4[u] + 4, ip_len[u] - 20)
    _put16(hdr, u, l4[u] + 6, rng.integers(0, 65536, len(u)))
    t = rows[tcp]
    _put32(hdr, t, l4[t] + 4, rng.integers(0, 1 << 32, len(t), dtype=np.uint64))
    _put32(hdr, t, l4[t] + 8, 0)
    hdr[t, l4[t] + 12] = 0x50
    hdr[t, l4[t] + 13] = 0x02  # SYN, so syn_check does not mask the ACL result
    _put16(hdr, t, l4[t] + 14, rng.integers(0, 65536, len(t)))
    if w < stride:
        pass  # bytes past 64 stay zero for well-formed packets (payload is never read)
    kinds = np.full(n, -1, np.int16)
    if malformed_frac > 0:
        bad = np.nonzero(rng.random(n) < malformed_frac)[0]
        kinds[bad] = rng.integers(0, N_MALFORMED_KINDS, len(bad))
        for i in bad:
            _malform(hdr, lens, int(i), int(kinds[i]), rng, stride)
    ts = None
    if with_ts:
        ts = (now + rng.integers(-1500, 1500, n)).astype(np.uint64)
    return dict(hdr=hdr, len=lens, ts=ts, kinds=kinds)


def make_flow_packets(n: int, rules: np.ndarray, n_flows: int, seed: int = SEED + 3, kind: str = "udp64",
                      stride: int = 64, rev_frac: float = 0.4, syn_frac: float = 0.3, tcp_frac: float | None = None,
                      malformed_frac: float = 0.0, template_seed: int | None = None):
    """Stateful traffic for the flow table: n packets drawn uniformly from n_flows flow templates (make_packets
    tuples), each sent in the reverse direction (addresses and ports swapped) with probability rev_frac; TCP packets
    carry SYN with probability syn_frac, else ACK (so syn_check drops some first packets).  Same dict as
    make_packets, plus flow=(n,) template index.  template_seed (default: seed) fixes the flow population, so
    batches drawn with different seeds revisit the same flows."""
    base = make_packets(n_flows, rules, seed=seed if template_seed is None else template_seed, kind=kind,
                        stride=stride, malformed_frac=0.0, tcp_frac=tcp_frac)
    rng = np.random.default_rng(seed ^ 0xF10)
    idx = rng.integers(0, n_flows, n)
    hdr = base["hdr"][idx].copy()
    lens = base["len"][idx].copy()
    rows = np.arange(n)
    l3 = np.where(hdr[:, 12] == 0x81, 18, 14)
    l4 = l3 + 20
    rev = rows[rng.random(n) < rev_frac]
    for a, b, w in ((12, 16, 4), (20, 22, 2)):  # sip <-> dip, sport <-> dport (offsets from L3)
        for k in range(w):
            x = hdr[rev, l3[rev] + a + k].copy()
            hdr[rev, l3[rev] + a + k] = hdr[rev, l3[rev] + b + k]
            hdr[rev, l3[rev] + b + k] = x
    t = rows[hdr[rows, l3 + 9] == 6]
    hdr[t, l4[t] + 13] = np.where(rng.random(len(t)) < syn_frac, 0x02, 0x10)
    kinds = np.full(n, -1, np.int16)
    if malformed_frac > 0:
        bad = np.nonzero(rng.random(n) < malformed_frac)[0]
        kinds[bad] = rng.integers(0, N_MALFORMED_KINDS, len(bad))
        for i in bad:
            _malform(hdr, lens, int(i), int(kinds[i]), rng, stride)
    return dict(hdr=hdr, len=lens, ts=None, kinds=kinds, flow=idx)


def _set16(h, off, v):
    h[off] = (v >> 8) & 0xFF
    h[off + 1] = v & 0xFF


def _malform(hdr, lens, i, k, rng, stride):
    """Rewrite packet i into malformed variant k (one per decoder drop/punt reason)."""
    h = hdr[i]
    vlan = h[12] == 0x81
    l3 = 18 if vlan else 14
    if k == 0:      # len < 14 → L2_HEADER_ERR
        lens[i] = int(rng.integers(0, 14))
    elif k == 1:    # zero dst MAC
        h[0:6] = 0
    elif k == 2:    # zero src MAC
        h[6:12] = 0
    elif k == 3:    # IPv6 ethertype → L2_UNSUPPORT
        _set16(h, 12, 0x86DD)
    elif k == 4:    # second VLAN tag → VLAN_LAYER_EXCEED
        _set16(h, 12, 0x8100)
        _set16(h, 16, 0x9100)
    elif k == 5:    # VLAN with ARP inside → VLAN_UNSUPPORT
        _set16(h, 12, 0x8100)
        _set16(h, 16, 0x0806)
    elif k == 6:    # IP version 6 → IPV4_VERSION_ERR
        h[l3] = 0x65
    elif k == 7:    # ihl 4 → IPV4_HEADER_ERR
        h[l3] = 0x44
    elif k == 8:    # ip_len > buffer → IPV4_LEN_ERR
        _set16(h, l3 + 2, int(lens[i]) - l3 + 1 + int(rng.integers(0, 100)))
    elif k == 9:    # ip_len < hlen → IPV4_LEN_ERR
        _set16(h, l3 + 2, int(rng.integers(0, 20)))
    elif k == 10:   # MF fragment → FRAG (punt)
        _set16(h, l3 + 6, 0x2000 | int(rng.integers(0, 8)))
    elif k == 11:   # fragment with no payload → FRAG_LEN_ERR
        lens[i] = l3 + 20
        _set16(h, l3 + 2, 20)
        _set16(h, l3 + 6, 0x0001)
    elif k == 12:   # ICMP → IPV4_UNSUPPORT
        h[l3 + 9] = 1
    elif k == 13:   # UDP length mismatch → UDP_LEN_ERR
        h[l3 + 9] = 17
        ul = (int(h[l3 + 24]) << 8) | int(h[l3 + 25])
        _set16(h, l3 + 24, (ul + 1 + int(rng.integers(0, 3))) & 0xFFFF)
    elif k == 14:   # l4len < 8 → UDP_HEADER_ERR
        h[l3 + 9] = 17
        _set16(h, l3 + 2, 20 + int(rng.integers(0, 8)))
    elif k == 15:   # TCP data offset < 5 → TCP_LEN_ERR
        h[l3 + 9] = 6
        h[l3 + 32] = int(rng.integers(0, 5)) << 4
        h[l3 + 33] = 0x02
    elif k == 16:   # TCP without SYN → FLOW_TCP_NO_SYN_FIRST
        h[l3 + 9] = 6
        h[l3 + 32] = 0x50
        h[l3 + 33] = 0x10
    elif k == 17:   # IPv4 options (ihl 6..8), UDP behind them → slow-path L4
        ihl = int(rng.integers(6, 9))
        ip_len = int(lens[i]) - l3
        h[l3] = 0x40 | ihl
        h[l3 + 9] = 17
        _set16(h, l3 + 2, ip_len)
        o = l3 + 4 * ihl
        h[l3 + 20:o] = 0x01  # NOP options
        sp, dp = int(rng.integers(0, 65536)), int(rng.integers(0, 65536))
        if o + 8 <= stride:
            _set16(h, o, sp)
            _set16(h, o + 2, dp)
            _set16(h, o + 4, ip_len - 4 * ihl)
    elif k == 18:   # OSPF fragment → not defragmented → IPV4_UNSUPPORT
        h[l3 + 9] = 89
        _set16(h, l3 + 6, 0x2000)
    elif k == 19:   # TCP header longer than l4len → TCP_LEN_ERR
        h[l3 + 9] = 6
        _set16(h, l3 + 2, 20 + 24)
        h[l3 + 32] = 0xF0
        h[l3 + 33] = 0x02
    elif k == 20:   # VLAN tag cut short → VLAN_HEADER_ERR
        _set16(h, 12, 0x8100)
        lens[i] = 14 + int(rng.integers(0, 4))
    elif k == 21:   # wire length > 65535: Decode() truncates to uint16 (decode.c:22)
        lens[i] = int(lens[i]) + 65536
    elif k == 22:   # ihl 15 + TCP: headers reach past byte 64 (WINDOW_PUNT at stride 64)
        ip_len = int(lens[i]) - l3
        if ip_len >= 80:
            h[l3] = 0x4F
            h[l3 + 9] = 6
            o = l3 + 60
            h[l3 + 20:min(o, stride)] = 0x01
            if o + 14 <= stride:
                _set16(h, o, int(rng.integers(0, 65536)))
                _set16(h, o + 2, int(rng.integers(0, 65536)))
                h[o + 12] = 0x50
                h[o + 13] = 0x02
        else:
            h[l3] = 0x4F  # ip_len < 60 → IPV4_LEN_ERR
    elif k == 23:   # TCP segment shorter than its 20-B header → TCP_HEADER_ERR
        h[l3 + 9] = 6
        _set16(h, l3 + 2, 20 + int(rng.integers(0, 20)))



# ---- IPv4 fragment streams (ppe_defrag) ------------------------------------------------------
def _frag_frame(rng, proto, sip, dip, ip_id, off_bytes, mf, chunk, ihl, vlan_tag, pad):
    hlen = ihl * 4
    offw = (off_bytes >> 3) | (0x2000 if mf else 0)
    ip = bytearray(hlen)
    ip[0] = 0x40 | ihl
    ip[2:4] = (hlen + len(chunk)).to_bytes(2, "big")
    ip[4:6] = int(ip_id).to_bytes(2, "big")
    ip[6:8] = offw.to_bytes(2, "big")
    ip[8] = 64
    ip[9] = proto
    ip[12:16] = int(sip).to_bytes(4, "big")
    ip[16:20] = int(dip).to_bytes(4, "big")
    for k in range(20, hlen):
        ip[k] = 1   # NOP options
    l2 = bytes([2, 0x11, 0x22, 0x33, 0x44, 0x55, 2, 0x66, 0x77, 0x88, 0x99, 0xAA])
    l2 += b"\x81\x00\x00\x05\x08\x00" if vlan_tag else b"\x08\x00"
    return l2 + bytes(ip) + chunk + bytes(pad)


def make_fragment_stream(n_dgrams: int, seed: int = SEED + 7, n_hosts: int = 64, oversize: float = 0.02,
                         reorder: float = 0.15, dup: float = 0.04, lose: float = 0.04, overlap: float = 0.02,
                         not_frag: float = 0.01, jumbo: float = 0.02, max_l4: int = 4000, align: int = 4):
    """A deterministic stream of IPv4 fragments of n_dgrams datagrams (UDP / TCP-SYN / ICMP, 30 % VLAN, some IP
    options and Ethernet padding), with the ways real fragment streams go wrong: reordered chains, duplicates, lost
    fragments (never complete → aging), overlaps, frames too long for the 2 KB copy, datagrams too large for the
    8 KB reassembly buffer, and a few non-fragments.
    Fragments of one datagram stay near each other; datagrams interleave.  Returns (arena u8, off u64, len u32)."""
    rng = np.random.default_rng(seed)
    hosts = rng.integers(1, 2**32 - 1, size=n_hosts, dtype=np.uint64)
    frames, keys = [], []
    for d in range(n_dgrams):
        r = rng.random()
        proto = 17 if r < 0.6 else (6 if r < 0.95 else 1)
        sip, dip = hosts[rng.integers(n_hosts)], hosts[rng.integers(n_hosts)]
        ip_id = int(rng.integers(0, 65536))
        ihl = 5 if rng.random() < 0.9 else int(rng.integers(6, 8))
        vlan_tag = rng.random() < 0.3
        is_jumbo = rng.random() < jumbo
        l4n = int(rng.integers(16, max_l4)) if not is_jumbo else int(rng.integers(8150, 9000))
        if proto == 17:
            l4 = (int(rng.integers(1, 65536)).to_bytes(2, "big") + int(rng.integers(1, 65536)).to_bytes(2, "big") +
                  l4n.to_bytes(2, "big") + b"\0\0" + rng.integers(0, 256, l4n - 8, dtype=np.uint8).tobytes())
        elif proto == 6:
            l4 = (int(rng.integers(1, 65536)).to_bytes(2, "big") + int(rng.integers(1, 65536)).to_bytes(2, "big") +
                  b"\0\0\0\1\0\0\0\0\x50\x02\x04\x00\0\0\0\0" + rng.integers(0, 256, max(0, l4n - 20),
                                                                            dtype=np.uint8).tobytes())
        else:
            l4 = rng.integers(0, 256, l4n, dtype=np.uint8).tobytes()
        big = rng.random() < oversize
        step = 8 * int(rng.integers(32, 186)) if not big else 8 * int(rng.integers(256, 400))
        if is_jumbo:
            step = 1480
        chunks, o = [], 0
        while o < len(l4):
            c = l4[o:o + step]
            chunks.append((o, c, o + step < len(l4)))
            o += step
        if len(chunks) == 1:   # make it a fragment: a lone chunk with MF set, or split once
            if len(l4) > 8:
                cut = 8 * max(1, (len(l4) // 2) // 8)
                chunks = [(0, l4[:cut], True), (cut, l4[cut:], False)]
            else:
                chunks = [(0, l4, True)]
        if rng.random() < overlap and len(chunks) > 1:
            o2, c2, m2 = chunks[1]
            chunks[1] = (max(0, o2 - 8), l4[max(0, o2 - 8):o2 - 8 + len(c2)], m2)
        if rng.random() < lose and len(chunks) > 1:
            del chunks[int(rng.integers(len(chunks)))]
        if rng.random() < dup:
            chunks.insert(int(rng.integers(len(chunks) + 1)), chunks[int(rng.integers(len(chunks)))])
        if rng.random() < reorder:
            rng.shuffle(chunks)
        base = d + rng.random() * 3.0   # datagrams interleave; a chain keeps its (possibly perturbed) order
        for k, (o, c, mf) in enumerate(chunks):
            # Ethernet trailer padding counts in frag_len (L3 length = frame − L2): on a non-final fragment it
            # overlaps the next one (decode-defrag.c:384-391), so only final fragments carry it here
            pad = int(rng.integers(1, 12)) if (not mf and rng.random() < 0.05) else 0
            frames.append(_frag_frame(rng, proto, sip, dip, ip_id, o, mf, c, ihl, vlan_tag, pad))
            keys.append(base + 0.5 * k)
        if rng.random() < not_frag:
            frames.append(_frag_frame(rng, 17, sip, dip, ip_id, 0, False, l4[:64], 5, False, 0))
            keys.append(base + rng.random() * 3.0)
    order = np.argsort(np.asarray(keys), kind="stable")
    lens = np.array([len(frames[i]) for i in order], np.uint32)
    sizes = (lens.astype(np.uint64) + (align - 1)) // align * align
    off = np.zeros(len(order), np.uint64)
    off[1:] = np.cumsum(sizes)[:-1]
    arena = np.zeros(int(sizes.sum()) + 64, np.uint8)
    for j, i in enumerate(order):
        arena[int(off[j]):int(off[j]) + int(lens[j])] = np.frombuffer(frames[i], np.uint8)
    return arena, off, lens
