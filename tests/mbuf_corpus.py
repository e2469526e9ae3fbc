"""Frames for the mbuf-field parity tests (tests/test_oracle_mbuf.py, tests/test_gpu_mbuf.py): every path through
the reference's decoders that writes a different set of mbuf fields (dataplane/src/decode/decode-*.c), with VLAN
tags, IPv4 options and TCP option layouts placed so that headers and options run past 64 and 128 bytes.

Helper module, no tests."""
import struct

import numpy as np

from pktbuild import eth, ip_frag, ipv4, tcp, udp, vlan

# Linux SYN option layout (MSS, SACK-permitted, timestamps, NOP, window scale): 20 option bytes, the window-scale
# option at TCP header byte 37, i.e. frame byte 71 behind a plain Ethernet + 20-B IPv4 header
LINUX_SYN_OPTS = b"\x02\x04\x05\xb4" + b"\x04\x02" + b"\x08\x0a" + b"\x00\x01\x02\x03" + b"\x00\x00\x00\x00" + \
    b"\x01" + b"\x03\x03\x07"
OPT_PIECES = [b"\x01", b"\x00", b"\x02\x04\x05\xb4", b"\x03\x03\x07", b"\x04\x02", b"\x08\x0a" + b"\x11" * 8,
              b"\x03\x04\x01\x01", b"\x05\x0a" + b"\x22" * 8, b"\x03\x03\x0e"]


def _l2(rng, etype=0x0800, tags=None):
    if tags is None:
        tags = 1 if rng.random() < 0.35 else 0
    if tags == 0:
        return eth(etype)
    if tags == 1:
        return eth(0x8100 if rng.random() < 0.5 else 0x9100) + vlan(etype)
    return eth(0x8100) + vlan(0x8100) + vlan(etype)


def _ihl(rng):
    r = rng.random()
    return 5 if r < 0.6 else int(rng.integers(6, 16))


def _opts(rng, space):
    if rng.random() < 0.1:
        return bytes(rng.integers(0, 256, space, dtype=np.uint8))
    o = b""
    while len(o) < space:
        o += OPT_PIECES[int(rng.integers(0, len(OPT_PIECES)))]
    return o[:space]


def _ip(rng):
    return int(rng.integers(1, 1 << 32))


def frame(rng, kind):
    """One frame of the given kind (see KINDS)."""
    sip, dip = _ip(rng), _ip(rng)
    if kind == "udp":
        l4 = udp(int(rng.integers(0, 65536)), int(rng.integers(0, 65536)), bytes(int(rng.integers(0, 40))))
        return _l2(rng) + ipv4(17, sip, dip, len(l4), ihl=_ihl(rng)) + l4
    if kind == "tcp_linux_syn":
        l4 = tcp(int(rng.integers(1, 65536)), int(rng.integers(1, 65536)), 0x02, off=10, opts=LINUX_SYN_OPTS,
                 payload=bytes(int(rng.integers(0, 16))))
        return _l2(rng) + ipv4(6, sip, dip, len(l4), ihl=_ihl(rng)) + l4
    if kind == "tcp_opts":
        off = int(rng.integers(6, 16))
        flags = 0x02 if rng.random() < 0.7 else 0x10
        l4 = tcp(int(rng.integers(1, 65536)), int(rng.integers(1, 65536)), flags, off=off,
                 opts=_opts(rng, 4 * (off - 5)), payload=bytes(int(rng.integers(0, 8))))
        return _l2(rng) + ipv4(6, sip, dip, len(l4), ihl=_ihl(rng)) + l4
    if kind == "frag":
        proto = int(rng.choice([6, 17, 1, 47]))
        mf = rng.random() < 0.6
        offb = 8 * int(rng.integers(0, 400)) if (not mf or rng.random() < 0.5) else 0
        if not mf and offb == 0:
            offb = 8 * int(rng.integers(1, 400))
        chunk = bytes(8 * int(rng.integers(1, 12)))
        return ip_frag(proto, sip, dip, int(rng.integers(0, 65536)), offb, mf, chunk, ihl=_ihl(rng),
                       vlan_tag=rng.random() < 0.35, pad=int(rng.integers(0, 3)) * 4)
    if kind == "frag_len_err":  # a fragment with no payload: the frame ends with its IPv4 header
        return ip_frag(17, sip, dip, int(rng.integers(0, 65536)), 8 * int(rng.integers(0, 100)), True, b"",
                       ihl=_ihl(rng), vlan_tag=rng.random() < 0.35)
    if kind == "ospf_frag":  # OSPF fragments are not handed to Defrag (decode-ipv4.c:102): unsupported protocol
        return ip_frag(89, sip, dip, 7, 0, True, bytes(16), vlan_tag=rng.random() < 0.3)
    if kind == "udp_len_err":
        l4 = udp(1, 2, bytes(8), ulen=int(rng.choice([9, 15, 17, 30])))
        return _l2(rng) + ipv4(17, sip, dip, len(l4), ihl=_ihl(rng)) + l4
    if kind == "udp_hdr_err":
        l4 = bytes(int(rng.integers(0, 8)))
        return _l2(rng) + ipv4(17, sip, dip, len(l4), ihl=_ihl(rng)) + l4
    if kind == "tcp_len_err":
        off = int(rng.choice([0, 1, 4, 12, 15]))
        l4 = tcp(5, 6, 0x02, off=off) + bytes(int(rng.integers(0, 8)))
        return _l2(rng) + ipv4(6, sip, dip, len(l4), ihl=_ihl(rng)) + l4
    if kind == "tcp_hdr_err":
        l4 = bytes(int(rng.integers(0, 20)))
        return _l2(rng) + ipv4(6, sip, dip, len(l4), ihl=_ihl(rng)) + l4
    if kind == "tcp_nosyn":
        l4 = tcp(int(rng.integers(1, 65536)), 80, 0x10, off=8, opts=_opts(rng, 12))
        return _l2(rng) + ipv4(6, sip, dip, len(l4), ihl=_ihl(rng)) + l4
    if kind == "ip_unsupport":
        pl = bytes(int(rng.integers(0, 30)))
        return _l2(rng) + ipv4(int(rng.choice([1, 2, 47, 50, 132])), sip, dip, len(pl), ihl=_ihl(rng)) + pl
    if kind == "ip_version":
        pl = bytes(20)
        return _l2(rng) + ipv4(17, sip, dip, len(pl), ver=int(rng.choice([0, 5, 6, 15]))) + pl
    if kind == "ip_short":  # fewer than 20 bytes of IPv4 header
        return _l2(rng) + ipv4(17, sip, dip, 0)[: int(rng.integers(0, 20))]
    if kind == "ip_ihl_err":
        h = bytearray(ipv4(17, sip, dip, 8) + udp(1, 2))
        h[0] = 0x40 | int(rng.integers(0, 5))
        return eth(0x0800) + bytes(h)
    if kind == "ip_len_err":
        l4 = udp(1, 2, bytes(8))
        ip_len = int(rng.choice([10, 19, 200, 1500]))
        return _l2(rng) + ipv4(17, sip, dip, len(l4), ip_len=ip_len) + l4
    if kind == "l2_zero_mac":
        z = bytes(6)
        d, s = (z, bytes([2, 1, 2, 3, 4, 5])) if rng.random() < 0.5 else (bytes([2, 1, 2, 3, 4, 5]), z)
        l4 = udp(1, 2)
        return eth(0x0800, dmac=d, smac=s) + ipv4(17, sip, dip, len(l4)) + l4
    if kind == "l2_short":
        return (eth(0x0800) + bytes(4))[: int(rng.integers(0, 14))]
    if kind == "l2_unsupport":
        return eth(int(rng.choice([0x86DD, 0x0806, 0x88A8]))) + bytes(30)
    if kind == "vlan_unsupport":
        return eth(0x8100) + vlan(0x86DD) + bytes(30)
    if kind == "vlan_short":
        return eth(0x8100) + bytes(int(rng.integers(0, 4)))
    if kind == "vlan_double":
        l4 = udp(1, 2)
        return _l2(rng, tags=2) + ipv4(17, sip, dip, len(l4)) + l4
    if kind == "vlan_double_short":  # the second tag's own length check (decode-vlan.c:28-33, via the recursion)
        return eth(0x8100) + vlan(0x8100) + bytes(int(rng.integers(0, 4)))
    raise ValueError(kind)


KINDS = ["udp", "tcp_linux_syn", "tcp_opts", "frag", "frag_len_err", "ospf_frag", "udp_len_err", "udp_hdr_err",
         "tcp_len_err", "tcp_hdr_err", "tcp_nosyn", "ip_unsupport", "ip_version", "ip_short", "ip_ihl_err",
         "ip_len_err", "l2_zero_mac", "l2_short", "l2_unsupport", "vlan_unsupport", "vlan_short", "vlan_double",
         "vlan_double_short"]
WEIGHTS = {"udp": 6, "tcp_linux_syn": 5, "tcp_opts": 8, "frag": 8, "frag_len_err": 2, "tcp_nosyn": 2}


def corpus(n, seed):
    rng = np.random.default_rng(seed)
    w = np.array([WEIGHTS.get(k, 1) for k in KINDS], float)
    kinds = rng.choice(len(KINDS), n, p=w / w.sum())
    return [frame(rng, KINDS[k]) for k in kinds], [KINDS[k] for k in kinds]


def windows(frames, stride):
    hdr = np.zeros((len(frames), stride), np.uint8)
    lens = np.zeros(len(frames), np.uint32)
    for i, f in enumerate(frames):
        c = min(len(f), stride)
        hdr[i, :c] = np.frombuffer(f[:c], np.uint8)
        lens[i] = len(f)
    return hdr, lens


def be16(b, o):
    return struct.unpack_from(">H", b, o)[0]
