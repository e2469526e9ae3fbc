"""Tiny explicit packet builder for known-answer tests (bytes laid out exactly as on the wire, big-endian)."""
import struct

DMAC = bytes([0x02, 0x11, 0x22, 0x33, 0x44, 0x55])
SMAC = bytes([0x02, 0x66, 0x77, 0x88, 0x99, 0xAA])


def eth(etype, dmac=DMAC, smac=SMAC):
    return dmac + smac + struct.pack(">H", etype)


def vlan(inner, tci=5):
    return struct.pack(">HH", tci, inner)


def ipv4(proto, sip, dip, payload_len, ihl=5, ver=4, ip_len=None, off=0, opts=b""):
    hlen = ihl * 4
    if ip_len is None:
        ip_len = hlen + payload_len
    h = struct.pack(">BBHHHBBHII", (ver << 4) | ihl, 0, ip_len, 0x1234, off, 64, proto, 0, sip, dip)
    return h + opts.ljust(hlen - 20, b"\x01")[: max(0, hlen - 20)]


def udp(sport, dport, payload=b"", ulen=None):
    if ulen is None:
        ulen = 8 + len(payload)
    return struct.pack(">HHHH", sport, dport, ulen, 0) + payload


def tcp(sport, dport, flags=0x02, off=5, opts=b"", payload=b""):
    hdr = struct.pack(">HHIIBBHHH", sport, dport, 1, 0, (off << 4), flags, 1024, 0, 0)
    return hdr + opts + payload


def udp_packet(sip=0x0A000001, dip=0x0A000002, sport=1234, dport=80, payload=b"\0" * 22, vlan_tag=False):
    l4 = udp(sport, dport, payload)
    l3 = ipv4(17, sip, dip, len(l4)) + l4
    return (eth(0x8100) + vlan(0x0800) if vlan_tag else eth(0x0800)) + l3


def tcp_packet(sip=0xC0A80101, dip=0xC0A80102, sport=12345, dport=443, flags=0x02, vlan_tag=False, payload=b""):
    l4 = tcp(sport, dport, flags, payload=payload)
    l3 = ipv4(6, sip, dip, len(l4)) + l4
    return (eth(0x8100) + vlan(0x0800) if vlan_tag else eth(0x0800)) + l3


def ip_frag(proto, sip, dip, ip_id, off_bytes, mf, chunk, ihl=5, vlan_tag=False, pad=0):
    """One IPv4 fragment frame: fragment offset off_bytes (a multiple of 8), MF flag, payload chunk."""
    hlen = ihl * 4
    offw = (off_bytes >> 3) | (0x2000 if mf else 0)
    h = struct.pack(">BBHHHBBHII", 0x40 | ihl, 0, hlen + len(chunk), ip_id, offw, 64, proto, 0, sip, dip)
    h += b"\x01" * (hlen - 20)
    l2 = eth(0x8100) + vlan(0x0800) if vlan_tag else eth(0x0800)
    return l2 + h + chunk + b"\0" * pad


def arena(frames, align=4):
    """Pack frames into one byte arena: (arena u8, off u64, len u32)."""
    import numpy as np
    off, buf = [], bytearray()
    for f in frames:
        off.append(len(buf))
        buf += f
        buf += b"\0" * ((-len(buf)) % align)
    buf += b"\0" * 64
    return (np.frombuffer(bytes(buf), np.uint8).copy(), np.array(off, np.uint64),
            np.array([len(f) for f in frames], np.uint32))


def ip_checksum_ok(ip_header: bytes) -> bool:
    s = sum(struct.unpack(">%dH" % (len(ip_header) // 2), ip_header))
    while s >> 16:
        s = (s & 0xFFFF) + (s >> 16)
    return s == 0xFFFF
