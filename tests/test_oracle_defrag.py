"""Known answers for the oracle's IPv4 reassembly (oracle/ppe_oracle_defrag.c), derived by hand from
dataplane/src/decode/decode-defrag.c — the reference ships no defrag tests or fixtures and its defrag cannot be built
here (Cavium SDK / mem_pool / hlist headers), so these answers are what pins the restatement (parity unpinned by
reference outputs).  Each test names the reference lines it exercises."""
import struct

import numpy as np
import pytest

from pktbuild import arena, ip_checksum_ok, ip_frag, udp, tcp, udp_packet
import pyoracle

S, D = 0x0A000001, 0x0A000002
DF = dict(CACHED=0, REASM=1, SETUP_ERR=2, FCB_FULL=3, HW2SW_ERR=4, DELETED=5, CACHE_FULL=6, DEFRAG_ERR=7,
          NOT_FRAG=8)
TEAR = 0x100


def run(d, frames, now=100, ids=None):
    a, o, l = arena(frames)
    return d.batch(a, o, l, now=now, ids=ids)


def udp_l4(n=40, sport=1234, dport=80):
    return udp(sport, dport, bytes(range(n - 8)))


def test_in_order_reassembly_matches_unfragmented():
    """Frag_defrag_process append path (:329-334), completion (:371-376), Frag_defrag_reasm (:222-289)."""
    l4 = udp_l4(40)
    frames = [ip_frag(17, S, D, 7, 0, True, l4[:16]), ip_frag(17, S, D, 7, 16, True, l4[16:32]),
              ip_frag(17, S, D, 7, 32, False, l4[32:])]
    d = pyoracle.OracleDefrag()
    r = run(d, frames, ids=np.array([10, 11, 12], np.uint64))
    assert list(r["status"]) == [DF["CACHED"], DF["CACHED"], DF["REASM"]]
    assert r["n_dgram"] == 1 and list(r["dgram_of"]) == [0xFFFFFFFF, 0xFFFFFFFF, 0]
    n = int(r["dgram_len"][0])
    got = bytes(r["dgram_pkt"][0, :n])
    # the unfragmented packet: same bytes except ip_id (kept from the head), and a valid recomputed checksum
    want = bytearray(udp_packet(S, D, 1234, 80, bytes(range(32))))
    want[18:20] = (7).to_bytes(2, "big")
    assert n == len(want) == 14 + 20 + 40
    assert got[:24] == bytes(want[:24]) and got[26:] == bytes(want[26:])
    assert ip_checksum_ok(got[14:34])
    assert list(r["dgram_frags"][0, :3]) == [10, 11, 12] and all(x == 2**64 - 1 for x in r["dgram_frags"][0, 3:])
    s = d.stats()
    assert (s["running"], s["new_fcb"], s["st_cached"], s["st_reasm"]) == (1, 1, 2, 1)


def test_two_fragments_reversed_complete():
    """Final first (:305-311), then offset 0: the scan (:344-349) stops at the final one (frag_len 8 >= 0)."""
    l4 = udp_l4(16)
    d = pyoracle.OracleDefrag()
    r = run(d, [ip_frag(17, S, D, 1, 8, False, l4[8:]), ip_frag(17, S, D, 1, 0, True, l4[:8])])
    assert list(r["status"]) == [DF["CACHED"], DF["REASM"]]
    n = int(r["dgram_len"][0])
    assert bytes(r["dgram_pkt"][0, 34:n]) == l4


def test_middle_fragment_last_is_a_teardrop_by_the_frag_len_scan():
    """The chain scan compares the chained fragment's frag_len with the new offset (:346): a middle fragment at
    offset 16 stops at the head (frag_len 16 >= 16) and is then 'overlapping' it (:388-391) → DEFRAG_ERR."""
    l4 = udp_l4(48)
    d = pyoracle.OracleDefrag()
    r = run(d, [ip_frag(17, S, D, 2, 0, True, l4[:16]), ip_frag(17, S, D, 2, 32, False, l4[32:]),
                ip_frag(17, S, D, 2, 16, True, l4[16:32])])
    assert list(r["status"]) == [DF["CACHED"], DF["CACHED"], DF["DEFRAG_ERR"] | TEAR]
    s = d.stats()
    assert s["teardrop"] == 1 and s["st_defrag_err"] == 1
    # the FCB keeps its two fragments until aging drops them (Frag_defrag_timeout :515-546)
    ids, freed = d.age(now=121, timeout=20)
    assert sorted(ids.tolist()) == [0, 1] and freed == 1
    assert d.stats()["timeout_drop"] == 2 and d.stats()["running"] == 0


def test_duplicate_is_teardrop():
    l4 = udp_l4(32)
    d = pyoracle.OracleDefrag()
    r = run(d, [ip_frag(17, S, D, 3, 0, True, l4[:16]), ip_frag(17, S, D, 3, 0, True, l4[:16])])
    assert list(r["status"]) == [DF["CACHED"], DF["DEFRAG_ERR"] | TEAR]


def test_short_final_and_second_final_are_errors():
    """Final fragment ending before total (:305-306), and a second final (:305, LAST_IN)."""
    l4 = udp_l4(48)
    d = pyoracle.OracleDefrag()
    r = run(d, [ip_frag(17, S, D, 4, 0, True, l4[:32]), ip_frag(17, S, D, 4, 16, False, l4[16:24]),
                ip_frag(17, S, D, 5, 32, False, l4[32:]), ip_frag(17, S, D, 5, 40, False, l4[40:])])
    assert list(r["status"]) == [DF["CACHED"], DF["DEFRAG_ERR"], DF["CACHED"], DF["DEFRAG_ERR"]]


def test_non_final_extends_total_even_when_rejected():
    """:313-320 raise total_fraglen before the overlap checks; a rejected fragment leaves it raised, so the chain
    can no longer complete at the original length."""
    l4 = udp_l4(32)
    d = pyoracle.OracleDefrag()
    r = run(d, [ip_frag(17, S, D, 6, 0, True, l4[:16]),
                ip_frag(17, S, D, 6, 8, True, bytes(32)),          # overlaps the head, end 40 > total → total 40
                ip_frag(17, S, D, 6, 16, False, l4[16:])])         # final, end 32 < total 40 → error
    assert list(r["status"]) == [DF["CACHED"], DF["DEFRAG_ERR"] | TEAR, DF["DEFRAG_ERR"]]


def test_cache_full():
    """cache_num >= defrag_cache_max (:429-437)."""
    d = pyoracle.OracleDefrag(cache_max=2)
    r = run(d, [ip_frag(17, S, D, 8, 0, True, bytes(8)), ip_frag(17, S, D, 8, 16, True, bytes(8)),
                ip_frag(17, S, D, 8, 32, True, bytes(8))])
    assert list(r["status"]) == [DF["CACHED"], DF["CACHED"], DF["CACHE_FULL"]]


def test_fcb_full_and_recovery_after_aging():
    """fcb_create's cap (:74-82): the third key fails, also on its later fragments; aging frees a slot."""
    d = pyoracle.OracleDefrag(fcb_max=2)
    r = run(d, [ip_frag(17, S, D, 1, 0, True, bytes(8)), ip_frag(17, S, D, 2, 0, True, bytes(8)),
                ip_frag(17, S, D, 3, 0, True, bytes(8)), ip_frag(17, S, D, 3, 8, False, bytes(8))], now=100)
    assert list(r["status"]) == [DF["CACHED"], DF["CACHED"], DF["FCB_FULL"], DF["FCB_FULL"]]
    run(d, [ip_frag(17, S, D, 2, 8, True, bytes(8))], now=110)     # refreshes FCB 2's timestamp
    ids, freed = d.age(now=121, timeout=20)                          # FCB 1 idle 21 s > 20
    assert sorted(ids.tolist()) == [0] and freed == 1
    r = run(d, [ip_frag(17, S, D, 3, 0, True, bytes(8))], now=121)
    assert list(r["status"]) == [DF["CACHED"]]


def test_hw2sw_error_still_creates_the_fcb():
    """Defrag creates the FCB before PACKET_HW2SW fails for a frame > 2024 B (:462-470, 415-420)."""
    d = pyoracle.OracleDefrag()
    r = run(d, [ip_frag(17, S, D, 9, 0, True, bytes(2024 - 34 + 1 - 7 + 7))])   # frame 2025 B
    assert list(r["status"]) == [DF["HW2SW_ERR"]]
    assert d.stats()["running"] == 1


def test_deleted_until_aged_then_new_fcb():
    """A completed FCB is DELETE until the timer frees it (:278-279, 422-427, 515-520)."""
    l4 = udp_l4(16)
    d = pyoracle.OracleDefrag()
    frames = [ip_frag(17, S, D, 1, 0, True, l4[:8]), ip_frag(17, S, D, 1, 8, False, l4[8:])]
    r = run(d, frames + [frames[0]])
    assert list(r["status"]) == [DF["CACHED"], DF["REASM"], DF["DELETED"]]
    ids, freed = d.age(now=100, timeout=20)      # DELETE: freed at the next tick, nothing to drop
    assert len(ids) == 0 and freed == 1
    r = run(d, frames)
    assert list(r["status"]) == [DF["CACHED"], DF["REASM"]]


def test_setup_error_keeps_chain():
    """MEM_8K_ALLOC(total + L2 + ihl*4) fails (:173-183): STAT_FRAG_SETUP_ERR, the chain stays until aging."""
    d = pyoracle.OracleDefrag(reasm_buf=49)   # needs 16 + 14 + 20 = 50
    l4 = udp_l4(16)
    r = run(d, [ip_frag(17, S, D, 1, 0, True, l4[:8]), ip_frag(17, S, D, 1, 8, False, l4[8:])])
    assert list(r["status"]) == [DF["CACHED"], DF["SETUP_ERR"]]
    assert r["n_dgram"] == 0
    ids, _ = d.age(now=200, timeout=20)
    assert sorted(ids.tolist()) == [0, 1]


def test_icmp_keeps_head_frame_only():
    """ICMP: 1000-B buffer, the head frame copied, pkt_totallen summed, ip_off = 0, no ip_len / checksum (:250-265)."""
    d = pyoracle.OracleDefrag()
    p1, p2 = bytes(range(16)), bytes(range(100, 116))
    r = run(d, [ip_frag(1, S, D, 1, 0, True, p1), ip_frag(1, S, D, 1, 16, False, p2)])
    assert list(r["status"]) == [DF["CACHED"], DF["REASM"]]
    n = int(r["dgram_len"][0])
    assert n == 14 + 20 + 16 + 16
    got = bytes(r["dgram_pkt"][0, :n])
    head = ip_frag(1, S, D, 1, 0, True, p1)
    assert got[:20] == head[:20] and got[20:22] == b"\0\0" and got[22:len(head)] == head[22:]
    assert got[len(head):] == bytes(16)


def test_vlan_options_padding_and_proto_blind_match():
    """VLAN frame, IP options (ihl 6), a padded final fragment (frag_len counts the padding), and ip4_frag_match
    ignoring the protocol (:115-121)."""
    l4 = tcp(1000, 2000, 0x02, payload=bytes(12))   # 32 B
    d = pyoracle.OracleDefrag()
    r = run(d, [ip_frag(6, S, D, 5, 0, True, l4[:16], ihl=6, vlan_tag=True),
                ip_frag(17, S, D, 5, 16, False, l4[16:], ihl=6, vlan_tag=True, pad=4)])
    assert list(r["status"]) == [DF["CACHED"], DF["REASM"]]
    n = int(r["dgram_len"][0])
    got = bytes(r["dgram_pkt"][0, :n])
    assert n == 18 + 24 + 32 + 4
    assert struct.unpack(">H", got[20:22])[0] == 24 + 36      # ip_len = ihl*4 + total (padding included)
    assert ip_checksum_ok(got[18:42])
    assert got[42:74] == l4


def test_not_a_fragment():
    d = pyoracle.OracleDefrag()
    r = run(d, [udp_packet(), b"\0" * 10])
    assert list(r["status"]) == [DF["NOT_FRAG"], DF["NOT_FRAG"]]
    assert d.stats()["running"] == 0


def test_age_keeps_fresh_and_equal_time():
    """now > cycle && now - cycle > timeout (:515-517): exactly 20 s idle is kept."""
    d = pyoracle.OracleDefrag()
    run(d, [ip_frag(17, S, D, 1, 0, True, bytes(8))], now=100)
    assert d.age(now=120, timeout=20)[1] == 0
    assert d.age(now=99, timeout=0)[1] == 0
    assert d.age(now=121, timeout=20)[1] == 1


@pytest.mark.parametrize("seed", [1, 2])
def test_stream_statistics_are_consistent(seed):
    """Property over a synthetic stream: every fragment gets one status, counters add up, datagram count =
    REASM count, reassembled UDP/TCP datagrams carry a valid header checksum."""
    from ppe import synth
    a, o, l = synth.make_fragment_stream(400, seed=seed)
    d = pyoracle.OracleDefrag()
    tot = np.zeros(9, np.int64)
    for b in range(0, len(l), 512):
        r = d.batch(a, o[b:b + 512], l[b:b + 512], now=100 + b // 512)
        st = r["status"] & 0xFF
        tot += np.bincount(st, minlength=9)
        assert r["n_dgram"] == int((st == DF["REASM"]).sum())
        for j in range(r["n_dgram"]):
            f = bytes(r["dgram_pkt"][j, :r["dgram_len"][j]])
            l2 = 18 if f[12:14] == b"\x81\x00" else 14
            if f[l2 + 9] != 1:
                assert ip_checksum_ok(f[l2:l2 + (f[l2] & 15) * 4])
        d.age(100 + b // 512, 20)
    s = d.stats()
    assert [s["st_" + k.lower()] for k in DF] == tot.tolist()
    assert s["new_fcb"] - s["del_fcb"] == s["running"]
