"""`show packet statistic` / `show flow statistic` text: ppe_format_pkt_stat /
ppe_format_flow_stat against golden output generated from the reference's dp_show_pkt_stat / dp_show_flow_stat
(tests/golden/gen_stat_golden.py).  Pure host functions of libppe_hip.so: no GPU needed."""
import ctypes as C
from pathlib import Path

from ppe import abi

GOLDEN = Path(__file__).resolve().parent / "golden"


def test_pkt_stat_text_matches_reference_layout():
    lib = abi.load()
    cnt = abi.Counters()
    for i, name in enumerate(abi.COUNTERS):
        cnt.c[i] = 1000 + 17 * i  # the generator's counter vector
    n = lib.ppe_format_pkt_stat(C.byref(cnt), None, 0)
    buf = C.create_string_buffer(n + 1)
    assert lib.ppe_format_pkt_stat(C.byref(cnt), buf, n + 1) == n
    assert buf.value.decode() == (GOLDEN / "pkt_stat_v1.txt").read_text()
    small = C.create_string_buffer(40)  # truncation keeps snprintf semantics
    assert lib.ppe_format_pkt_stat(C.byref(cnt), small, 40) == n and len(small.value) == 39


def test_flow_stat_text():
    lib = abi.load()
    fi = abi.FlowInfo(live=5, new_flow=123456, del_flow=7890)
    buf = C.create_string_buffer(512)
    n = lib.ppe_format_flow_stat(C.byref(fi), buf, 512)
    assert buf.value.decode() == (GOLDEN / "flow_stat_v1.txt").read_text() and n == len(buf.value)


def _defrag_info():
    df = abi.DefragInfo()
    for k in range(9):
        df.st[k] = 501 + k  # the generator's reassembly vector (DF_COUNTS, st index = enum ppe_defrag_status)
    df.teardrop = 510
    df.new_fcb, df.del_fcb = 4242, 4141
    return df


def test_pkt_stat_text_with_reassembly_counters():
    """ip_frag_stat lines and the attack section's teardrop line from ppe_defrag_info, golden
    text generated from dp_show_pkt_stat with the STAT_FRAG_* / STAT_ATTACK_TEARDROP fields set."""
    lib = abi.load()
    cnt = abi.Counters()
    for i in range(len(abi.COUNTERS)):
        cnt.c[i] = 1000 + 17 * i
    df = _defrag_info()
    n = lib.ppe_format_pkt_stat_ex(C.byref(cnt), C.byref(df), 1, None, 0)
    buf = C.create_string_buffer(n + 1)
    assert lib.ppe_format_pkt_stat_ex(C.byref(cnt), C.byref(df), 1, buf, n + 1) == n
    assert buf.value.decode() == (GOLDEN / "pkt_stat_v2.txt").read_text()
    # teardrop monitor off (the reference's default attack configuration): the teardrop line stays 0
    lib.ppe_format_pkt_stat_ex(C.byref(cnt), C.byref(df), 0, buf, n + 1)
    assert "teardrop: 0\n" in buf.value.decode() and "reasm_ok: 502\n" in buf.value.decode()
    # no table: identical to the plain form
    lib.ppe_format_pkt_stat_ex(C.byref(cnt), None, 1, buf, n + 1)
    assert buf.value.decode() == (GOLDEN / "pkt_stat_v1.txt").read_text()


def test_flow_stat_text_with_fcb_counters():
    lib = abi.load()
    fi = abi.FlowInfo(live=5, new_flow=123456, del_flow=7890)
    df = _defrag_info()
    buf = C.create_string_buffer(512)
    n = lib.ppe_format_flow_stat_ex(C.byref(fi), C.byref(df), buf, 512)
    assert buf.value.decode() == (GOLDEN / "flow_stat_v2.txt").read_text() and n == len(buf.value)
