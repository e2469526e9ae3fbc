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
