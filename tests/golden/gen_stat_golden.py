#!/usr/bin/env python3
"""Generate tests/golden/pkt_stat_v1.txt + flow_stat_v1.txt (engine counters only) and pkt_stat_v2.txt +
flow_stat_v2.txt (plus the IPv4 reassembly table's counters, teardrop monitor enabled): the text the reference's
`show packet statistic` / `show flow statistic` would print for a fixed counter vector.

Run in the build container (needs /root/reference): it walks dp_show_pkt_stat / dp_show_flow_stat in
dataplane/src/common/dp_cmd.c statement by statement — each `x += pktstat[i]-><field>` sum followed by its
`sprintf(ptr, "<fmt>", x)` — and evaluates them with the pktstat fields this engine counts (mapped below by field
name; every other field is 0).  Only the resulting output text is committed (a golden vector); the reference file
itself is not."""
import re
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT / "packet-process-engine_amd")]
from ppe.abi import COUNTERS  # noqa: E402

REF = Path("/root/reference/dataplane/src/common/dp_cmd.c")
OUT = Path(__file__).resolve().parent

# pktstat field → engine counter (decode-statistic.h names; oct-rxtx.c:212-222 counts every received packet)
FIELD = {
    "rc.recv_packet_count": "pkts", "rc.recv_packet_bytes": "rx_bytes", "rc.recv_packet_count_sum": "pkts",
    "rc.recv_packet_bytes_sum": "rx_bytes", "rxstat.rx_fromhwport_ok": "pkts",
    "l2stat.headerlen_err": "l2_headerlen_err", "l2stat.unsupport": "l2_unsupport", "l2stat.rx_ok": "l2_rx_ok",
    "vlanstat.headerlen_err": "vlan_headerlen_err", "vlanstat.vlanlayer_exceed": "vlan_layer_exceed",
    "vlanstat.unsupport": "vlan_unsupport", "vlanstat.rx_ok": "vlan_rx_ok",
    "ipv4stat.headerlen_err": "ipv4_headerlen_err", "ipv4stat.version_err": "ipv4_version_err",
    "ipv4stat.pktlen_err": "ipv4_pktlen_err", "ipv4stat.unsupport": "ipv4_unsupport", "ipv4stat.rx_ok": "ipv4_rx_ok",
    "fragstat.fraglen_err": "frag_fraglen_err",
    "tcpstat.headerlen_err": "tcp_headerlen_err", "tcpstat.pktlen_err": "tcp_pktlen_err", "tcpstat.rx_ok": "tcp_rx_ok",
    "udpstat.headerlen_err": "udp_headerlen_err", "udpstat.pktlen_err": "udp_pktlen_err", "udpstat.rx_ok": "udp_rx_ok",
    "aclstat.drop": "acl_drop", "aclstat.fw": "acl_fw",
    "flowstat.node_nomem": "flow_node_nomem", "flowstat.proc_ok": "flow_proc_ok",
    "flowstat.proc_fail": "flow_proc_fail", "flowstat.tcp_no_syn_first": "flow_tcp_no_syn_first",
}
COUNTS = {name: 1000 + 17 * i for i, name in enumerate(COUNTERS)}  # distinct values per counter
FLOW = {"new_flow": 123456, "del_flow": 7890}
# v2: the reassembly table's per-outcome fragment counts (ppe_defrag_info_t.st[], enum ppe_defrag_status) and
# teardrops, by the STAT_FRAG_* / STAT_ATTACK_TEARDROP site each outcome increments (decode-defrag.c)
DF_FIELD = {"fragstat.cache_ok": "st0", "fragstat.reasm_ok": "st1", "fragstat.setup_err": "st2",
            "fragstat.fcb_full": "st3", "fragstat.hw2sw_err": "st4", "fragstat.cache_full": "st6",
            "fragstat.defrag_err": "st7", "attstat.teardrop": "teardrop"}
DF_COUNTS = {"st0": 501, "st1": 502, "st2": 503, "st3": 504, "st4": 505, "st5": 506, "st6": 507, "st7": 508,
             "st8": 509, "teardrop": 510}
FCB = {"new_fcb": 4242, "del_fcb": 4141}


def body(src: str, name: str) -> str:
    i = src.index(f"void {name}()")
    j = src.index("\n}\n", i)
    return src[i:j]


PAT = re.compile(r'(?P<reset>\bx\s*=\s*0;)|x\s*\+=\s*pktstat\[i\]->(?P<field>[a-z_0-9.]+);'
                 r'|sprintf\(\(void \*\)ptr,\s*"(?P<fmt>(?:[^"\\]|\\.)*)"\s*(?P<arg>,\s*x)?\)')


def eval_show(text: str, defrag: bool = False) -> str:
    out, x = [], 0
    for m in PAT.finditer(text):
        if m.group("reset"):
            x = 0
        elif m.group("field"):
            f = m.group("field")
            if f in FIELD:
                x += COUNTS[FIELD[f]]
            elif defrag and f in DF_FIELD:
                x += DF_COUNTS[DF_FIELD[f]]
        else:
            fmt = m.group("fmt").replace("\\n", "\n").replace("%ld", "%d")
            out.append(fmt % x if m.group("arg") else fmt)
    return "".join(out)


def main():
    src = REF.read_text(errors="replace")
    (OUT / "pkt_stat_v1.txt").write_text(eval_show(body(src, "dp_show_pkt_stat")))
    fb = body(src, "dp_show_flow_stat")
    vals = {"new_flow": FLOW["new_flow"], "del_flow": FLOW["del_flow"]}
    lines = []
    for pre in ("flow", "fcb", "pcb"):  # new_flow / new_fcb / new_pcb blocks, in the order of the function
        assert f"new {pre} is: " in fb
    for kind, (n, d) in (("flow", (vals["new_flow"], vals["del_flow"])), ("fcb", (0, 0)), ("pcb", (0, 0))):
        lines.append(f"new {kind} is: {n}\ndel {kind} is: {d}\n")
    (OUT / "flow_stat_v1.txt").write_text("".join(lines))
    (OUT / "pkt_stat_v2.txt").write_text(eval_show(body(src, "dp_show_pkt_stat"), defrag=True))
    lines = []
    for kind, (n, d) in (("flow", (vals["new_flow"], vals["del_flow"])), ("fcb", (FCB["new_fcb"], FCB["del_fcb"])),
                         ("pcb", (0, 0))):
        lines.append(f"new {kind} is: {n}\ndel {kind} is: {d}\n")
    (OUT / "flow_stat_v2.txt").write_text("".join(lines))
    print("wrote", OUT / "pkt_stat_v1.txt", OUT / "flow_stat_v1.txt", OUT / "pkt_stat_v2.txt",
          OUT / "flow_stat_v2.txt")


if __name__ == "__main__":
    main()
