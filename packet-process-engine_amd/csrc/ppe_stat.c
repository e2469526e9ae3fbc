/*
 * ppe_stat.c — the text of the reference's `show packet statistic` and `show flow statistic` commands
 * (dp_show_pkt_stat, dataplane/src/common/dp_cmd.c:844-1818; dp_show_flow_stat, :2346-2392), produced from this
 * engine's per-reason counters (ppe_counters_read) and flow-table totals (ppe_flow_info).
 *
 * Sections, line names and order follow the reference.  The ip_frag_stat lines, the attack section's teardrop line and
 * the flow text's fcb lines come from the IPv4 reassembly table (ppe_defrag_info) when one is given to the _ex forms:
 * fragments per Defrag outcome are exactly the STAT_FRAG_* increments of decode-defrag.c (cache_ok :391, reasm_ok
 * :279, setup_err :282, fcb_full :80, hw2sw_err :418, cache_full :437, defrag_err :401; fcb_no :87 is a memory-pool
 * failure the device table cannot have, out_oversize is commented out at :285), new / del fcb are :481 / :526, and
 * teardrop is counted only while the teardrop monitor is enabled (DP_Teardrop_Attack_Monitor, dataplane/src/attack/
 * dp_attack.c:487-498; disabled in the default configuration).  Lines whose counter has no source on the GPU path
 * print 0: the receive-error / from-linux / address counters of the Octeon I/O layer, ARP / ICMP / OSPF hand-offs to
 * Linux, TX, the other attack monitors (pass-through at default configuration), and output_* (the reference's
 * SELF_TEST build forwards without STAT_OUTPUT_*, flow.c:21,376-377).
 */
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include "ppe_hip.h"

#define NONE (-1)
/* reassembly-table sources (ppe_defrag_info_t), printed 0 without one */
#define DF(st) (1000 + (st))   /* fragments with Defrag outcome st */
#define DF_TEARDROP 2000       /* overlaps, while the teardrop monitor is enabled */

typedef struct {
    const char *name;  /* printed as "<name>: %ld" */
    int counter;       /* enum ppe_counter, or NONE */
} stat_line_t;

typedef struct {
    const char *title;
    const stat_line_t *lines;
    int n;
    int blank_after;   /* the reference prints an empty line after most sections */
} stat_section_t;

/* dp_cmd.c:866-917 */
static const stat_line_t k_recv[] = {{"recv_packet_count", PPE_C_PKTS}, {"recv_packet_bytes", PPE_C_RX_BYTES},
                                     {"recv_packet_count_sum", PPE_C_PKTS}, {"recv_packet_bytes_sum", PPE_C_RX_BYTES}};
/* :923-992 (oct-rxtx.c:160-222: every packet here arrived through a hardware port) */
static const stat_line_t k_rx[] = {{"grp_err", NONE},          {"rx_fromhwport_err", NONE}, {"rx_fromlinux_err", NONE},
                                   {"rx_fromhwport_ok", PPE_C_PKTS}, {"rx_fromlinux_ok", NONE}, {"addr_err", NONE}};
static const stat_line_t k_ether[] = {{"headerlen_err", PPE_C_L2_HEADERLEN_ERR}, {"unsupport", PPE_C_L2_UNSUPPORT},
                                      {"rx_ok", PPE_C_L2_RX_OK}, {"arp_se2linux_ok", NONE},
                                      {"arp_se2linux_fail", NONE}};
static const stat_line_t k_vlan[] = {{"headerlen_err", PPE_C_VLAN_HEADERLEN_ERR},
                                     {"vlanlayer_exceed", PPE_C_VLAN_LAYER_EXCEED},
                                     {"unsupport", PPE_C_VLAN_UNSUPPORT}, {"rx_ok", PPE_C_VLAN_RX_OK},
                                     {"arp_se2linux_fail", NONE}, {"arp_se2linux_ok", NONE}};
static const stat_line_t k_ipv4[] = {{"headerlen_err", PPE_C_IPV4_HEADERLEN_ERR}, {"version_err", PPE_C_IPV4_VERSION_ERR},
                                     {"pktlen_err", PPE_C_IPV4_PKTLEN_ERR},     {"unsupport", PPE_C_IPV4_UNSUPPORT},
                                     {"rx_ok", PPE_C_IPV4_RX_OK},               {"icmp_se2linux_ok", NONE},
                                     {"icmp_se2linux_fail", NONE},              {"ospf_se2linux_ok", NONE},
                                     {"ospf_se2linux_fail", NONE}};
static const stat_line_t k_frag[] = {{"fraglen_err", PPE_C_FRAG_FRAGLEN_ERR}, {"fcb_no", NONE},
                                     {"hw2sw_err", DF(PPE_DF_HW2SW_ERR)}, {"fcb_full", DF(PPE_DF_FCB_FULL)},
                                     {"cache_full", DF(PPE_DF_CACHE_FULL)}, {"defrag_err", DF(PPE_DF_DEFRAG_ERR)},
                                     {"setup_err", DF(PPE_DF_SETUP_ERR)}, {"out_oversize", NONE},
                                     {"cache_ok", DF(PPE_DF_CACHED)}, {"reasm_ok", DF(PPE_DF_REASM)}};
static const stat_line_t k_icmp[] = {{"rx_ok", NONE}, {"drop", NONE}};
static const stat_line_t k_tcp[] = {{"headerlen_err", PPE_C_TCP_HEADERLEN_ERR}, {"pktlen_err", PPE_C_TCP_PKTLEN_ERR},
                                    {"rx_ok", PPE_C_TCP_RX_OK}};
static const stat_line_t k_udp[] = {{"headerlen_err", PPE_C_UDP_HEADERLEN_ERR}, {"pktlen_err", PPE_C_UDP_PKTLEN_ERR},
                                    {"rx_ok", PPE_C_UDP_RX_OK}};
static const stat_line_t k_acl[] = {{"drop", PPE_C_ACL_DROP}, {"fw", PPE_C_ACL_FW}};
static const stat_line_t k_flow[] = {{"node_nomem", PPE_C_FLOW_NODE_NOMEM}, {"proc_ok", PPE_C_FLOW_PROC_OK},
                                     {"proc_fail", PPE_C_FLOW_PROC_FAIL}, {"proc_drop", NONE},
                                     {"tcp_no_syn_first", PPE_C_FLOW_TCP_NO_SYN_FIRST}};
static const stat_line_t k_out[] = {{"output_fw", NONE}, {"output_drop", NONE}, {"output_cache", NONE},
                                    {"output_unsupport", NONE}};
static const stat_line_t k_tx[] = {{"port_err", NONE}, {"hw_send_err", NONE}, {"sw_desc_err", NONE},
                                   {"sw_send_err", NONE}, {"send_over", NONE}};
static const stat_line_t k_att[] = {{"land_drop", NONE}, {"teardrop", DF_TEARDROP}, {"pingdeath", NONE},
                                    {"ping flood drop", NONE}, {"udp flood drop", NONE}, {"syn flood drop", NONE},
                                    {"syncount", NONE}, {"portscan_drop", NONE}};

#define SEC(t, a, b) {t, a, (int)(sizeof a / sizeof a[0]), b}
static const stat_section_t k_sections[] = {
    SEC("recv_count", k_recv, 1), SEC("rx_stat", k_rx, 1),     SEC("ether_stat", k_ether, 1),
    SEC("vlan_stat", k_vlan, 1),  SEC("ipv4_stat", k_ipv4, 1), SEC("ip_frag_stat", k_frag, 1),
    SEC("icmp_stat", k_icmp, 1),  SEC("tcp_stat", k_tcp, 1),   SEC("udp_stat", k_udp, 1),
    SEC("acl_stat", k_acl, 1),    SEC("flow_stat", k_flow, 1), SEC("output", k_out, 0),
    SEC("tx_stat", k_tx, 0),      SEC("attack stat", k_att, 1),
};

typedef struct {
    char *buf;
    size_t cap, len;
} out_t;

static void put(out_t *o, const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    const size_t room = o->len < o->cap ? o->cap - o->len : 0;
    const int k = vsnprintf(o->buf ? o->buf + o->len : NULL, o->buf ? room : 0, fmt, ap);
    va_end(ap);
    if (k > 0) o->len += (size_t)k;
}

static long line_value(const ppe_counters_t *c, const ppe_defrag_info_t *df, int teardrop_monitor, int ci) {
    if (ci == NONE) return 0L;
    if (ci == DF_TEARDROP) return df && teardrop_monitor ? (long)df->teardrop : 0L;
    if (ci >= 1000) return df ? (long)df->st[ci - 1000] : 0L;
    return (long)c->c[ci];
}

int ppe_format_pkt_stat(const ppe_counters_t *c, char *buf, size_t cap) {
    return ppe_format_pkt_stat_ex(c, NULL, 0, buf, cap);
}

int ppe_format_pkt_stat_ex(const ppe_counters_t *c, const ppe_defrag_info_t *df, int teardrop_monitor, char *buf,
                           size_t cap) {
    if (!c) return PPE_EINVAL;
    out_t o = {buf, buf ? cap : 0, 0};
    if (buf && cap) buf[0] = 0;
    put(&o, "packet statistic:\n");
    put(&o, "----------------------------------\n");
    put(&o, "\n");
    for (size_t s = 0; s < sizeof k_sections / sizeof k_sections[0]; s++) {
        const stat_section_t *sec = &k_sections[s];
        put(&o, "%s:\n", sec->title);
        put(&o, "----------------\n");
        for (int i = 0; i < sec->n; i++) {
            const int ci = sec->lines[i].counter;
            put(&o, "%s: %ld\n", sec->lines[i].name, line_value(c, df, teardrop_monitor, ci));
        }
        put(&o, "----------------\n");
        if (sec->blank_after) put(&o, "\n");
    }
    return (int)o.len;
}

int ppe_format_flow_stat(const ppe_flow_info_t *f, char *buf, size_t cap) {
    return ppe_format_flow_stat_ex(f, NULL, buf, cap);
}

int ppe_format_flow_stat_ex(const ppe_flow_info_t *f, const ppe_defrag_info_t *df, char *buf, size_t cap) {
    if (!f) return PPE_EINVAL;
    out_t o = {buf, buf ? cap : 0, 0};
    if (buf && cap) buf[0] = 0;
    put(&o, "new flow is: %ld\ndel flow is: %ld\n", (long)f->new_flow, (long)f->del_flow);
    /* FCBs created / freed by the reassembly table (new_fcb / del_fcb, decode-defrag.c:15-16,481,526) */
    put(&o, "new fcb is: %ld\ndel fcb is: %ld\n", df ? (long)df->new_fcb : 0L, df ? (long)df->del_fcb : 0L);
    put(&o, "new pcb is: %ld\ndel pcb is: %ld\n", 0L, 0L);
    return (int)o.len;
}
