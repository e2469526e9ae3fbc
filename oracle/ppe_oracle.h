/*
 * ppe_oracle.h — TEST INFRASTRUCTURE ONLY.  CPU restatement of the reference's per-packet decode → flow hash →
 * ACL path, used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as the checker.  The product
 * (libppe_hip.so) never links, loads or calls it.
 *
 * Pinning:
 *   - flow hash: checked against the reference's own dataplane/src/flow/tluhash.h compiled unmodified into
 *     oracle/_ref/libref_tluhash.so (tests/test_oracle_ref.py) and the two known answers of SURVEY.md §8(a) A9;
 *   - decode: the reference decoders cannot be built here without stand-ins for the Cavium SDK headers they
 *     include (cvmx*.h via mbuf.h / oct-common.h), which this task forbids, so decode is pinned by hand-derived
 *     known-answer packets, one per reason, each citing the reference line it exercises (tests/test_oracle_kat.py);
 *   - ACL: the reference engine source is absent (dataplane/src/acl/acl.mk:13-15 builds files not in the tree):
 *     PARITY UNPINNED by reference code; the semantics are the build's definition, frozen by
 *     tests/golden/ fixtures and hand-written known answers.
 */
#ifndef PPE_ORACLE_H
#define PPE_ORACLE_H

#include <stdint.h>
#include "ppe_acl.h"
#include "ppe_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    uint32_t unsupport_proto_action; /* 0 drop, 1 fw */
    uint32_t syn_check;
    uint64_t now_seconds;            /* packet timestamp when ts == NULL */
} oracle_cfg_t;

typedef struct {
    uint32_t status;     /* enum ppe_status */
    uint32_t action;     /* enum ppe_action */
    uint32_t flags;      /* PPE_F_* */
    uint32_t flow_hash;  /* flow_hashfn, 0 unless PPE_F_L4 */
    int32_t acl_hit;     /* -1 unless a rule matched */
    uint32_t sip, dip, sport, dport, proto, paylen;
    uint32_t counters;   /* bit i set = counter i (enum ppe_counter) incremented once */
    uint32_t reach;      /* 1 + highest frame byte offset the verdict depends on */
    uint32_t tcp_ws;     /* byte offset (from the TCP header) of the window-scale option DecodeTCPOptions recorded
                            (m->tcpvars.ws, decode-tcp.c:61-70), 0 = none; no verdict effect */
    /* the mbuf fields the reference's decoders write (dataplane/src/include/mbuf.h:23-87), for Decode()'s parity */
    uint32_t mset;       /* ORACLE_M_* bits: which of them this packet's decode wrote */
    uint32_t l3off, l4off, payoff;  /* frame offsets of network_header, transport_header, payload */
    uint32_t frag_id, frag_off, frag_len;  /* defrag_id, frag_offset, frag_len (decode-ipv4.c:107-109) */
    uint32_t opt_past;   /* 1: no window-scale option was found before the option parse needed a byte past the
                            available window (the reference reads the whole option space; ppe_hip.h
                            PPE_TUPLE_OPT_PAST) */
} oracle_result_t;

/* oracle_result_t.mset: mbuf fields written, with the reference line that writes them */
#define ORACLE_M_ETH   0x001u  /* ethh, eth_dst, eth_src            decode-ethernet.c:57,71-72 */
#define ORACLE_M_VLAN  0x002u  /* vlanh, vlan_idx = 1               decode-vlan.c:41,46 */
#define ORACLE_M_L3    0x004u  /* network_header                    decode-ipv4.c:42 */
#define ORACLE_M_IP    0x008u  /* ipv4.sip, ipv4.dip, proto         decode-ipv4.c:62-63,97 */
#define ORACLE_M_FRAG  0x010u  /* defrag_id, frag_offset, frag_len  decode-ipv4.c:107-109 */
#define ORACLE_M_L4H   0x020u  /* transport_header                  decode-udp.c:24, decode-tcp.c:146 */
#define ORACLE_M_L4    0x040u  /* sport, dport, payload, payload_len decode-udp.c:38-45, decode-tcp.c:179-187 */
#define ORACLE_M_WS    0x080u  /* tcpvars.ws = &TCP_OPTS[0]         decode-tcp.c:63-70 */
#define ORACLE_M_FLOW  0x100u  /* flags |= PKT_TO_SERVER|CLIENT, PKT_HAS_FLOW (flow.c:294-307: the flow exists) */

/* rule set used by oracle_classify (pointer kept; caller owns the memory) */
void oracle_set_rules(const RCP_BLOCK_ACL_RULE_TUPLE *rules, const uint8_t *used, uint32_t n,
                      uint32_t default_action);
/* optional: walk a classifier image (ppe_image.h) instead of the linear first-match scan */
void oracle_set_image(const uint32_t *img, uint32_t n_words);

uint32_t oracle_tluhash(uint32_t u1, uint32_t u2);
uint32_t oracle_flow_hashfn(uint32_t proto, uint32_t sip, uint32_t dip, uint32_t sport, uint32_t dport);

/* linear first-match ACL (A11): returns the lowest matching USED index or -1; *action = its action or default */
int32_t oracle_acl_linear(uint32_t sip, uint32_t dip, uint32_t sport, uint32_t dport, uint32_t proto,
                          const uint8_t *dmac, const uint8_t *smac, uint64_t ts, uint32_t *action);
/* decision-tree walk over the image set by oracle_set_image; same contract */
int32_t oracle_acl_tree(uint32_t sip, uint32_t dip, uint32_t sport, uint32_t dport, uint32_t proto,
                        const uint8_t *dmac, const uint8_t *smac, uint64_t ts, uint32_t *action);
int32_t oracle_acl_blocks(uint32_t sip, uint32_t dip, uint32_t sport, uint32_t dport, uint32_t proto,
                        const uint8_t *dmac, const uint8_t *smac, uint64_t ts, uint32_t *action);
/* lookup in the image's cut lists (v7; TCP / UDP keys); same contract */
int32_t oracle_acl_cut(uint32_t sip, uint32_t dip, uint32_t sport, uint32_t dport, uint32_t proto,
                       const uint8_t *dmac, const uint8_t *smac, uint64_t ts, uint32_t *action);

/* One packet.  pkt holds at least `avail` bytes of the frame; len is the wire length (pkt_totallen).
 * Bytes past `avail` read as 0 (the reach field says whether the verdict depended on them). */
void oracle_classify(const uint8_t *pkt, uint32_t avail, uint32_t len, uint64_t ts, const oracle_cfg_t *cfg,
                     oracle_result_t *out);

/* Batch over windows (n × stride bytes), optionally multi-threaded (run-to-completion shards like mainloop);
 * use_tree selects the image walk.  Any output pointer may be NULL.  Returns 0. */
/* Pin the batch's shard threads: thread t on cpus[t % n] (n = 0: unpinned, the default). */
int oracle_set_pin_cpus(const int *cpus, int n);
int oracle_classify_batch(const uint8_t *hdr, uint32_t stride, const uint32_t *len, const uint64_t *ts, uint32_t n,
                          const oracle_cfg_t *cfg, int nthreads, int use_tree, uint32_t *verdict,
                          uint32_t *flow_hash, int32_t *acl_hit, uint32_t *tuple, uint32_t *reach,
                          uint64_t *counters /* [32] */);

/* ---- flow table (dataplane/src/flow/flow.c): one core's chained table over a pool of `capacity` items ---- */
typedef struct oracle_flow oracle_flow_t;
oracle_flow_t *oracle_flow_create(uint32_t capacity);
void oracle_flow_destroy(oracle_flow_t *f);
/* FlowHandlePacket with the table for packets 0..n-1 in order; cfg->now_seconds is the batch time (the flows'
 * last-seen `cycle`).  Same outputs as oracle_classify_batch (tuple optional). */
int oracle_flow_classify_batch(oracle_flow_t *f, const uint8_t *hdr, uint32_t stride, const uint32_t *len,
                               const uint64_t *ts, uint32_t n, const oracle_cfg_t *cfg, int use_tree,
                               uint32_t *verdict, uint32_t *flow_hash, int32_t *acl_hit, uint32_t *tuple,
                               uint64_t *counters /* [32] */);
/* FlowAgeTimeoutCB: removes flows with now > cycle && now - cycle > timeout; returns the count */
uint64_t oracle_flow_age(oracle_flow_t *f, uint64_t now, uint64_t timeout);
/* live flows in bucket order (first `max` copied); returns the live count */
uint32_t oracle_flow_dump(const oracle_flow_t *f, ppe_flow_entry_t *out, uint32_t max);
void oracle_flow_stats(const oracle_flow_t *f, uint64_t *live, uint64_t *new_flow, uint64_t *del_flow);

/* ---- IPv4 reassembly (dataplane/src/decode/decode-defrag.c; ppe_oracle_defrag.c): one core's FCB table ---- */
typedef struct oracle_defrag oracle_defrag_t;
/* 0 → the reference defaults (1024 FCBs, 8 cached fragments, 2024-B / 8168-B buffers) */
oracle_defrag_t *oracle_defrag_create(uint32_t fcb_max, uint32_t cache_max, uint32_t frag_buf, uint32_t reasm_buf);
void oracle_defrag_destroy(oracle_defrag_t *d);
/* Defrag for frames 0..n-1 in order (frame i: pkt + off[i], len[i] bytes); status[i] = enum ppe_defrag_status
 * (| PPE_DF_TEARDROP); datagram j (completion order): dgram_pkt + j * reasm_buf (zero-filled), dgram_len[j],
 * dgram_frags[j * cache_max ..] (ids in chain order, ~0 pad); dgram_of[i] = j for the completing fragment, else ~0.
 * Output pointers other than status may be NULL.  Returns the datagram count. */
uint32_t oracle_defrag_batch(oracle_defrag_t *d, const uint8_t *pkt, const uint64_t *off, const uint32_t *len,
                             const uint64_t *ids, uint32_t n, uint64_t now, uint32_t *status, uint32_t *dgram_of,
                             uint8_t *dgram_pkt, uint32_t *dgram_len, uint64_t *dgram_frags);
/* Frag_defrag_timeout: returns the number of fragments dropped (first `max` ids copied), *n_freed = FCBs freed */
uint32_t oracle_defrag_age(oracle_defrag_t *d, uint64_t now, uint64_t timeout, uint64_t *dropped, uint32_t max,
                           uint32_t *n_freed);
/* out[5 + PPE_DF__COUNT]: running, new_fcb, del_fcb, st[PPE_DF__COUNT], teardrop, timeout_drop, datagrams */
void oracle_defrag_stats(const oracle_defrag_t *d, uint64_t *out);

#ifdef __cplusplus
}
#endif
#endif
