/*
 * ppe_hip.h — C ABI of the MI355X-native decode + 5-tuple ACL classify engine.
 *
 * One call classifies a whole batch of packets on the GPU: Ethernet → [one VLAN tag] → IPv4 → TCP|UDP header parse,
 * 5-tuple extraction, the symmetric TluHash flow hash and the first-match ACL lookup, with per-reason counters and
 * per-tile ballot-compacted FW/DROP index lists.  It replaces, for a whole batch at once, the reference's per-mbuf
 * hot path:
 *
 *   Decode(mbuf)                         dataplane/src/decode/decode.c:19-28
 *   └ DecodeEthernet / DecodeVLAN        dataplane/src/decode/decode-ethernet.c:23-115, decode-vlan.c:23-89
 *   └ DecodeIPV4 / DecodeIPV4Packet      dataplane/src/decode/decode-ipv4.c:27-247
 *   └ DecodeUDP / DecodeTCP              dataplane/src/decode/decode-udp.c:16-71, decode-tcp.c:135-222
 *   └ FlowHandlePacket → flow_hashfn     dataplane/src/flow/flow.c:181-245,271-292, flow/tluhash.h:7-35
 *     └ (first packet) syn_check, DP_Acl_Lookup   dataplane/src/flow/flow.c:204-243
 *
 * Stateless semantics: every packet is treated as the first packet of its flow (flow-table miss), which is the
 * reference behaviour for the unique-flow inputs of the benchmark configs.  Fragments and
 * packets whose headers extend past the header window are PUNTed to the host (status PPE_ST_FRAG /
 * PPE_ST_WINDOW_PUNT); the reference hands fragments to Defrag (decode-ipv4.c:216-239), out of scope here.
 *
 * All pointers in ppe_batch_t / ppe_result_t passed to ppe_classify() are DEVICE pointers (hipMalloc / torch
 * cuda tensors) on the context's device.  ppe_classify_host() takes host pointers and runs the pipelined
 * H2D → classify → D2H path.  Functions return 0 or a negative errno-style code (PPE_E*).
 * Thread-compatible per context: one host thread per context (as one run-to-completion core per mainloop).
 */
#ifndef PPE_HIP_H
#define PPE_HIP_H

#include <stddef.h>
#include <stdint.h>
#include "ppe_acl.h"

#ifdef __cplusplus
extern "C" {
#endif

/* 2: ppe_tuning_t grew to 20 B (batches_per_launch) and mbuf_t (ppe_decode.h) took the reference's field layout;
 * 3: ppe_tuple's word 3 carries the TCP window-scale option offset (bits 9-15); 4: ppe_result_t.part8;
 * 5: the tuple carries a fragment's Defrag fields and the option-past-the-window bit; strides 64..256;
 * 6: ppe_acl_stats_t cut fields; 7: ppe_rules_stage / _publish; 8: ppe_result_t.packed (8-B verdict + flow hash +
 * ACL hit) */
#define PPE_ABI_VERSION 8

/* error codes (negative return values) */
#define PPE_OK       0
#define PPE_EINVAL  (-22)
#define PPE_ENOMEM  (-12)
#define PPE_ENODEV  (-19)
#define PPE_EIO     (-5)
#define PPE_ENOTSUP (-95)

/* ---- per-packet verdict word: status (bits 0-7) | action (bits 8-15) | flags (bits 16-31) ---- */
/* status = the terminal reason, one per reference drop/ok reason (dataplane/src/decode/decode-statistic.h:239-327) */
enum ppe_status {
    PPE_ST_ACL_FW = 0,            /* ACL passed (hit with action FW, or default FW)      STAT_ACL_FW        flow.c:240   */
    PPE_ST_ACL_DROP = 1,          /* ACL drop                                             STAT_ACL_DROP      flow.c:234   */
    PPE_ST_L2_HEADER_ERR = 2,     /* len<14, or all-zero dst/src MAC                      decode-ethernet.c:29-54      */
    PPE_ST_L2_UNSUPPORT = 3,      /* ethertype not 0x0800/0x8100/0x9100                   decode-ethernet.c:102-111    */
    PPE_ST_VLAN_HEADER_ERR = 4,   /* len<4 at a VLAN tag                                  decode-vlan.c:28-33          */
    PPE_ST_VLAN_LAYER_EXCEED = 5, /* second VLAN tag                                      decode-vlan.c:35-39          */
    PPE_ST_VLAN_UNSUPPORT = 6,    /* inner type not 0x0800/0x8100/0x9100                  decode-vlan.c:76-84          */
    PPE_ST_IPV4_HEADER_ERR = 7,   /* len<20 or ihl*4<20                                   decode-ipv4.c:30-48          */
    PPE_ST_IPV4_VERSION_ERR = 8,  /* version != 4                                         decode-ipv4.c:36-40          */
    PPE_ST_IPV4_LEN_ERR = 9,      /* ip_len<ihl*4 or len<ip_len                           decode-ipv4.c:50-60          */
    PPE_ST_FRAG_LEN_ERR = 10,     /* fragment with zero payload                           decode-ipv4.c:227-232        */
    PPE_ST_FRAG = 11,             /* fragment → Defrag (PUNT to host)                     decode-ipv4.c:216-239        */
    PPE_ST_IPV4_UNSUPPORT = 12,   /* protocol not TCP/UDP                                 decode-ipv4.c:347-357        */
    PPE_ST_UDP_HEADER_ERR = 13,   /* l4len<8                                              decode-udp.c:18-22           */
    PPE_ST_UDP_LEN_ERR = 14,      /* uh_len != l4len                                      decode-udp.c:26-36           */
    PPE_ST_TCP_HEADER_ERR = 15,   /* l4len<20                                             decode-tcp.c:140-144         */
    PPE_ST_TCP_LEN_ERR = 16,      /* l4len<hlen or (u8)(hlen-20)>40                        decode-tcp.c:148-160         */
    PPE_ST_FLOW_TCP_NO_SYN_FIRST = 17, /* flow miss, TCP without SYN, syn_check on        flow.c:204-214               */
    PPE_ST_WINDOW_PUNT = 18,      /* needed header bytes lie beyond the header window (engine-specific PUNT)          */
    PPE_ST_FLOW_NOMEM = 19,       /* flow table: ACL passed but the flow pool is exhausted  STAT_FLOW_NODE_NOMEM flow.c:127 */
    PPE_ST__COUNT = 20
};

enum ppe_action { PPE_ACT_FW = 0, PPE_ACT_DROP = 1, PPE_ACT_PUNT = 2 };

#define PPE_F_VLAN   0x0001u   /* one VLAN tag decoded (mbuf->vlan_idx == 1)          */
#define PPE_F_L4     0x0002u   /* 5-tuple valid (reached FlowHandlePacket)            */
#define PPE_F_TCP    0x0004u
#define PPE_F_SYN    0x0008u   /* TCP SYN flag set                                    */
#define PPE_F_ACL    0x0010u   /* ACL consulted (acl_hit is its result)               */
#define PPE_F_FRAG   0x0020u   /* IPv4 fragment seen                                  */
#define PPE_F_FLOW   0x0040u   /* flow table: the packet has a flow (PKT_HAS_FLOW, flow.c:307)              */
#define PPE_F_TOCLIENT 0x0080u /* flow table: PKT_TO_CLIENT (clear with PPE_F_FLOW: PKT_TO_SERVER, flow.c:248-301) */
#define PPE_F_NEWFLOW 0x0100u  /* flow table: this packet created its flow (FlowAdd, flow.c:120-158)             */

#define PPE_PART_INDEX(e)  ((e) & 0x3fffffffu)   /* partition-layout entry → packet index                */
#define PPE_PART_ACTION(e) ((e) >> 30)           /* partition-layout entry → enum ppe_action             */
#define PPE_PART8_OFFSET(e) ((e) & 63u)          /* compact entry (part8) → packet index - 64 × tile      */
#define PPE_PART8_ACTION(e) ((e) >> 6)           /* compact entry (part8) → enum ppe_action               */

/* tuple word 3: the window-scale option DecodeTCPOptions records (decode-tcp.c:61-70), as its byte offset from the
 * TCP header (0 = none); OPT_PAST: none was found before the option parse needed a byte past the header window
 * (stride), so the answer needs a wider window (the reference reads the whole option space) */
#define PPE_TUPLE_WS(w3)      (((w3) >> 9) & 63u)
#define PPE_TUPLE_OPT_PAST    (1u << 15)

#define PPE_VERDICT_STATUS(v) ((v) & 0xffu)
#define PPE_VERDICT_ACTION(v) (((v) >> 8) & 0xffu)
#define PPE_VERDICT_FLAGS(v)  ((v) >> 16)

/* ---- packed result (ppe_result_t.packed): one 8-B word per packet holding verdict, flow hash and ACL hit ----
 * bits 0-31 flow hash | 32-36 status | 37-38 action | 39-44 flags (PPE_F_VLAN .. PPE_F_FRAG, the stateless path's
 * six) | 45-63 acl_hit + 1 (0 = -1).  Exactly the information of the three 4-B words in 8 B (13 → 9 B written per
 * packet with part8).  ppe_classify / ppe_classify_batches only, classifiers of at most PPE_PACKED_MAX_RULES rule
 * slots (the `n` of the commit). */
#define PPE_PACKED_MAX_RULES  ((1u << 19) - 1u)
#define PPE_PACKED_HASH(x)    ((uint32_t)(x))
#define PPE_PACKED_STATUS(x)  ((uint32_t)((x) >> 32) & 31u)
#define PPE_PACKED_ACTION(x)  ((uint32_t)((x) >> 37) & 3u)
#define PPE_PACKED_FLAGS(x)   ((uint32_t)((x) >> 39) & 63u)
#define PPE_PACKED_HIT(x)     ((int32_t)((uint32_t)((x) >> 45)) - 1)
#define PPE_PACKED_VERDICT(x) (PPE_PACKED_STATUS(x) | PPE_PACKED_ACTION(x) << 8 | PPE_PACKED_FLAGS(x) << 16)

/* ---- per-reason counters (sums over every batch since the last clear) ---- */
enum ppe_counter {
    PPE_C_L2_HEADERLEN_ERR = 0, PPE_C_L2_UNSUPPORT, PPE_C_L2_RX_OK,
    PPE_C_VLAN_HEADERLEN_ERR, PPE_C_VLAN_LAYER_EXCEED, PPE_C_VLAN_UNSUPPORT, PPE_C_VLAN_RX_OK,
    PPE_C_IPV4_HEADERLEN_ERR, PPE_C_IPV4_VERSION_ERR, PPE_C_IPV4_PKTLEN_ERR, PPE_C_IPV4_UNSUPPORT, PPE_C_IPV4_RX_OK,
    PPE_C_FRAG_FRAGLEN_ERR, PPE_C_FRAG_PUNT,
    PPE_C_UDP_HEADERLEN_ERR, PPE_C_UDP_PKTLEN_ERR, PPE_C_UDP_RX_OK,
    PPE_C_TCP_HEADERLEN_ERR, PPE_C_TCP_PKTLEN_ERR, PPE_C_TCP_RX_OK,
    PPE_C_ACL_DROP, PPE_C_ACL_FW,
    PPE_C_FLOW_PROC_OK, PPE_C_FLOW_PROC_FAIL, PPE_C_FLOW_TCP_NO_SYN_FIRST,
    PPE_C_OUT_FW, PPE_C_OUT_DROP, PPE_C_OUT_PUNT, PPE_C_WINDOW_PUNT, PPE_C_PKTS,
    PPE_C_FLOW_NODE_NOMEM,     /* flow table only: FlowAdd found the pool empty (decode-statistic.h:304) */
    PPE_C_RX_BYTES,            /* sum of pkt_totallen (STAT_RECV_PB_ADD, oct-rxtx.c:213)                 */
    PPE_C__COUNT /* 32 */
};

typedef struct {
    uint64_t c[32];            /* indexed by enum ppe_counter */
} ppe_counters_t;

/* ---- batch input: structure of arrays, one header window per packet ---- */
typedef struct {
    const uint8_t  *hdr;       /* n × stride bytes: the first min(len, stride) bytes of each packet            */
    const uint32_t *len;       /* n × wire length (mbuf->pkt_totallen; truncated to 16 bits like Decode())      */
    const uint64_t *ts;        /* optional n × seconds since 1970 (mbuf->timestamp); NULL → cfg->now_seconds    */
    uint32_t        n;
    uint32_t        stride;    /* a multiple of 16 from 64 to 256: 64 holds every header of a 64-B packet without
                                  VLAN / IPv4 / TCP options; 144 every byte the reference's decoders read
                                  (Ethernet 14 + VLAN 4 + IPv4 60 + TCP 60), so no WINDOW_PUNT and no
                                  PPE_TUPLE_OPT_PAST can occur                                                   */
} ppe_batch_t;

/* ---- batch output (SoA; any pointer may be NULL to skip that output) ---- */
typedef struct {
    uint32_t *verdict;         /* n × verdict word                                                            */
    uint32_t *flow_hash;       /* n × flow_hashfn(proto,sip,dip,sport,dport); 0 unless PPE_F_L4                */
    int32_t  *acl_hit;         /* n × lowest matching rule index, -1 on no match / not consulted               */
    uint32_t *fw_idx;          /* n slots: per 64-packet tile t, the FW packet indices packed at [64t, 64t+k)  */
    uint32_t *drop_idx;        /* n slots: same for DROP                                                      */
                               /* fw_idx == drop_idx selects the PARTITION layout: slots [64t, 64t+v) of tile t
                                  (v = its packet count) hold all of its packet indices, FW ascending from the
                                  front, DROP ascending at the back, PUNT ascending in between; each entry is
                                  index | action << 30 (PPE_PART_*), so no tile_cnt is needed to split them     */
    uint32_t *tile_cnt;        /* ceil(n/64) × (nfw | ndrop << 8 | npunt << 16)                                */
    uint32_t *tuple;           /* optional n × 4 words, what the reference's decoders record in the mbuf:
                                  [0] sip [1] dip (0 unless the IPv4 checks passed, decode-ipv4.c:62-63)
                                  [2] sport | dport << 16 (PPE_F_L4), or for a fragment (status FRAG /
                                      FRAG_LEN_ERR) defrag_id | frag_offset << 16 (decode-ipv4.c:107-108)
                                  [3] proto | vlan << 8 | PPE_TUPLE_WS | PPE_TUPLE_OPT_PAST | payload_len << 16
                                      (a fragment: frag_len << 16, decode-ipv4.c:109)                            */
    uint8_t  *part8;           /* optional n bytes: the PARTITION layout in compact form (with fw_idx, drop_idx
                                  and tile_cnt NULL): slot [64t + i] of tile t holds the i-th entry of the
                                  partition order above as (packet index - 64t) | action << 6 (PPE_PART8_*);
                                  1 B written per packet instead of 4 (ABI version 4)                         */
    uint64_t *packed;          /* optional n × 8 B (PPE_PACKED_*), with verdict, flow_hash and acl_hit NULL
                                  (ABI version 8)                                                             */
} ppe_result_t;

typedef struct {
    uint32_t unsupport_proto_action;  /* 0 drop (default, dp_cmd.c:37), 1 forward                            */
    uint32_t syn_check;               /* 1 (default, flow.c:26): TCP flow must start with SYN                 */
    uint64_t now_seconds;             /* timestamp used for rule time windows when batch.ts == NULL           */
} ppe_cfg_t;

typedef struct {
    uint32_t n_rules;          /* USED rules in the committed set                                          */
    uint32_t n_nodes;          /* tree nodes                                                               */
    uint32_t n_leaves;
    uint32_t n_leaf_entries;
    uint32_t max_depth;
    double   avg_depth;
    uint32_t blob_bytes;       /* device image size                                                        */
    uint32_t lds_resident;     /* 1 if the image is staged into LDS by the kernel                          */
    double   build_ms;
    uint32_t cut_bits;         /* cut-list section (image v8): sip bits | dip bits << 8; 0 with cut_entries
                                  0 = no cut lists (ABI version 6)                                            */
    uint32_t cut_entries;      /* entries of the cut lists (rules replicated into the buckets they meet)   */
} ppe_acl_stats_t;

typedef struct ppe_ctx ppe_ctx_t;

int  ppe_abi_version(void);
/* device = HIP device ordinal */
int  ppe_ctx_create(int device, ppe_ctx_t **out);
int  ppe_ctx_destroy(ppe_ctx_t *ctx);
int  ppe_ctx_device(ppe_ctx_t *ctx);

/* Build the classifier from rules[0..n) (entry i is eligible iff used == NULL || used[i] == USED) and publish it
 * for subsequent batches (double-buffered: the previous image stays valid for launches already queued).
 * n may exceed RULE_ENTRY_MAX (extended rule API, up to 1<<24).  default_action: ACL_RULE_ACTION_FW/DROP. */
int  ppe_rules_commit(ppe_ctx_t *ctx, const RCP_BLOCK_ACL_RULE_TUPLE *rules, const uint8_t *used, uint32_t n,
                      uint32_t default_action, ppe_acl_stats_t *stats);
/* The two steps of ppe_rules_commit, as the reference's commit protocol takes them (dp_cmd.c:2019-2030: build the
 * back tree, then set_running_acltree): ppe_rules_stage builds the classifier and uploads it into the back image
 * slot without publishing it (launches keep reading the running image; the upload waits only for launches that read
 * the slot it overwrites) and returns a token (> 0); ppe_rules_publish(token) makes that image the running one for
 * later launches.  A later stage replaces an unpublished one: publishing the earlier token then fails (PPE_EINVAL),
 * as does publishing a token twice.  ABI version 7. */
int  ppe_rules_stage(ppe_ctx_t *ctx, const RCP_BLOCK_ACL_RULE_TUPLE *rules, const uint8_t *used, uint32_t n,
                     uint32_t default_action, ppe_acl_stats_t *stats, uint64_t *token);
int  ppe_rules_publish(ppe_ctx_t *ctx, uint64_t token);

/* Classify one device-resident batch, enqueued on `stream` (a hipStream_t; NULL = the legacy default stream). */
int  ppe_classify(ppe_ctx_t *ctx, const ppe_batch_t *in, const ppe_result_t *out, const ppe_cfg_t *cfg,
                  void *stream);

/* Several device-resident batches (in[i] → out[i]), pipelined: consecutive batches alternate over two internal
 * streams so that one batch's launch ramp-up overlaps the previous batch's tail.  Stream-ordered like
 * ppe_classify: the batches run after the work already queued on `stream`, and work queued on `stream` after this
 * call runs after all of them.  The batches' output buffers must not overlap (two may be written at once). */
int  ppe_classify_batches(ppe_ctx_t *ctx, const ppe_batch_t *in, const ppe_result_t *out, uint32_t nbatch,
                          const ppe_cfg_t *cfg, void *stream);

/* Host-resident batch.  When every buffer is pinned and device-mapped (hipHostMalloc, hipHostRegister, a pinned
 * torch tensor), the kernel reads and writes them across PCIe directly (zero-copy; PPE_HOST_ZEROCOPY=0 disables);
 * otherwise pipelined H2D → classify → D2H over `chunk`-packet slices on internal streams.
 * Output pointers are host pointers (NULL to skip).  Blocks until done. */
int  ppe_classify_host(ppe_ctx_t *ctx, const ppe_batch_t *in, const ppe_result_t *out, const ppe_cfg_t *cfg,
                       uint32_t chunk);

/* ACL-only lookup over already-decoded 5-tuples (DP_Acl_Lookup, dataplane/src/flow/flow.c:232).
 * tuple: n × 4 words {sip, dip, sport | dport << 16, proto} — the same layout as ppe_result_t.tuple;
 * macs (optional): n × 4 words {dmac bytes 0-3, dmac bytes 4-5, smac bytes 0-3, smac bytes 4-5} (little-endian);
 * ts (optional): n × seconds, else now_seconds.  hit: lowest matching rule index or -1; action: the matched rule's
 * action word or the default action. */
typedef struct {
    const uint32_t *tuple;
    const uint32_t *macs;
    const uint64_t *ts;
    uint32_t        n;
} ppe_tuples_t;
int  ppe_acl_lookup(ppe_ctx_t *ctx, const ppe_tuples_t *in, int32_t *hit, uint32_t *action, uint64_t now_seconds,
                    void *stream);                                   /* device pointers, asynchronous */
int  ppe_acl_lookup_host(ppe_ctx_t *ctx, const ppe_tuples_t *in, int32_t *hit, uint32_t *action,
                         uint64_t now_seconds);                      /* host pointers, blocking */

/* Memory helpers for C integrators (device / pinned host buffers on the context's device). */
void *ppe_dev_alloc(ppe_ctx_t *ctx, size_t bytes);
void  ppe_dev_free(ppe_ctx_t *ctx, void *p);
void *ppe_host_alloc(ppe_ctx_t *ctx, size_t bytes);   /* pinned */
void  ppe_host_free(ppe_ctx_t *ctx, void *p);
int   ppe_memcpy_h2d(ppe_ctx_t *ctx, void *dst, const void *src, size_t bytes);
int   ppe_memcpy_d2h(ppe_ctx_t *ctx, void *dst, const void *src, size_t bytes);
int   ppe_memset_d(ppe_ctx_t *ctx, void *dst, int value, size_t bytes);
int   ppe_sync(ppe_ctx_t *ctx);

/* Counters: per-workgroup slots in device memory, reduced on read.  Synchronises the device. */
int  ppe_counters_read(ppe_ctx_t *ctx, ppe_counters_t *out);
int  ppe_counters_clear(ppe_ctx_t *ctx);

/* Kernel timing with HIP events recorded around each ppe_classify launch on its stream. */
int  ppe_timing_enable(ppe_ctx_t *ctx, int on);
/* Synchronises, then returns the sum of launch durations (ms) and the launch count since the last reset. */
int  ppe_timing_read(ppe_ctx_t *ctx, double *total_ms, uint32_t *launches, int reset);

/* Copy the current device classifier image to host (for tests / tools).  words may be NULL to query size. */
int  ppe_acl_image(ppe_ctx_t *ctx, uint32_t *words, uint32_t *n_words);

/* Launch tuning of the classify kernel for this context.  Defaults come from the fastest measured variant (and the
 * PPE_BLOCK / PPE_BLOCKS_PER_CU / PPE_PIPELINE / PPE_LDS_IMG environment variables); 0 = automatic. */
typedef struct {
    uint32_t block;          /* workgroup size 256, 512 or 1024; 0 = chosen per classifier image   */
    uint32_t blocks_per_cu;  /* workgroups per CU (<= 32); 0 = resident count from the occupancy API */
    uint32_t pipeline;       /* tile fetch / walk: 0 auto (4 when the image's tree fits in LDS, else 5
                                when it has cut lists, else 3), 1 first tile loaded at the loop top,
                                4 first tile requested before the image staging, 3 four tiles per
                                wave loaded, decoded and walked together through the 2-level blocks
                                (one 1024-thread workgroup per CU), 5 the cut lists (image v7: one
                                tile per wave, bucket groups in LDS, list entries from L2; an image
                                without cut lists takes the automatic choice); others PPE_EINVAL   */
    uint32_t lds_image;      /* 1 = stage the image (or its top) in LDS, 0 = read it from global   */
    uint32_t batches_per_launch;  /* ppe_classify_batches: batches one launch takes (<= 4096); 0 = all
                                     of a call's batches in ONE persistent launch (descriptor ring)  */
} ppe_tuning_t;
int  ppe_set_tuning(ppe_ctx_t *ctx, const ppe_tuning_t *t);
int  ppe_get_tuning(ppe_ctx_t *ctx, ppe_tuning_t *t);

/* Launch geometry in use (for profiling notes).  variant = image mode (0 global, 1 LDS, 2 split) | fetch << 4
 * (fetch 0 first tile at the loop top, 1 first tile requested before the image staging, 3 four tiles per wave,
 * 5 cut lists). */
int  ppe_launch_info(ppe_ctx_t *ctx, uint32_t *grid, uint32_t *block, uint32_t *lds_bytes, uint32_t *variant);


/* ---- Stateful flow table (dataplane/src/flow/flow.c) ----
 * One table per context (the reference keeps one per core, flow_table[LOCAL_CPU_ID]; across GPUs, shard packets by
 * flow hash so each flow lives on one device).  ppe_classify_flow() runs the reference's FlowHandlePacket for a whole
 * batch with exactly the sequential semantics of one core processing the batch in index order:
 *   - a packet whose flow exists (FlowFind: 5-tuple match in either direction, flow.c:81-115) is forwarded without
 *     an ACL lookup, counted ACL_FW / FLOW_PROC_OK, and updates the flow's per-direction packet / byte counters
 *     (FlowUpdate, flow.c:163-178, bytes = pkt_totallen) and last-seen time (FLOW_UPDATE_TIMESTAMP = cfg->now_seconds);
 *   - otherwise syn_check and the ACL decide as in the stateless path; an ACL FW creates the flow (FlowAdd, oriented
 *     as that packet), or fails with PPE_ST_FLOW_NOMEM when `capacity` flows are live (flow.c:124-129);
 *   - later packets of the same batch see flows created by earlier ones (in index order).
 * acl_hit is -1 and PPE_F_ACL clear for packets that found their flow.  Aging (FlowTimeOut / FlowAgeTimeoutCB, flow.c:391-467) is
 * explicit: ppe_flow_age() removes flows idle for more than `timeout_seconds` (reference: FLOW_MAX_TIMEOUT = 20 s).
 * Batches go through one stream in order; out->verdict is required; n <= max_batch. */
typedef struct {
    uint32_t sip, dip;            /* flow_item_t.ipv4 of the creating packet (flow.h:57)                        */
    uint16_t sport, dport;
    uint8_t  protocol, pad[3];
    uint32_t flowflags;           /* FLOW_FLAG_* (always 0: nothing sets PERSISTENT in the reference)            */
    uint32_t slot;                /* device table slot (diagnostic)                                              */
    uint64_t pktcnts2d, pktcntd2s, bytecnts2d, bytecntd2s;   /* flow.h:66-69                                       */
    uint64_t last_seen;           /* `cycle`: cfg->now_seconds of the last packet of the flow                    */
} ppe_flow_entry_t;

typedef struct {
    uint64_t live;                /* flows in the table                                                          */
    uint64_t new_flow, del_flow;  /* FlowAdd / aging totals since create or ppe_flow_clear_stat (dp_cmd.c:2327)  */
    uint32_t capacity;            /* flow pool size (reference MEM_POOL_FLOW_NODE_NUM = 100000)                  */
    uint32_t max_batch;
    uint32_t slots;               /* open-addressing slots (power of two >= 2 x (capacity + max_batch))          */
    uint32_t tombstones;          /* deleted slots not yet reclaimed by a rehash                                 */
    uint32_t rehashes;
    uint32_t pad;
} ppe_flow_info_t;

/* FlowInit (flow.c:471-516): create / replace the context's table.  capacity 0 = 100000, max_batch 0 = 1<<20. */
int  ppe_flow_create(ppe_ctx_t *ctx, uint32_t capacity, uint32_t max_batch);
int  ppe_flow_destroy(ppe_ctx_t *ctx);                                /* FlowRelease (flow.c:519-530) */
/* FlowHandlePacket for a device-resident batch (same buffers as ppe_classify), stream-ordered on `stream`.
 * A batch is two launches (classify, then finalize + counter update).  If the second one cannot be launched, the call
 * returns PPE_EIO and the table is unusable from then on: every later ppe_classify_flow / ppe_flow_age / _info /
 * _clear_stat / _dump returns PPE_EIO at once, until ppe_flow_destroy (or a new ppe_flow_create). */
int  ppe_classify_flow(ppe_ctx_t *ctx, const ppe_batch_t *in, const ppe_result_t *out, const ppe_cfg_t *cfg,
                       void *stream);
/* FlowAgeTimeoutCB: delete flows with now > last_seen && now - last_seen > timeout_seconds; *deleted = count
 * (may be NULL).  Synchronises. */
int  ppe_flow_age(ppe_ctx_t *ctx, uint64_t now_seconds, uint64_t timeout_seconds, uint64_t *deleted);
int  ppe_flow_info(ppe_ctx_t *ctx, ppe_flow_info_t *info);         /* dp_show_flow_stat (dp_cmd.c:2346); syncs */
int  ppe_flow_clear_stat(ppe_ctx_t *ctx);                           /* dp_clear_flow_stat (dp_cmd.c:2327) */
/* Copy up to `max` live flows to host (table order); *n = live flows.  Synchronises. */
int  ppe_flow_dump(ppe_ctx_t *ctx, ppe_flow_entry_t *entries, uint32_t max, uint32_t *n);

/* ---- Flow-hash steering across GPUs (the stateful path shards by flow, like Octeon's PIP tag
 * steering of a flow to one core, dataplane/src/platform/oct-init.c:139-151) ----
 * ppe_steer_partition: from a stateless ppe_classify of the batch (verdict + flow_hash), each packet's owner GPU is
 * flow_hash % world if it reaches the flow table (PPE_F_L4), else `rank` (its stateless verdict is final anyway).
 * perm[n] = packet indices grouped by owner, ascending within each owner; counts[world] = packets per owner.
 * ppe_gather_rows: dst[i] = src[perm[i]]; ppe_scatter_rows: dst[perm[i]] = src[i] (rows of row_bytes, a multiple of
 * 4, <= 256).  All device pointers, stream-ordered.  world <= 16.  The exchange itself is an all-to-all of the
 * gathered windows (RCCL over xGMI), then ppe_classify_flow on the received packets and the reverse all-to-all of
 * their verdicts: packet-process-engine_amd/ppe/dist.py steered_classify_flow. */
int  ppe_steer_partition(ppe_ctx_t *ctx, const uint32_t *verdict, const uint32_t *flow_hash, uint32_t n,
                         uint32_t world, uint32_t rank, uint32_t *perm, uint32_t *counts, void *stream);
int  ppe_gather_rows(ppe_ctx_t *ctx, const void *src, uint32_t row_bytes, const uint32_t *perm, uint32_t n,
                     void *dst, void *stream);
int  ppe_scatter_rows(ppe_ctx_t *ctx, const void *src, uint32_t row_bytes, const uint32_t *perm, uint32_t n,
                      void *dst, void *stream);

/* Operator text of the reference's `show` commands, from counters / flow info read with ppe_counters_read /
 * ppe_flow_info: dp_show_pkt_stat (dataplane/src/common/dp_cmd.c:844-1818; same sections, names and order; the
 * reference's SELF_TEST build (flow.c:21) never counts output_*, and the I/O, ARP/ICMP/OSPF, TX and other attack
 * counters have no source on this path: those lines print 0) and dp_show_flow_stat (dp_cmd.c:2346-2392); the
 * reassembly lines come from ppe_defrag_info (ppe_format_*_ex, declared with the reassembly API below).
 * snprintf semantics: returns the full length, writes at most cap bytes including the NUL. */


/* ---- IPv4 reassembly (dataplane/src/decode/decode-defrag.c) ----
 * ppe_classify PUNTs fragments (PPE_ST_FRAG).  ppe_defrag runs the reference's Defrag (decode-defrag.c:449-487) for
 * a batch of them, with exactly the sequential semantics of one core handling the fragments in index order:
 *   FragFind / fcb_create on (sip, dip, ip_id) (decode-defrag.c:115-146, 71-97; at most fcb_max FCBs, STAT_FRAG_FCB_FULL),
 *   PACKET_HW2SW into a 2 KB buffer (mbuf.c:117-156: pkt_totallen > frag_buf_bytes drops, STAT_FRAG_HW2SW_ERR),
 *   the DELETE / cache_max checks of Frag_defrag_begin (decode-defrag.c:412-446) and Frag_defrag_process
 *   (decode-defrag.c:292-406) — ordered fragment chain, overlap ("teardrop") and last-fragment checks, including the
 *   reference's chain scan that compares frag_len (not frag_offset) with the new offset (decode-defrag.c:344-349);
 *   on completion Frag_defrag_reasm (decode-defrag.c:222-289): the head fragment's whole frame followed by every
 *   later fragment's last frag_len bytes, ip_len = ihl*4 + total, ip_off = 0, header checksum recomputed (ICMP: the
 *   head frame only, ip_off = 0).  A datagram whose buffer (total + L2 + ihl*4) exceeds reasm_buf_bytes fails as
 *   STAT_FRAG_SETUP_ERR (MEM_8K_ALLOC, decode-defrag.c:173-183) and its fragments stay cached.
 * Reassembled datagrams come out as a classify-ready batch: the reference continues with DecodeTCP / DecodeUDP /
 * the flow table on them (decode-ipv4.c:241-290), which ppe_classify / ppe_classify_flow of that batch reproduce
 * (their L2 / IPv4 checks pass by construction; the counters of that classify count the datagram once more).
 * The datagram's verdict applies to all of its fragments (the reference forwards or frees the chain with it).
 * Aging (Frag_defrag_timeout, decode-defrag.c:490-551, every second): ppe_defrag_age frees completed FCBs and those
 * idle for more than timeout_seconds (FRAG_MAX_TIMEOUT 20 s), dropping the fragments they still hold. */
enum ppe_defrag_status {
    PPE_DF_CACHED = 0,        /* held in its FCB's chain                                  STAT_FRAG_CACHE_OK   */
    PPE_DF_REASM = 1,         /* completed its datagram (dgram_of = its index)            STAT_FRAG_REASM_OK   */
    PPE_DF_SETUP_ERR = 2,     /* completed, but the reassembly buffer is too small: held  STAT_FRAG_SETUP_ERR  */
    PPE_DF_FCB_FULL = 3,      /* drop: fcb_max FCBs in use                                STAT_FRAG_FCB_FULL   */
    PPE_DF_HW2SW_ERR = 4,     /* drop: frame longer than frag_buf_bytes                   STAT_FRAG_HW2SW_ERR  */
    PPE_DF_DELETED = 5,       /* drop: its FCB already reassembled, awaiting aging (decode-defrag.c:422-427)    */
    PPE_DF_CACHE_FULL = 6,    /* drop: cache_max fragments already held                   STAT_FRAG_CACHE_FULL */
    PPE_DF_DEFRAG_ERR = 7,    /* drop: overlap / duplicate last fragment / short final    STAT_FRAG_DEFRAG_ERR */
    PPE_DF_NOT_FRAG = 8,      /* input is not an IPv4 fragment Defrag would see (caller error; untouched)      */
    PPE_DF__COUNT = 9
};
#define PPE_DF_TEARDROP 0x100u   /* | PPE_DF_DEFRAG_ERR: an overlap (DP_Teardrop_Attack_Monitor, decode-defrag.c:395-398) */

typedef struct {
    uint32_t fcb_max;          /* 0 → DEFRAG_FCB_MAX 1024 (decode-defrag.h:11)                                 */
    uint32_t cache_max;        /* 0 → defrag_cache_max 8 (decode-defrag.c:24); <= 16                           */
    uint32_t frag_buf_bytes;   /* 0 → 2024: the 2 KB small-buffer slice minus its 24-B control block
                                  (mem_pool.c:249, mem_pool.h:62); <= 4096                                     */
    uint32_t reasm_buf_bytes;  /* 0 → 8168: the 8 KB large-buffer slice minus its control block (mem_pool.c:269) */
    uint32_t max_batch;        /* fragments per ppe_defrag call; 0 → 65536                                      */
    uint32_t pad;
} ppe_defrag_cfg_t;

typedef struct {
    const uint8_t  *pkt;       /* whole frames, frame i at pkt + off[i] (device)                                 */
    const uint64_t *off;
    const uint32_t *len;       /* n × pkt_totallen                                                              */
    const uint64_t *id;        /* optional n × caller packet ids, echoed in dgram_frags (NULL → the batch index) */
    uint32_t        n;
    uint32_t        pad;
    uint64_t        now_seconds;   /* FCB_UPDATE_TIMESTAMP of every FCB the batch touches                       */
} ppe_frag_batch_t;

typedef struct {
    uint32_t *status;          /* n × (enum ppe_defrag_status | PPE_DF_TEARDROP)                                 */
    uint32_t *dgram_of;        /* optional n: datagram index of a PPE_DF_REASM fragment, else 0xffffffff        */
    uint8_t  *dgram_hdr;       /* n × hdr_stride: the first bytes of datagram j (a ppe_batch_t.hdr; zero-padded) */
    uint32_t *dgram_len;       /* n: its pkt_totallen (a ppe_batch_t.len); 0 for j >= the datagram count        */
    uint8_t  *dgram_pkt;       /* optional n × reasm_buf_bytes: the whole reassembled frames                    */
    uint64_t *dgram_frags;     /* optional n × cache_max: ids of datagram j's fragments in chain order, ~0 pad   */
                               /* (dgram_hdr / dgram_pkt / dgram_frags rows j >= the datagram count: not written) */
    uint32_t *n_dgram;         /* optional device word: datagrams written                                      */
    uint32_t  hdr_stride;      /* 64 or 128                                                                    */
    uint32_t  pad;
} ppe_defrag_out_t;

typedef struct {
    uint64_t running;          /* FCBs in use (fcb_running_num)                                                 */
    uint64_t new_fcb, del_fcb; /* decode-defrag.c:15-16                                                         */
    uint64_t st[PPE_DF__COUNT];/* fragments per enum ppe_defrag_status                                          */
    uint64_t teardrop;         /* overlaps among PPE_DF_DEFRAG_ERR                                              */
    uint64_t timeout_drop;     /* fragments dropped by ppe_defrag_age                                           */
    uint64_t datagrams;        /* reassembled datagrams emitted                                                 */
    uint32_t fcb_max, cache_max, frag_buf_bytes, reasm_buf_bytes, max_batch, slots;
} ppe_defrag_info_t;

typedef struct ppe_defrag_table ppe_defrag_t;
/* FragModule_init (decode-defrag.c:582-625): a device FCB table on ctx's device.  cfg may be NULL (defaults). */
int  ppe_defrag_create(ppe_ctx_t *ctx, const ppe_defrag_cfg_t *cfg, ppe_defrag_t **out);
int  ppe_defrag_destroy(ppe_defrag_t *d);                              /* FragModule_Release */
/* Defrag for a device-resident batch of fragments, stream-ordered on `stream` (batches in call order).
 * status, dgram_of and dgram_len are written for all n entries (dgram_len 0 past the datagram count: a runt frame
 * whose verdict does not depend on its window bytes), so a ppe_classify of {dgram_hdr, dgram_len, n, hdr_stride}
 * can follow on the same stream without a host sync. */
int  ppe_defrag(ppe_defrag_t *d, const ppe_frag_batch_t *in, const ppe_defrag_out_t *out, void *stream);
/* Frag_defrag_timeout: free FCBs that completed, or with now > last && now - last > timeout_seconds; the ids of
 * the fragments they still held go to dropped[0..max) (host; may be NULL), *n_dropped = their count, *n_freed =
 * FCBs freed (either may be NULL).  Synchronises. */
int  ppe_defrag_age(ppe_defrag_t *d, uint64_t now_seconds, uint64_t timeout_seconds, uint64_t *dropped,
                    uint32_t max, uint32_t *n_dropped, uint32_t *n_freed);
int  ppe_defrag_info(ppe_defrag_t *d, ppe_defrag_info_t *info);      /* synchronises */

/* `show packet statistic` / `show flow statistic` text (dp_show_pkt_stat / dp_show_flow_stat,
 * dataplane/src/common/dp_cmd.c:844-1818, 2346-2392) into buf (NUL-terminated, truncated to cap); returns the full
 * length.  The _ex forms take the IPv4 reassembly table's counters (NULL: those lines print 0, as the plain forms
 * do): the ip_frag_stat section, the new / del fcb lines and, while the teardrop monitor is enabled
 * (teardrop_monitor != 0; off in the reference's default configuration), the attack section's teardrop line. */
int  ppe_format_pkt_stat(const ppe_counters_t *c, char *buf, size_t cap);
int  ppe_format_flow_stat(const ppe_flow_info_t *f, char *buf, size_t cap);
int  ppe_format_pkt_stat_ex(const ppe_counters_t *c, const ppe_defrag_info_t *df, int teardrop_monitor, char *buf,
                            size_t cap);
int  ppe_format_flow_stat_ex(const ppe_flow_info_t *f, const ppe_defrag_info_t *df, char *buf, size_t cap);
const char *ppe_defrag_last_error(ppe_defrag_t *d);

/* Human-readable last error of this context (static storage of the ctx). */
const char *ppe_last_error(ppe_ctx_t *ctx);

/* Host-side classifier compiler (no device needed): rule list → image words (ppe_image.h layout, malloc'd;
 * free with ppe_acl_free_image).  binth = max rules in a leaf list before splitting (0 → default 1). */
int  ppe_acl_build_image(const RCP_BLOCK_ACL_RULE_TUPLE *rules, const uint8_t *used, uint32_t n,
                         uint32_t default_action, uint32_t binth, uint32_t **words, uint32_t *n_words,
                         ppe_acl_stats_t *stats);
void ppe_acl_free_image(uint32_t *words);

#ifdef __cplusplus
}
#endif
#endif /* PPE_HIP_H */
