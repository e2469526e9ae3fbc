/*
 * ppe_decode.h — PPE-compatible decoder / plugin / log-hook surface over the GPU engine.
 *
 * Reference interfaces this replaces:
 *   void Decode(mbuf_t *m)                                dataplane/src/decode/decode.c:19-28
 *   DECODE_OK / DECODE_DROP / DECODE_DONE                 dataplane/src/decode/decode.h:7-9
 *   mbuf_t parse fields (eth_dst/src, ipv4, sport, dport, proto, vlan_idx, payload_len, timestamp, flags)
 *                                                         dataplane/src/include/mbuf.h:23-87
 *   PluginModule / plugin_modules[PLUGIN_SIZE]            dataplane/src/plugin/plugin-mod/plugin.h:9-19, plugin.c:8
 *   reg_fw_alert / DP_Log_Func                            dataplane/src/common/dp_log.c:12-31
 *   int DP_Acl_Lookup(mbuf_t *)                           dataplane/src/flow/flow.c:232
 *
 * The reference decodes one mbuf per call on the calling core and has finished with it when Decode returns
 * (decode.c:13-28).  So does this Decode by default: the burst size is 1, and Decode(m) classifies m on the GPU and
 * delivers it before it returns.  A caller that wants GPU-sized batches opts in with Decode_Set_Burst(n): Decode(m)
 * then appends the mbuf to the calling thread's own burst (one per thread, as the reference's per-core mainloop),
 * classified when it reaches n entries or when that thread calls Decode_Flush() (or exits).  Either way the
 * verdict is delivered exactly as the reference does — output_fw_proc(m) / output_drop_proc(m) hooks, with
 * DP_Log_Func(m) on the drop reasons the reference logs — and the mbuf's parse fields are filled in.
 * Every classification runs on the GPU; there is no CPU decode path.
 */
#ifndef PPE_DECODE_H
#define PPE_DECODE_H

#include <stdint.h>
#include "ppe_acl.h"

#ifdef __cplusplus
extern "C" {
#endif

#define DECODE_OK   0
#define DECODE_DROP 1
#define DECODE_DONE 2

/* mbuf flags (dataplane/src/decode/decode.h:12-21) */
#define PKT_IP_FRAG    (1 << 1)
#define PKT_TO_SERVER  (1 << 4)
#define PKT_TO_CLIENT  (1 << 5)
#define PKT_HAS_FLOW   (1 << 8)

#ifndef PPE_HAVE_CVMX
/* the Octeon SDK's 64-bit work-queue buffer word (cvmx-packet.h); a build that includes cvmx.h defines
 * PPE_HAVE_CVMX and uses the SDK's own type */
typedef union {
    uint64_t u64;
} cvmx_buf_ptr_t;
#endif

#ifndef __DECODE_TCP_H__
/* dataplane/src/decode/decode-tcp.h:24-46 (only the types mbuf_t embeds) */
typedef struct TCPOpt_ {
    uint8_t type;
    uint8_t len;
    uint8_t *data;
} TCPOpt;

typedef struct TCPVars_ {
    TCPOpt tcp_opts[1];
    TCPOpt *ws;                /* the window-scale option DecodeTCPOptions recorded (decode-tcp.c:61-70), filled by
                                  Decode from the kernel's option parse; NULL (as allocated) when there is none */
} TCPVars;
#define TCP_OPTS tcpvars.tcp_opts  /* m->TCP_OPTS[0], decode-tcp.c:66-68 */
#endif

typedef void (*FreeAlState)(void *s);

typedef struct {
    uint32_t sip;
    uint32_t dip;
} ipv4_tuple_t;

/* The reference's mbuf_t, field for field in the reference's order (dataplane/src/include/mbuf.h:23-87), so
 * oct_rx_process_work-style producers (dataplane/src/platform/oct-rxtx.c:190-206: magic_flag, pkt_space,
 * packet_ptr, input_port, pkt_totallen, pkt_ptr, tag, timestamp) compile against it unchanged; on LP64 every
 * reference field keeps its reference offset (sizeof of the reference part = 232 B, the memset of
 * oct-rxtx.c:192).  The engine's results are appended after `tag`. */
typedef struct m_buf_ {
    uint32_t magic_flag;       /* MBUF_MAGIC_NUM                                                 */
    uint8_t pkt_space;         /* PKTBUF_HW / PKTBUF_SW                                          */
    uint8_t flow_log;
    uint16_t frag_len;
    cvmx_buf_ptr_t packet_ptr;
    struct m_buf_ *next;
    void *pkt_ptr;             /* start of the L2 frame                                         */
    void *ethh;                /* set on decode                                                  */
    void *vlanh;
    void *network_header;
    void *transport_header;
    uint32_t input_port;
    uint8_t eth_dst[6];
    uint8_t eth_src[6];
    ipv4_tuple_t ipv4;
    uint16_t sport;
    uint16_t dport;
    uint8_t proto;
    uint8_t vlan_idx;
    uint16_t payload_len;
    uint16_t vlan_id;          /* never written by the reference decoder             */
    uint16_t defrag_id;
    uint64_t timestamp;        /* seconds since 1970; the ACL time window is checked against it */
    void *payload;
    union {
        TCPVars tcpvars;
    };
    uint16_t frag_offset;
    uint16_t tcp_reasm_overlap;
    uint32_t pkt_totallen;     /* wire length                                                   */
    uint32_t flags;
    uint32_t fcb_hash;
    void *fcb;
    struct m_buf_ *fragments;
    void *flow;
    struct m_buf_ *tcp_seg_raw;
    struct m_buf_ *tcp_seg_raw_tail;
    struct m_buf_ *tcp_seg_reassem;
    void *alState;
    FreeAlState FreeState;
    uint32_t tag;
    /* engine results (no reference counterpart) */
    uint32_t ppe_verdict;      /* status | action << 8 | flags << 16 (ppe_hip.h)                 */
    uint32_t ppe_flow_hash;    /* flow_hashfn value (bucket = & 0xFFFF, dataplane/src/flow/flow.c:76-79) */
    int32_t ppe_acl_hit;       /* lowest matching rule index or -1                               */
    void *user;
} mbuf_t;

#define MBUF_MAGIC_NUM 0xab00ab00 /* dataplane/src/include/mbuf.h:91 */
#define PKTBUF_HW 1
#define PKTBUF_SW 2

/* Output hooks (the reference's output_fw_proc / output_drop_proc, dataplane/src/output/output.c:106,151).
 * punt: fragments for Defrag (decode-ipv4.c:234) and packets whose headers exceed the header window. */
typedef void (*ppe_output_fn)(mbuf_t *m);
void ppe_set_output_hooks(ppe_output_fn fw, ppe_output_fn drop, ppe_output_fn punt);

/* config knobs pushed by the manager in the reference (dp_cmd.c:37 unsupport_proto_action, flow.c:26 syn_check) */
extern uint32_t unsupport_proto_action;
extern uint32_t syn_check;

void Decode(mbuf_t *m);
/* Classify every mbuf the calling thread has queued; returns the number delivered through the output hooks, or a
 * negative PPE_E* code when the GPU step failed, in which case every queued mbuf was handed to the drop hook (the
 * reference ends every undelivered packet in output_drop_proc).  Hooks run with no engine lock held, so a hook
 * may call Decode() again (e.g. a punt hook feeding reassembled datagrams back). */
int  Decode_Flush(void);
/* Burst size at which Decode() flushes automatically: 1 (the default) = synchronous, the reference's contract; a
 * larger n queues up to n mbufs per thread (the caller then calls Decode_Flush() at its batch boundaries).  May be
 * changed at any time; it applies to every thread's next Decode().  n = 0 is ignored. */
void Decode_Set_Burst(uint32_t n);

/* Batch form of DP_Acl_Lookup over already-decoded mbufs (ACL_RULE_ACTION_FW / _DROP per mbuf). */
int  DP_Acl_Lookup_Burst(mbuf_t **m, uint32_t n, int *actions);
int  DP_Acl_Lookup(mbuf_t *m);

/* ---- plugin ABI (dataplane/src/plugin/plugin-mod/plugin.h:9-19) ---- */
typedef enum {
    PLUGIN_STREAMTCP,
    PLUGIN_SIZE,
} PluginId;

typedef struct {
    char *name;
    int (*Init)(void);
    int (*Func)(mbuf_t *m);
} PluginModule;

extern PluginModule plugin_modules[PLUGIN_SIZE];

/* ---- drop-log hook (dataplane/src/common/dp_log.c:12-31) ---- */
typedef int (*fw_alert)(void *);
void reg_fw_alert(fw_alert fun);
void DP_Log_Func(mbuf_t *m);

/* engine context behind the compat layer (created by DP_Acl_Rule_Init) */
struct ppe_ctx;
struct ppe_ctx *ppe_compat_ctx(void);

#ifdef __cplusplus
}
#endif
#endif /* PPE_DECODE_H */
