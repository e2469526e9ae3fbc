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
 * The reference decodes one mbuf per call on the calling core.  Here Decode(m) appends the mbuf to the calling
 * thread's burst and the burst is classified on the GPU when it is full or when Decode_Flush() is called; the
 * verdict is then delivered exactly as the reference does — output_fw_proc(m) / output_drop_proc(m) hooks, with
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

typedef struct {
    uint32_t sip;
    uint32_t dip;
} ipv4_tuple_t;

/* The hot-path subset of the reference mbuf_t (dataplane/src/include/mbuf.h:23-87), same field names.
 * Octeon buffer-pool fields (packet_ptr, fcb, fragments, tcp segment chains) have no counterpart. */
typedef struct m_buf_ {
    void *pkt_ptr;             /* start of the L2 frame                                         */
    uint32_t pkt_totallen;     /* wire length                                                   */
    uint32_t input_port;
    void *ethh, *vlanh, *network_header, *transport_header;  /* set on decode                  */
    uint8_t eth_dst[6];
    uint8_t eth_src[6];
    ipv4_tuple_t ipv4;
    uint16_t sport;
    uint16_t dport;
    uint8_t proto;
    uint8_t vlan_idx;
    uint16_t payload_len;
    uint64_t timestamp;        /* seconds since 1970; the ACL time window is checked against it */
    void *payload;
    uint32_t flags;
    /* engine results (no reference counterpart) */
    uint32_t ppe_verdict;      /* status | action << 8 | flags << 16 (ppe_hip.h)                 */
    uint32_t ppe_flow_hash;    /* flow_hashfn value (bucket = & 0xFFFF, dataplane/src/flow/flow.c:76-79) */
    int32_t ppe_acl_hit;       /* lowest matching rule index or -1                               */
    void *user;
} mbuf_t;

/* Output hooks (the reference's output_fw_proc / output_drop_proc, dataplane/src/output/output.c:106,151).
 * punt: fragments for Defrag (decode-ipv4.c:234) and packets whose headers exceed the header window. */
typedef void (*ppe_output_fn)(mbuf_t *m);
void ppe_set_output_hooks(ppe_output_fn fw, ppe_output_fn drop, ppe_output_fn punt);

/* config knobs pushed by the manager in the reference (dp_cmd.c:37 unsupport_proto_action, flow.c:26 syn_check) */
extern uint32_t unsupport_proto_action;
extern uint32_t syn_check;

void Decode(mbuf_t *m);
/* Classify every queued mbuf now; returns the number delivered or a negative PPE_E* code. */
int  Decode_Flush(void);
/* Burst size at which Decode() flushes automatically (default 4096). */
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
