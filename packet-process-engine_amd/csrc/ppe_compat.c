/*
 * ppe_compat.c — the reference's decoder / ACL / plugin / log entry points as thin shims over the GPU engine.
 *
 *   DP_Acl_Rule_Init        main.c:177
 *   DP_Acl_Load_Rule        dataplane/src/common/dp_cmd.c:2019 (builds the back classifier; published when
 *                           g_acltree_running names its unit_tree_t, set_running_acltree, dp_cmd.c:1980-1985)
 *   DP_Acl_Rule_Clean       dataplane/src/common/dp_cmd.c:2030
 *   DP_Acl_Rule_Release     dataplane/src/platform/oct-init.c:755
 *   DP_Acl_Rule_Commit      the dp_acl_rule_commit protocol, dataplane/src/common/dp_cmd.c:1987-2053
 *   DP_Acl_Lookup           dataplane/src/flow/flow.c:232
 *   Decode                  dataplane/src/decode/decode.c:19-28 (synchronous by default, burst-queued on request;
 *                           see ppe_decode.h)
 *   reg_fw_alert/DP_Log_Func dataplane/src/common/dp_log.c:12-31
 *   plugin_modules          dataplane/src/plugin/plugin-mod/plugin.c:8
 * Every packet decision is made by the HIP kernels; nothing here inspects packet bytes to classify them.
 */
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#include "ppe_decode.h"
#include "ppe_hip.h"

uint32_t dp_acl_action_default = ACL_RULE_ACTION_DROP;
int gWstDepth = 0, gAvgDepth = 0, gChildCount = 0, gNumTreeNode = 0, gNumLeafNode = 0;
uint32_t unsupport_proto_action = 0; /* dataplane/src/common/dp_cmd.c:37 */
uint32_t syn_check = 1;              /* dataplane/src/flow/flow.c:26 */
PluginModule plugin_modules[PLUGIN_SIZE];

struct ppe_tree_set {
    uint32_t generation;
    uint64_t token;  /* ppe_rules_stage's: published when this set's unit becomes the running one */
    ppe_acl_stats_t stats;
};
struct ppe_tree_node {
    uint32_t generation;
};

static ppe_ctx_t *g_ctx = NULL;
static uint32_t g_generation = 0;

unit_tree_t g_acltree_1, g_acltree_2;
unsigned long g_acltree_running = 0;
rwlock_t acltree_running_rwlock = PPE_RWLOCK_INITIALIZER;
static uint64_t g_published = 0;  /* the token of the classifier the engine runs (under g_ctx_lock) */
static pthread_mutex_t g_lock = PTHREAD_MUTEX_INITIALIZER;
/* The engine context is thread-compatible, not thread-safe (include/ppe_hip.h): every call that uses g_ctx — a
 * Decode flush's classify, a rule commit, an ACL lookup, the release — holds g_ctx_lock, always the innermost lock
 * (g_lock and rulelist_mutex may be held around it, never taken inside it). */
static pthread_mutex_t g_ctx_lock = PTHREAD_MUTEX_INITIALIZER;
static fw_alert fw_log_fun = NULL;
static ppe_output_fn out_fw = NULL, out_drop = NULL, out_punt = NULL;

struct ppe_ctx *ppe_compat_ctx(void) { return g_ctx; }

void reg_fw_alert(fw_alert fun) { fw_log_fun = fun; }

void DP_Log_Func(mbuf_t *m) {
    if (m && fw_log_fun) fw_log_fun((void *)m);
}

void ppe_set_output_hooks(ppe_output_fn fw, ppe_output_fn drop, ppe_output_fn punt) {
    out_fw = fw;
    out_drop = drop;
    out_punt = punt;
}

int DP_Acl_Rule_Init(void) {
    pthread_mutex_lock(&g_lock);
    int rc = SEC_OK;
    if (!g_ctx) {
        const char *d = getenv("PPE_DEVICE");
        if (ppe_ctx_create(d ? atoi(d) : 0, &g_ctx) != PPE_OK) {
            g_ctx = NULL;
            rc = SEC_NO;
        }
    }
    if (rc == SEC_OK && !rule_list && ppe_rule_list_init() != 0) rc = SEC_NO;
    pthread_mutex_unlock(&g_lock);
    return rc;
}

static void publish_stats(const ppe_acl_stats_t *st) {
    gWstDepth = (int)st->max_depth;
    gChildCount = (int)st->n_leaves;
    gAvgDepth = (int)(st->avg_depth * st->n_leaves + 0.5);
    gNumTreeNode = (int)st->n_nodes;
    gNumLeafNode = (int)st->n_leaves;
}

/* The classifier the running unit names (g_acltree_running, set by dp_cmd.c's set_running_acltree) becomes the
 * engine's running image at the next classify step or lookup: its token is read under the rwlock's read side (the
 * unit's handles stay valid while it is running: dp_cmd.c cleans only the back unit), then published once.
 * Caller holds g_ctx_lock. */
static void sync_running_locked(void) {
    read_lock(&acltree_running_rwlock);
    const unit_tree_t *u = (const unit_tree_t *)g_acltree_running;
    const uint64_t token = (u && u->TreeSet) ? u->TreeSet->token : 0;
    read_unlock(&acltree_running_rwlock);
    if (g_ctx && token && token != g_published && ppe_rules_publish(g_ctx, token) == PPE_OK) g_published = token;
}

uint32_t DP_Acl_Load_Rule(rule_list_t *rl, TreeSet **tset, TreeNode **tnode) {
    if (!rl) return SEC_NO;
    RCP_BLOCK_ACL_RULE_TUPLE *t = (RCP_BLOCK_ACL_RULE_TUPLE *)malloc(sizeof(*t) * RULE_ENTRY_MAX);
    uint8_t *used = (uint8_t *)malloc(RULE_ENTRY_MAX);
    if (!t || !used) {
        free(t);
        free(used);
        return SEC_NO;
    }
    for (int i = 0; i < RULE_ENTRY_MAX; i++) {
        memcpy(&t[i], &rl->rule_entry[i].rule_tuple, sizeof(*t));
        used[i] = (uint8_t)rl->rule_entry[i].entry_status;
    }
    ppe_acl_stats_t st;
    uint64_t token = 0;
    pthread_mutex_lock(&g_ctx_lock);
    /* A switch of g_acltree_running that no classify step has synced yet reaches the engine first: the engine has
     * two slots, and the stage below reuses the back one, which may hold exactly that unpublished classifier. */
    sync_running_locked();
    const int rc = g_ctx ? ppe_rules_stage(g_ctx, t, used, RULE_ENTRY_MAX, dp_acl_action_default, &st, &token)
                         : PPE_ENODEV;
    pthread_mutex_unlock(&g_ctx_lock);
    free(t);
    free(used);
    if (rc != PPE_OK) return SEC_NO;
    publish_stats(&st);
    ++g_generation;
    if (tset) {
        struct ppe_tree_set *s = (struct ppe_tree_set *)calloc(1, sizeof *s);
        if (s) {
            s->generation = g_generation;
            s->token = token;
            s->stats = st;
        }
        *tset = s;
    }
    if (tnode) {
        struct ppe_tree_node *n = (struct ppe_tree_node *)calloc(1, sizeof *n);
        if (n) n->generation = g_generation;
        *tnode = n;
    }
    return SEC_OK;
}

void DP_Acl_Rule_Clean(TreeSet **tset, TreeNode **tnode) {
    if (tset && *tset) {
        free(*tset);
        *tset = NULL;
    }
    if (tnode && *tnode) {
        free(*tnode);
        *tnode = NULL;
    }
}

void DP_Acl_Rule_Release(void) {
    pthread_mutex_lock(&g_lock);
    pthread_mutex_lock(&g_ctx_lock);  /* no flush, commit or lookup is using the context being destroyed */
    if (g_ctx) ppe_ctx_destroy(g_ctx);
    g_ctx = NULL;
    g_published = 0;  /* (a new context numbers its tokens from 1 again) */
    pthread_mutex_unlock(&g_ctx_lock);
    write_lock(&acltree_running_rwlock);
    g_acltree_running = 0;
    write_unlock(&acltree_running_rwlock);
    DP_Acl_Rule_Clean(&g_acltree_1.TreeSet, &g_acltree_1.TreeNode);
    DP_Acl_Rule_Clean(&g_acltree_2.TreeSet, &g_acltree_2.TreeNode);
    pthread_mutex_unlock(&g_lock);
}

int DP_Acl_Rule_Commit(void) {
    if (!rule_list) return SEC_NO;
    int rc = SEC_OK;
    pthread_mutex_lock(&rule_list->rulelist_mutex);
    if (rule_list->build_status != RULE_BUILD_COMMIT) {
        /* dp_cmd.c:2017-2031: build the back tree, make it the running one, clean the new back one */
        unit_tree_t *back = g_acltree_running == (unsigned long)(void *)&g_acltree_1 ? &g_acltree_2 : &g_acltree_1;
        if (DP_Acl_Load_Rule(rule_list, &back->TreeSet, &back->TreeNode) != SEC_OK) {
            rc = SEC_NO;  /* "commit failed" */
        } else {
            write_lock(&acltree_running_rwlock);
            g_acltree_running = (unsigned long)(void *)back;
            write_unlock(&acltree_running_rwlock);
            pthread_mutex_lock(&g_ctx_lock);
            sync_running_locked();  /* (published now, not at the next batch: the commit's caller expects it) */
            pthread_mutex_unlock(&g_ctx_lock);
            unit_tree_t *old = back == &g_acltree_1 ? &g_acltree_2 : &g_acltree_1;
            DP_Acl_Rule_Clean(&old->TreeSet, &old->TreeNode);
        }
        rule_list->build_status = RULE_BUILD_COMMIT;  /* set either way, dp_cmd.c:2048 */
    }
    pthread_mutex_unlock(&rule_list->rulelist_mutex);
    return rc;
}

static void mbuf_tuple(const mbuf_t *m, uint32_t *tw, uint32_t *mw) {
    tw[0] = m->ipv4.sip;
    tw[1] = m->ipv4.dip;
    tw[2] = (uint32_t)m->sport | ((uint32_t)m->dport << 16);
    tw[3] = m->proto;
    const uint8_t *d = m->eth_dst, *s = m->eth_src;
    mw[0] = (uint32_t)d[0] | ((uint32_t)d[1] << 8) | ((uint32_t)d[2] << 16) | ((uint32_t)d[3] << 24);
    mw[1] = (uint32_t)d[4] | ((uint32_t)d[5] << 8);
    mw[2] = (uint32_t)s[0] | ((uint32_t)s[1] << 8) | ((uint32_t)s[2] << 16) | ((uint32_t)s[3] << 24);
    mw[3] = (uint32_t)s[4] | ((uint32_t)s[5] << 8);
}

int DP_Acl_Lookup_Burst(mbuf_t **m, uint32_t n, int *actions) {
    if (!m) return PPE_EINVAL;
    if (n == 0) return PPE_OK;
    /* a short burst (DP_Acl_Lookup's one flow miss, flow.c:232) stays on the stack: no allocation per call */
    enum { kStack = 64 };
    uint32_t s_tw[4 * kStack], s_mw[4 * kStack], s_act[kStack];
    uint64_t s_ts[kStack];
    int32_t s_hit[kStack];
    const int heap = n > kStack;
    uint32_t *tw = heap ? (uint32_t *)malloc((size_t)n * 16) : s_tw, *mw = heap ? (uint32_t *)malloc((size_t)n * 16) : s_mw;
    uint64_t *ts = heap ? (uint64_t *)malloc((size_t)n * 8) : s_ts;
    int32_t *hit = heap ? (int32_t *)malloc((size_t)n * 4) : s_hit;
    uint32_t *act = heap ? (uint32_t *)malloc((size_t)n * 4) : s_act;
    int rc = PPE_ENOMEM;
    if (tw && mw && ts && hit && act) {
        for (uint32_t i = 0; i < n; i++) {
            mbuf_tuple(m[i], tw + 4 * i, mw + 4 * i);
            ts[i] = m[i]->timestamp;
        }
        ppe_tuples_t in = {tw, mw, ts, n};
        pthread_mutex_lock(&g_ctx_lock);
        sync_running_locked();
        rc = g_ctx ? ppe_acl_lookup_host(g_ctx, &in, hit, act, 0) : PPE_EINVAL;
        pthread_mutex_unlock(&g_ctx_lock);
        if (rc == PPE_OK)
            for (uint32_t i = 0; i < n; i++) {
                m[i]->ppe_acl_hit = hit[i];
                if (actions) actions[i] = act[i] == ACL_RULE_ACTION_DROP ? ACL_RULE_ACTION_DROP : ACL_RULE_ACTION_FW;
            }
    }
    if (heap) {
        free(tw);
        free(mw);
        free(ts);
        free(hit);
        free(act);
    }
    return rc;
}

int DP_Acl_Lookup(mbuf_t *m) {
    int a = ACL_RULE_ACTION_FW;
    if (!m || DP_Acl_Lookup_Burst(&m, 1, &a) != PPE_OK) return (int)dp_acl_action_default;
    return a;
}

/* ---- Decode burst ----
 * One burst per thread (the reference decodes on the core that received the packet, main.c:301).  The GPU step of a
 * flush is serialised per process (one engine context, thread-compatible); the output hooks run after it with no
 * lock held.  The header window holds every byte the reference's decoders read (Ethernet 14 + VLAN 4 + IPv4 60 +
 * TCP 60 = 138 B): no packet PUNTs for its window and every TCP option is parsed (ppe_hip.h ppe_batch_t.stride). */
#define PPE_COMPAT_STRIDE 144u
typedef struct {
    mbuf_t **m;
    uint32_t n, alloc;
} burst_t;

/* 1 (the default): Decode(m) classifies m and delivers it through a hook before it returns, the reference's contract
 * (decode.c:13-28: the packet is output or dropped inside Decode), so a mainloop linked unchanged (main.c:296-301)
 * sees every packet completed; a caller that calls Decode_Flush() opts into bursts with Decode_Set_Burst(n). */
static volatile uint32_t g_burst_cap = 1;
static pthread_key_t g_burst_key;
static pthread_once_t g_burst_once = PTHREAD_ONCE_INIT;
static __thread burst_t *t_burst = NULL;

/* Test hook (tests/test_compat_host.py only, not in the public headers): the next `k` allocations of the Decode
 * path fail, so the allocation-failure branches can be exercised without exhausting memory. */
static volatile uint32_t g_fail_alloc = 0;
void ppe_compat_debug_fail_alloc(uint32_t k) { __atomic_store_n(&g_fail_alloc, k, __ATOMIC_RELAXED); }
static int take_fail(void) {
    uint32_t k = __atomic_load_n(&g_fail_alloc, __ATOMIC_RELAXED);
    while (k)
        if (__atomic_compare_exchange_n(&g_fail_alloc, &k, k - 1, 0, __ATOMIC_RELAXED, __ATOMIC_RELAXED)) return 1;
    return 0;
}
static void *burst_alloc(size_t bytes, size_t align) {
    if (take_fail()) return NULL;
    return align ? aligned_alloc(align, (bytes + align - 1) / align * align) : malloc(bytes);
}

static int flush_burst(burst_t *b);

static void burst_exit(void *p) {  /* thread exit: deliver what the thread left queued, then free its burst */
    burst_t *b = (burst_t *)p;
    if (!b) return;
    flush_burst(b);
    /* a Decode() from a later TLS destructor of this thread must start a new burst, not touch this one */
    t_burst = NULL;
    free(b->m);
    free(b);
}

static void burst_key_init(void) { pthread_key_create(&g_burst_key, burst_exit); }

static burst_t *my_burst(void) {
    if (!t_burst) {
        pthread_once(&g_burst_once, burst_key_init);
        t_burst = (burst_t *)calloc(1, sizeof(burst_t));
        if (t_burst) pthread_setspecific(g_burst_key, t_burst);
    }
    return t_burst;
}

void Decode_Set_Burst(uint32_t n) {
    if (n) __atomic_store_n(&g_burst_cap, n, __ATOMIC_RELAXED);
}

/* statuses on which the reference calls DP_Log_Func before dropping */
static int logged_drop(uint32_t st) {
    switch (st) {
        case PPE_ST_L2_HEADER_ERR: case PPE_ST_VLAN_HEADER_ERR: case PPE_ST_IPV4_HEADER_ERR:
        case PPE_ST_IPV4_VERSION_ERR: case PPE_ST_IPV4_LEN_ERR: case PPE_ST_FRAG_LEN_ERR:
        case PPE_ST_UDP_HEADER_ERR: case PPE_ST_UDP_LEN_ERR: case PPE_ST_TCP_HEADER_ERR:
        case PPE_ST_TCP_LEN_ERR: case PPE_ST_ACL_DROP:
            return 1;
        default:
            return 0;
    }
}

/* The mbuf fields the reference's decoders write, exactly on the packets where they write them, from the kernel's
 * outputs for the packet (verdict, tuple) and its length.  Which layer wrote what follows from the terminal status:
 * the decoders run in order and each writes its fields once its own checks have passed.  Header pointers are the
 * packet's own addresses at the offsets the decoders use (IPV4_GET_HLEN / TCP_GET_HLEN read the same header bytes
 * the reference reads); no field is derived by re-decoding the packet here.  The stateless path has no flow object:
 * m->flow stays as it was (FlowHandlePacket sets it to the flow item, flow.c:306). */
static void fill_mbuf(mbuf_t *m, uint32_t v, uint32_t fhash, int32_t hit, const uint32_t *tu) {
    const uint32_t st = PPE_VERDICT_STATUS(v), fl = PPE_VERDICT_FLAGS(v);
    uint8_t *pkt = (uint8_t *)m->pkt_ptr;
    m->ppe_verdict = v;
    m->ppe_flow_hash = fhash;
    m->ppe_acl_hit = hit;
    if (!pkt || st == PPE_ST_L2_HEADER_ERR) return;  /* DecodeEthernet failed before writing anything */
    /* DecodeEthernet: decode-ethernet.c:57, 71-72 */
    m->ethh = pkt;
    memcpy(m->eth_dst, pkt, 6);
    memcpy(m->eth_src, pkt + 6, 6);
    if (fl & PPE_F_VLAN) {  /* DecodeVLAN passed its checks: decode-vlan.c:41, 46 */
        m->vlanh = pkt + 14;
        m->vlan_idx = 1;
    }
    if (st == PPE_ST_L2_UNSUPPORT || st == PPE_ST_VLAN_HEADER_ERR || st == PPE_ST_VLAN_LAYER_EXCEED ||
        st == PPE_ST_VLAN_UNSUPPORT)
        return;  /* never reached DecodeIPV4 */
    /* DecodeIPV4Packet: network_header once len >= 20 and the version is 4 (decode-ipv4.c:30-42): an
     * IPV4_HEADER_ERR is either check order's first failure (len < 20) or the header length (after :42) */
    const uint32_t l3off = 14u + ((fl & PPE_F_VLAN) ? 4u : 0u);
    const uint32_t l3len = ((m->pkt_totallen & 0xffffu) - l3off) & 0xffffu;
    if (st == PPE_ST_IPV4_VERSION_ERR || (st == PPE_ST_IPV4_HEADER_ERR && l3len < 20u)) return;
    uint8_t *l3 = pkt + l3off;
    m->network_header = l3;
    if (st == PPE_ST_IPV4_HEADER_ERR || st == PPE_ST_IPV4_LEN_ERR) return;
    /* every IPv4 check passed: decode-ipv4.c:62-63, 97 */
    m->ipv4.sip = tu[0];
    m->ipv4.dip = tu[1];
    m->proto = (uint8_t)tu[3];
    if (st == PPE_ST_FRAG || st == PPE_ST_FRAG_LEN_ERR) {  /* decode-ipv4.c:106-109 (Defrag reads them) */
        m->defrag_id = (uint16_t)tu[2];
        m->frag_offset = (uint16_t)(tu[2] >> 16);
        m->frag_len = (uint16_t)(tu[3] >> 16);
        return;
    }
    const int tcp = m->proto == 6u;
    if (st == PPE_ST_IPV4_UNSUPPORT || st == PPE_ST_UDP_HEADER_ERR || st == PPE_ST_TCP_HEADER_ERR) return;
    /* the L4 decoder's first length check passed: decode-udp.c:24, decode-tcp.c:146 */
    uint8_t *l4 = l3 + (l3[0] & 0x0fu) * 4u;
    m->transport_header = l4;
    if (!(fl & PPE_F_L4)) return;  /* UDP_LEN_ERR / TCP_LEN_ERR */
    /* decode-udp.c:38-45, decode-tcp.c:175-187 */
    m->sport = (uint16_t)tu[2];
    m->dport = (uint16_t)(tu[2] >> 16);
    m->payload_len = (uint16_t)(tu[3] >> 16);
    m->payload = l4 + (tcp ? (uint32_t)(l4[12] >> 4) * 4u : 8u);
    const uint32_t ws = PPE_TUPLE_WS(tu[3]);
    if (tcp && ws && !m->tcpvars.ws) {  /* DecodeTCPOptions' window-scale record (decode-tcp.c:61-70), found by the
                                          * kernel; like the reference, only into an mbuf with none recorded yet */
        uint8_t *o = l4 + ws;
        m->tcpvars.tcp_opts[0].type = o[0];
        m->tcpvars.tcp_opts[0].len = o[1];
        m->tcpvars.tcp_opts[0].data = o + 2;
        m->tcpvars.ws = &m->tcpvars.tcp_opts[0];
    }
    /* FlowHandlePacket found or created the flow (ACL passed): flow.c:294-307.  Every packet of the stateless path
     * is its flow's first, and FlowAdd orients the flow as that packet, so the direction is to-server. */
    if (st == PPE_ST_ACL_FW) m->flags |= PKT_TO_SERVER | PKT_HAS_FLOW;
}

/* Classify `n` mbufs on the GPU (serialised) and fill their parse fields; returns PPE_OK or a PPE_E* code. */
static int classify_mbufs(mbuf_t **mb, uint32_t n) {
    uint8_t *hdr = (uint8_t *)burst_alloc((size_t)n * PPE_COMPAT_STRIDE, 16);
    uint32_t *len = (uint32_t *)burst_alloc((size_t)n * 4, 0), *verdict = (uint32_t *)burst_alloc((size_t)n * 4, 0);
    uint32_t *fh = (uint32_t *)burst_alloc((size_t)n * 4, 0), *tuple = (uint32_t *)burst_alloc((size_t)n * 16, 0);
    uint64_t *ts = (uint64_t *)burst_alloc((size_t)n * 8, 0);
    int32_t *hit = (int32_t *)burst_alloc((size_t)n * 4, 0);
    int rc = PPE_ENOMEM;
    if (hdr && len && verdict && fh && tuple && ts && hit) {
        memset(hdr, 0, (size_t)n * PPE_COMPAT_STRIDE);
        for (uint32_t i = 0; i < n; i++) {
            mbuf_t *m = mb[i];
            const uint32_t c = m->pkt_totallen < PPE_COMPAT_STRIDE ? m->pkt_totallen : PPE_COMPAT_STRIDE;
            if (m->pkt_ptr && c) memcpy(hdr + (size_t)i * PPE_COMPAT_STRIDE, m->pkt_ptr, c);
            len[i] = m->pkt_totallen;
            ts[i] = m->timestamp;
        }
        ppe_batch_t b = {hdr, len, ts, n, PPE_COMPAT_STRIDE};
        ppe_result_t r;
        memset(&r, 0, sizeof r);
        r.verdict = verdict;
        r.flow_hash = fh;
        r.acl_hit = hit;
        r.tuple = tuple;
        ppe_cfg_t cfg = {unsupport_proto_action ? 1u : 0u, syn_check ? 1u : 0u, 0};
        pthread_mutex_lock(&g_ctx_lock);
        sync_running_locked();
        rc = g_ctx ? ppe_classify_host(g_ctx, &b, &r, &cfg, 0) : PPE_ENODEV;
        pthread_mutex_unlock(&g_ctx_lock);
        if (rc == PPE_OK)
            for (uint32_t i = 0; i < n; i++) fill_mbuf(mb[i], verdict[i], fh[i], hit[i], tuple + 4 * (size_t)i);
    }
    free(hdr);
    free(len);
    free(verdict);
    free(fh);
    free(tuple);
    free(ts);
    free(hit);
    return rc;
}

/* Take the burst's mbufs out (the burst is empty and reusable before any hook runs), classify, deliver.  The queued
 * array itself is taken, so a flush allocates nothing of its own: when the classify step cannot run (no context,
 * no memory, a GPU error), every taken mbuf still reaches the drop hook (decode.c:24-27; ppe_decode.h). */
static int flush_burst(burst_t *b) {
    const uint32_t n = b->n, alloc = b->alloc;
    if (n == 0) return 0;
    mbuf_t **mb = b->m;
    b->m = NULL;
    b->n = b->alloc = 0;
    const int rc = classify_mbufs(mb, n);
    for (uint32_t i = 0; i < n; i++) {
        mbuf_t *m = mb[i];
        if (rc != PPE_OK) {  /* undelivered: every packet ends in output_drop_proc (decode.c:24-27) */
            if (out_drop) out_drop(m);
            continue;
        }
        const uint32_t v = m->ppe_verdict;
        switch (PPE_VERDICT_ACTION(v)) {
            case PPE_ACT_FW:
                if (out_fw) out_fw(m);
                break;
            case PPE_ACT_DROP:
                if (logged_drop(PPE_VERDICT_STATUS(v))) DP_Log_Func(m);
                if (out_drop) out_drop(m);
                break;
            default:
                if (out_punt) out_punt(m);
                break;
        }
    }
    if (b == t_burst && !b->m) {  /* no hook queued anything meanwhile: the array goes back to the burst */
        b->m = mb;
        b->alloc = alloc;
    } else {
        free(mb);
    }
    return rc == PPE_OK ? (int)n : rc;
}

int Decode_Flush(void) {
    burst_t *b = t_burst;
    return b ? flush_burst(b) : 0;
}

void Decode(mbuf_t *m) {
    if (!m) return;
    burst_t *b = my_burst();
    const uint32_t cap = __atomic_load_n(&g_burst_cap, __ATOMIC_RELAXED);
    if (b && b->n >= b->alloc) {  /* grow to the current cap (or one more slot when the cap was lowered) */
        const uint32_t want = cap > b->n ? cap : b->n + 1;
        mbuf_t **nb = take_fail() ? NULL : (mbuf_t **)realloc(b->m, sizeof(mbuf_t *) * want);
        if (nb) {
            b->m = nb;
            b->alloc = want;
        }
    }
    if (!b || b->n >= b->alloc) {  /* no memory for the burst slot */
        if (out_drop) out_drop(m);
        return;
    }
    b->m[b->n++] = m;
    if (b->n >= cap) flush_burst(b);
}
