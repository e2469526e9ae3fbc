/*
 * ppe_oracle.c — TEST INFRASTRUCTURE ONLY (see ppe_oracle.h).  A sequential restatement of the reference
 * dataplane, layer by layer, with the reference's check order, uint16_t lengths and big-endian field reads
 * (the reference targets big-endian cnMIPS64 and reads header fields raw).
 */
#define _GNU_SOURCE
#include "ppe_oracle.h"

#include <pthread.h>
#include <sched.h>
#include <stdlib.h>
#include <string.h>

#include "ppe_hip.h"
#include "../packet-process-engine_amd/csrc/ppe_image.h"

#define DEC_OK 0
#define DEC_DROP 1

/* the mbuf fields the path touches (dataplane/src/include/mbuf.h:23-87) plus the recorded verdict */
typedef struct {
    const uint8_t *frame;
    uint32_t avail;
    uint64_t ts;
    const oracle_cfg_t *cfg;
    oracle_result_t *r;
    int vlan_idx;
    uint8_t smac[6], dmac[6];
    int decided;
    uint32_t totallen;  /* mbuf->pkt_totallen (FlowUpdate byte counts) */
} omb_t;

static const RCP_BLOCK_ACL_RULE_TUPLE *g_rules;
static const uint8_t *g_used;
static uint32_t g_nrules, g_defact = ACL_RULE_ACTION_DROP;
static const uint32_t *g_img;
static uint32_t g_img_words;

void oracle_set_rules(const RCP_BLOCK_ACL_RULE_TUPLE *rules, const uint8_t *used, uint32_t n,
                      uint32_t default_action) {
    g_rules = rules;
    g_used = used;
    g_nrules = n;
    g_defact = default_action;
}

void oracle_set_image(const uint32_t *img, uint32_t n_words) {
    g_img = img;
    g_img_words = n_words;
}

/* byte at frame offset `off`, tracking how far into the frame the verdict reads */
static uint32_t rd8(omb_t *m, const uint8_t *p) {
    const uint32_t off = (uint32_t)(p - m->frame);
    if (off + 1 > m->r->reach) m->r->reach = off + 1;
    return off < m->avail ? p[0] : 0u;
}
static uint32_t rd16(omb_t *m, const uint8_t *p) { return (rd8(m, p) << 8) | rd8(m, p + 1); }
static uint32_t rd32(omb_t *m, const uint8_t *p) { return (rd16(m, p) << 16) | rd16(m, p + 2); }

static void cnt(omb_t *m, int c) { m->r->counters |= 1u << c; }

/* output_fw_proc / output_drop_proc (dataplane/src/output/output.c:106,151): the first call decides */
static void out_fw(omb_t *m) {
    if (!m->decided) { m->r->action = PPE_ACT_FW; m->decided = 1; }
}
static void out_drop(omb_t *m) {
    if (!m->decided) { m->r->action = PPE_ACT_DROP; m->decided = 1; }
}
static void set_status(omb_t *m, uint32_t st) {
    if (m->r->status == 0xffu) m->r->status = st;
}

/* dataplane/src/decode/decode.c:31-45 */
static void unsupport_proto_handle(omb_t *m) {
    if (m->cfg->unsupport_proto_action == 1) out_fw(m);
    else out_drop(m);
}

/* dataplane/src/flow/tluhash.h:7-23 */
uint32_t oracle_tluhash(uint32_t u1, uint32_t u2) {
    uint32_t a = u2 + 0x9e3779b9u, b = u1 + 0x9e3779b9u, c = 0;
    a = a - b; a = a - c; a = a ^ (c >> 13);
    b = b - c; b = b - a; b = b ^ (a << 8);
    c = c - a; c = c - b; c = c ^ (b >> 13);
    a = a - b; a = a - c; a = a ^ (c >> 12);
    b = b - c; b = b - a; b = b ^ (a << 16);
    c = c - a; c = c - b; c = c ^ (b >> 5);
    a = a - b; a = a - c; a = a ^ (c >> 3);
    b = b - c; b = b - a; b = b ^ (a << 10);
    c = c - a; c = c - b; c = c ^ (b >> 15);
    return c;
}

/* dataplane/src/flow/tluhash.h:26-35 (argument order: proto, sip, dip, sport, dport) */
uint32_t oracle_flow_hashfn(uint32_t proto, uint32_t sip, uint32_t dip, uint32_t sport, uint32_t dport) {
    return oracle_tluhash(sip, sport & 0xffffu) ^ oracle_tluhash(dip, dport & 0xffffu) ^
           oracle_tluhash(proto & 0xffu, 0);
}

/* ---- ACL (the reference engine is absent) ---- */
static int prefix_match(uint32_t x, uint32_t rule_ip, uint32_t len) {
    if (len == 0) return 1;
    const uint32_t mask = len >= 32 ? 0xffffffffu : ~(0xffffffffu >> len);
    return ((x ^ rule_ip) & mask) == 0;
}
static int mac_zero(const uint8_t *a) { return (a[0] | a[1] | a[2] | a[3] | a[4] | a[5]) == 0; }

static int rule_matches(const RCP_BLOCK_ACL_RULE_TUPLE *r, uint32_t sip, uint32_t dip, uint32_t sport,
                        uint32_t dport, uint32_t proto, const uint8_t *dmac, const uint8_t *smac, uint64_t ts) {
    if (!prefix_match(sip, r->sip, r->sip_mask)) return 0;
    if (!prefix_match(dip, r->dip, r->dip_mask)) return 0;
    if (sport < r->sport_start || sport > r->sport_end) return 0;
    if (dport < r->dport_start || dport > r->dport_end) return 0;
    if (proto < r->protocol_start || proto > r->protocol_end) return 0;
    if (!mac_zero(r->smac) && memcmp(r->smac, smac, 6) != 0) return 0;
    if (!mac_zero(r->dmac) && memcmp(r->dmac, dmac, 6) != 0) return 0;
    if ((r->time_start != 0 || r->time_end != 0) && (ts < r->time_start || ts > r->time_end)) return 0;
    return 1;
}

int32_t oracle_acl_linear(uint32_t sip, uint32_t dip, uint32_t sport, uint32_t dport, uint32_t proto,
                          const uint8_t *dmac, const uint8_t *smac, uint64_t ts, uint32_t *action) {
    for (uint32_t i = 0; i < g_nrules; i++) {
        if (g_used && g_used[i] != RULE_ENTRY_STATUS_USED) continue;
        if (rule_matches(&g_rules[i], sip, dip, sport, dport, proto, dmac, smac, ts)) {
            if (action) *action = g_rules[i].action;
            return (int32_t)i;
        }
    }
    if (action) *action = g_defact;
    return -1;
}

static uint32_t mac_lo(const uint8_t *m) {
    return (uint32_t)m[0] | ((uint32_t)m[1] << 8) | ((uint32_t)m[2] << 16) | ((uint32_t)m[3] << 24);
}
static uint32_t mac_hi(const uint8_t *m) { return (uint32_t)m[4] | ((uint32_t)m[5] << 8); }

/* Walk of the device classifier image (format v4, packet-process-engine_amd/csrc/ppe_image.h): the same tree the
 * GPU walks, checked here against oracle_acl_linear (the definition).  Test infrastructure only. */
static int oracle_rule_match(const uint32_t *im, uint32_t slot, uint32_t sip, uint32_t dip, uint32_t sport,
                             uint32_t dport, uint32_t proto, const uint8_t *dmac, const uint8_t *smac, uint64_t ts) {
    const uint32_t *r = im + im[PPE_IMG_W_OFFRULES] + 8u * slot;
    int m = sip - r[0] <= r[1] && dip - r[2] <= r[3] && (uint16_t)(sport - (r[4] & 0xffffu)) <= (r[5] & 0xffffu) &&
            (uint16_t)(dport - (r[4] >> 16)) <= (r[5] >> 16) && proto - (r[6] & 0xffu) <= ((r[6] >> 8) & 0xffu);
    const uint32_t rs = r[7] >> 29;
    const uint32_t *x8 = im + im[PPE_IMG_W_OFFRESID] + 8u * slot;
    if (m && (rs & PPE_RESID_DMAC)) m = x8[0] == mac_lo(dmac) && x8[1] == mac_hi(dmac);
    if (m && (rs & PPE_RESID_SMAC)) m = x8[2] == mac_lo(smac) && x8[3] == mac_hi(smac);
    if (m && (rs & PPE_RESID_TIME)) {
        const uint64_t t0 = x8[4] | ((uint64_t)x8[5] << 32), t1 = x8[6] | ((uint64_t)x8[7] << 32);
        m = ts >= t0 && ts <= t1;
    }
    return m;
}

int32_t oracle_acl_tree(uint32_t sip, uint32_t dip, uint32_t sport, uint32_t dport, uint32_t proto,
                        const uint8_t *dmac, const uint8_t *smac, uint64_t ts, uint32_t *action) {
    const uint32_t *im = g_img;
    const uint32_t key[6] = {sip, dip, sport, dport, proto, 0u};
    uint32_t noff = 4u * im[PPE_IMG_W_OFFNODES], ks = im[PPE_IMG_W_ROOTKS] >> 8;
    const uint32_t jw = im[PPE_IMG_W_JUMP];
    if (jw) {  /* jump root (v4): bucket = key[dim] >> shift selects a subtree root */
        const uint32_t e = im[PPE_IMG_HDR_WORDS + (key[jw & 0xffu] >> ((jw >> 8) & 0xffu))];
        noff = e & 0xffffffu;
        ks = e >> 24;
    }
    const uint32_t *nd = im + noff / 4u;
    for (int it = 0; it <= PPE_MAX_DEPTH + 1; it++) {
        nd = im + noff / 4u;
        if (nd[0] == PPE_LEAF_THR) break;
        const int gt = key[ks] > nd[0];
        noff = gt ? nd[2] : nd[1];
        ks = ((gt ? nd[3] >> 16 : nd[3]) >> 8) & 0xffu;
    }
    const uint32_t max_leaf = im[PPE_IMG_W_MAXLEAF];
    uint32_t first = 0, cnt = 0;
    const uint32_t *lf = im + im[PPE_IMG_W_OFFLEAF];
    uint32_t one = nd[2];
    if (max_leaf <= 1) {
        lf = &one;  /* payload = the candidate slot, or the sentinel (n_rules: matches all, index -1, default) */
        cnt = 1;
    } else {
        first = nd[2] & 0xffffffu;
        cnt = nd[2] >> 24;
        if (cnt == PPE_LEAF_CNT_ESC) cnt = lf[first++];
    }
    for (uint32_t j = 0; j < cnt; j++) {
        const uint32_t slot = lf[first + j];
        if (oracle_rule_match(im, slot, sip, dip, sport, dport, proto, dmac, smac, ts)) {
            const uint32_t *r = im + im[PPE_IMG_W_OFFRULES] + 8u * slot;
            if (action) *action = r[6] >> 16;
            return (int32_t)(r[7] << 3) >> 3;
        }
    }
    if (action) *action = im[PPE_IMG_W_DEFACT];
    return -1;
}

static uint32_t oracle_rule_action(uint32_t id) { return id < g_nrules ? g_rules[id].action : 0u; }

/* Walk of the image's block section (format v5: 2-level blocks, what the GPU's multi-tile kernel walks), from the
 * same jump bucket; the leaf reached must be the binary walk's (test_acl_build.py checks all three walks agree). */
int32_t oracle_acl_blocks(uint32_t sip, uint32_t dip, uint32_t sport, uint32_t dport, uint32_t proto,
                          const uint8_t *dmac, const uint8_t *smac, uint64_t ts, uint32_t *action) {
    const uint32_t *im = g_img;
    const uint32_t key[6] = {sip, dip, sport, dport, proto, 0u};
    const uint32_t jw = im[PPE_IMG_W_JUMP];
    uint32_t b = jw ? im[im[PPE_IMG_W_OFFBSEC] + (key[jw & 0xffu] >> ((jw >> 8) & 0xffu))] : 0u;
    uint32_t x = 0;
    const uint32_t K = im[PPE_IMG_W_BLKLV] == 3u ? 3u : 2u, npos = (1u << K) - 1u;
    for (int it = 0; it <= PPE_MAX_DEPTH + 1; it++) {
        /* K levels per block: position p (children 2p + 1, 2p + 2), key slots at bits 4p of word 2^K - 1, exits
         * after it indexed by the K comparison bits (ppe_image.h) */
        const uint32_t *w = im + im[PPE_IMG_W_OFFBLOCKS] + (npos + 1u) * 2u * b;
        uint32_t p = 0, e = 0;
        for (uint32_t l = 0; l < K; l++) {
            const uint32_t bit = key[(w[npos] >> (4u * p)) & 0xfu] > w[p];
            e = 2u * e + bit;
            p = 2u * p + 1u + bit;
        }
        x = w[npos + 1u + e];
        if (x & PPE_BLK_LEAF) break;
        b = x;
    }
    x &= ~PPE_BLK_LEAF;
    if (im[PPE_IMG_W_OFFCREC]) {
        /* compact leaf (image v6): the exit's flags + the slot's 16-B record (prefix marker bits, port spans); only
         * TCP / UDP keys reach the ACL on the classify path, which is the only user of the block walk */
        const uint32_t slot = x & PPE_CX_SLOT;
        const uint32_t *r = im + im[PPE_IMG_W_OFFCREC] + PPE_CREC_WORDS * slot;
        const uint32_t ms = (x & PPE_CX_S32) ? ~0u : ~(((r[0] & (0u - r[0])) << 1) - 1u);
        const uint32_t md = (x & PPE_CX_D32) ? ~0u : ~(((r[1] & (0u - r[1])) << 1) - 1u);
        const int m = ((sip ^ r[0]) & ms) == 0 && ((dip ^ r[1]) & md) == 0 &&
                      (uint16_t)(sport - (r[2] & 0xffffu)) <= (r[3] & 0xffffu) &&
                      (uint16_t)(dport - (r[2] >> 16)) <= (r[3] >> 16) &&
                      (proto == 6 ? (x & PPE_CX_TCP) : proto == 17 ? (x & PPE_CX_UDP) : 0) != 0;
        const uint32_t id = im[PPE_IMG_W_OFFIDTAB] ? im[im[PPE_IMG_W_OFFIDTAB] + slot] : slot;
        const int drop = m ? (x & PPE_CX_DROP) != 0 : im[PPE_IMG_W_DEFACT] == ACL_RULE_ACTION_DROP;
        (void)dmac; (void)smac; (void)ts;
        /* the action word a drop-or-forward decision needs: the classify path compares it with DROP only */
        if (action) *action = m && !(x & PPE_CX_NOHIT) ? (drop ? ACL_RULE_ACTION_DROP : oracle_rule_action(id))
                                                        : im[PPE_IMG_W_DEFACT];
        return m && !(x & PPE_CX_NOHIT) ? (int32_t)id : -1;
    }
    const uint32_t max_leaf = im[PPE_IMG_W_MAXLEAF];
    const uint32_t *lf = im + im[PPE_IMG_W_OFFLEAF];
    uint32_t first = 0, cnt = 1, one = x;
    if (max_leaf <= 1) {
        lf = &one;
    } else {
        first = x & 0x7fffffu;
        cnt = (x >> 23) & 0xffu;
        if (cnt == PPE_LEAF_CNT_ESC) cnt = lf[first++];
    }
    for (uint32_t j = 0; j < cnt; j++) {
        const uint32_t slot = lf[first + j];
        if (oracle_rule_match(im, slot, sip, dip, sport, dport, proto, dmac, smac, ts)) {
            const uint32_t *r = im + im[PPE_IMG_W_OFFRULES] + 8u * slot;
            if (action) *action = r[6] >> 16;
            return (int32_t)(r[7] << 3) >> 3;
        }
    }
    if (action) *action = im[PPE_IMG_W_DEFACT];
    return -1;
}

/* Lookup in the image's cut lists (format v8, ppe_image.h): the bucket of the key's top sip / dip bits, then its
 * list's entries in priority order, each checked as a compact record (prefix marker bits, port spans, the exit's
 * protocol bits).  Like the compact leaf, only TCP / UDP keys reach it (the classify path). */
int32_t oracle_acl_cut(uint32_t sip, uint32_t dip, uint32_t sport, uint32_t dport, uint32_t proto,
                       const uint8_t *dmac, const uint8_t *smac, uint64_t ts, uint32_t *action) {
    const uint32_t *im = g_img;
    const uint32_t *h = im + im[PPE_IMG_W_OFFCUT];
    const uint32_t b0 = h[0] & 0xffu, b1 = (h[0] >> 8) & 0xffu;
    const uint32_t bk = ((sip >> (32u - b0)) << b1) | (dip >> (32u - b1));
    /* the bucket's list: the group's base + the bit-sliced lengths of the buckets before it in its group */
    const uint32_t *sl = im + h[4] + 4u * (bk >> 5);
    uint32_t first = im[h[8] + (bk >> 5)], cnt = 0;
    for (uint32_t k = 0; k <= (bk & 31u); k++) {
        uint32_t len = 0;
        for (uint32_t b = 0; b < 4u; b++) len |= ((sl[b] >> k) & 1u) << b;
        if (k < (bk & 31u)) first += len;
        else cnt = len;
    }
    const uint32_t ks = sip << b0, kd = dip << b1;
    const uint32_t ksb = (sip >> (31u - b0)) & 1u, kdb = (dip >> (31u - b1)) & 1u;
    const uint8_t *fp = (const uint8_t *)(im + h[9]);
    (void)dmac; (void)smac; (void)ts;
    for (uint32_t j = 0; j < cnt; j++) {
        const uint32_t e = first + j;
        const uint32_t *line = im + h[5] + PPE_CUT_LINE_WORDS * (e / h[7]);  /* 128-B line of h[7] entries + ids */
        const uint32_t *r = line + PPE_CUT_ENT_WORDS * (e % h[7]);
        /* the prefixes relative to the bucket: the bits above the marker (lowest set bit above the flag bits: TCP and
         * DROP at bits 0-1 of the sip word, UDP at bit 0 of the dip word) */
        const uint32_t sm = r[0] & ~3u, dm = r[1] & ~1u;
        const uint32_t ms = ~(((sm & (0u - sm)) << 1) - 1u), md = ~(((dm & (0u - dm)) << 1) - 1u);
        const int m = ((ks ^ sm) & ms) == 0 && ((kd ^ dm) & md) == 0 &&
                      (uint16_t)(sport - (r[2] & 0xffffu)) <= (r[3] & 0xffffu) &&
                      (uint16_t)(dport - (r[2] >> 16)) <= (r[3] >> 16) &&
                      (proto == 6 ? (r[0] & 1u) : proto == 17 ? (r[1] & 1u) : 0) != 0;
        /* the kernel skips an entry whose fingerprint rejects the key: such an entry must never match */
        const uint32_t f = (fp[e >> 1] >> (4u * (e & 1u))) & 15u;
        const int rejected = ((f & 2u) && (f & 1u) != ksb) || ((f & 8u) && ((f >> 2) & 1u) != kdb);
        if (rejected && m) return -2;  /* a fingerprint that would drop a match: an image error, reported as hit -2 */
        if (m) {
            /* the ids after the line's entries (PPE_CUT_LINES), else in the array at h[12] */
            const uint32_t *ids = (h[0] & PPE_CUT_LINES) ? line + PPE_CUT_ENT_WORDS * h[7] : im + h[12];
            const uint32_t k = (h[0] & PPE_CUT_LINES) ? e % h[7] : e;
            const uint32_t rid = (h[0] & PPE_CUT_IDS16) ? ((const uint16_t *)ids)[k] : ids[k];
            /* the entry's DROP flag must agree with the rule's action (the classify path compares it with DROP only) */
            const uint32_t act = oracle_rule_action(rid);
            if (((r[0] >> 1) & 1u) != (act == ACL_RULE_ACTION_DROP)) return -3;
            if (action) *action = act;
            return (int32_t)rid;
        }
    }
    if (action) *action = im[PPE_IMG_W_DEFACT];
    return -1;
}

/* ---- flow table: one core's flow_table[LOCAL_CPU_ID] (dataplane/src/flow/flow.c, flow.h) ----
 * FLOW_BUCKET_NUM chained buckets indexed by flow_hashfn & FLOW_BUCKET_MASK (flow.c:76-79, flow.h:87-88), items from
 * a fixed pool of `capacity` (the FPA flow-node pool, mem_pool.h:72), head insertion (FlowInsert, flow.c:69-72). */
#define OFLOW_BUCKETS 65536u
typedef struct oflow_item {
    struct oflow_item *next;
    uint64_t cycle;                               /* FLOW_UPDATE_TIMESTAMP: the batch time */
    uint32_t sip, dip;
    uint16_t sport, dport, protocol;
    uint64_t pkts2d, pktd2s, bytes2d, byted2s;    /* flow.h:66-69 */
} oflow_item_t;

struct oracle_flow {
    oflow_item_t *bucket[OFLOW_BUCKETS];
    oflow_item_t *pool, *free_list;
    uint32_t capacity;
    uint64_t live, new_flow, del_flow;
};

oracle_flow_t *oracle_flow_create(uint32_t capacity) {
    oracle_flow_t *f = (oracle_flow_t *)calloc(1, sizeof *f);
    if (!f) return NULL;
    f->capacity = capacity;
    f->pool = (oflow_item_t *)calloc(capacity ? capacity : 1, sizeof(oflow_item_t));
    if (!f->pool) {
        free(f);
        return NULL;
    }
    for (uint32_t i = 0; i < capacity; i++) {
        f->pool[i].next = f->free_list;
        f->free_list = &f->pool[i];
    }
    return f;
}

void oracle_flow_destroy(oracle_flow_t *f) {
    if (!f) return;
    free(f->pool);
    free(f);
}

/* FlowMatch, flow.c:81-94: the 5-tuple in either direction */
static int flow_match(const oflow_item_t *f, const oracle_result_t *r) {
    return (f->sip == r->sip && f->dip == r->dip && f->sport == r->sport && f->dport == r->dport &&
            f->protocol == r->proto) ||
           (f->sip == r->dip && f->dip == r->sip && f->sport == r->dport && f->dport == r->sport &&
            f->protocol == r->proto);
}

static __thread oracle_flow_t *t_flow;  /* table of the current batch (NULL: stateless, every packet a miss) */
static __thread uint64_t t_now;

static void flow_miss_drop(omb_t *m, uint32_t st, int c) {
    cnt(m, c);
    set_status(m, st);
    out_drop(m);  /* FlowHandlePacket: f == NULL → output_drop_proc, STAT_FLOW_PROC_FAIL, flow.c:278-284 */
    cnt(m, PPE_C_FLOW_PROC_FAIL);
}

/* ---- FlowHandlePacket, dataplane/src/flow/flow.c:271-310 with FlowGetFlowFromHash :181-245 ---- */
static __thread int t_use_tree;  /* per shard: 1 = walk the image's nodes, 2 = its blocks, 3 = its cut lists, 0 = linear
                                    first match */

static void flow_handle_packet(omb_t *m) {
    oracle_result_t *r = m->r;
    r->flags |= PPE_F_L4;
    r->flow_hash = oracle_flow_hashfn(r->proto, r->sip, r->dip, r->sport, r->dport);  /* flow.c:189 */
    oracle_flow_t *ft = t_flow;
    oflow_item_t *f = NULL;
    uint32_t b = r->flow_hash & (OFLOW_BUCKETS - 1u);
    if (ft) {  /* FlowFind, flow.c:96-115 */
        for (f = ft->bucket[b]; f; f = f->next)
            if (flow_match(f, r)) break;
    }
    if (f) {
        f->cycle = t_now;       /* flow.c:110 */
        cnt(m, PPE_C_ACL_FW);   /* flow.c:197-201 */
        set_status(m, PPE_ST_ACL_FW);
    } else {
        if (m->cfg->syn_check && r->proto == 6 && !(r->flags & PPE_F_SYN)) {  /* flow.c:204-214 */
            flow_miss_drop(m, PPE_ST_FLOW_TCP_NO_SYN_FIRST, PPE_C_FLOW_TCP_NO_SYN_FIRST);
            return;
        }
        /* PortScan_Detect disabled (portscan_able = 0) */
        uint32_t act;
        r->flags |= PPE_F_ACL;
        r->acl_hit = t_use_tree == 3 ? oracle_acl_cut(r->sip, r->dip, r->sport, r->dport, r->proto, m->dmac,
                                                       m->smac, m->ts, &act)
                   : t_use_tree == 2 ? oracle_acl_blocks(r->sip, r->dip, r->sport, r->dport, r->proto, m->dmac,
                                                          m->smac, m->ts, &act)
                   : t_use_tree ? oracle_acl_tree(r->sip, r->dip, r->sport, r->dport, r->proto, m->dmac, m->smac,
                                                  m->ts, &act)
                                : oracle_acl_linear(r->sip, r->dip, r->sport, r->dport, r->proto, m->dmac, m->smac,
                                                    m->ts, &act);
        if (act == ACL_RULE_ACTION_DROP) {  /* flow.c:232-237 */
            flow_miss_drop(m, PPE_ST_ACL_DROP, PPE_C_ACL_DROP);
            return;
        }
        cnt(m, PPE_C_ACL_FW);  /* flow.c:240 */
        set_status(m, PPE_ST_ACL_FW);
        if (ft) {  /* FlowAdd, flow.c:120-158 */
            f = ft->free_list;
            if (!f) {  /* flow.c:124-129 */
                cnt(m, PPE_C_FLOW_NODE_NOMEM);
                r->status = PPE_ST_FLOW_NOMEM;
                out_drop(m);
                cnt(m, PPE_C_FLOW_PROC_FAIL);
                return;
            }
            ft->free_list = f->next;
            memset(f, 0, sizeof *f);
            f->sip = r->sip;
            f->dip = r->dip;
            f->sport = (uint16_t)r->sport;
            f->dport = (uint16_t)r->dport;
            f->protocol = (uint16_t)r->proto;
            f->cycle = t_now;
            f->next = ft->bucket[b];  /* FlowInsert: hlist_add_head */
            ft->bucket[b] = f;
            ft->live++;
            ft->new_flow++;
            r->flags |= PPE_F_NEWFLOW;
        }
    }
    if (f) {
        /* FlowGetPacketDirection, flow.c:248-269 (TCP/UDP only reach here) */
        const int to_server = r->sport != r->dport ? f->sport == r->sport : f->sip == r->sip;
        r->flags |= PPE_F_FLOW | (to_server ? 0u : PPE_F_TOCLIENT);
        if (r->sport == f->sport) {  /* FlowUpdate, flow.c:163-178 */
            f->pkts2d++;
            f->bytes2d += m->totallen;
        } else {
            f->pktd2s++;
            f->byted2s += m->totallen;
        }
    }
    r->mset |= ORACLE_M_FLOW;    /* PKT_TO_SERVER / PKT_TO_CLIENT, PKT_HAS_FLOW: flow.c:294-307 */
    cnt(m, PPE_C_FLOW_PROC_OK);  /* flow.c:309 */
    out_fw(m);                   /* SELF_TEST, flow.c:376-377 */
}

/* FlowTimeOut + FlowAgeTimeoutCB, flow.c:391-467 (no flow is ever PERSISTENT) */
uint64_t oracle_flow_age(oracle_flow_t *ft, uint64_t now, uint64_t timeout) {
    uint64_t n = 0;
    for (uint32_t b = 0; b < OFLOW_BUCKETS; b++) {
        oflow_item_t **pp = &ft->bucket[b];
        while (*pp) {
            oflow_item_t *f = *pp;
            if (now > f->cycle && now - f->cycle > timeout) {
                *pp = f->next;
                f->next = ft->free_list;
                ft->free_list = f;
                ft->live--;
                ft->del_flow++;
                n++;
            } else {
                pp = &f->next;
            }
        }
    }
    return n;
}

uint32_t oracle_flow_dump(const oracle_flow_t *ft, ppe_flow_entry_t *out, uint32_t max) {
    uint32_t k = 0;
    for (uint32_t b = 0; b < OFLOW_BUCKETS; b++)
        for (const oflow_item_t *f = ft->bucket[b]; f; f = f->next, k++) {
            if (k >= max) continue;
            ppe_flow_entry_t *e = &out[k];
            memset(e, 0, sizeof *e);
            e->sip = f->sip;
            e->dip = f->dip;
            e->sport = f->sport;
            e->dport = f->dport;
            e->protocol = (uint8_t)f->protocol;
            e->pktcnts2d = f->pkts2d;
            e->pktcntd2s = f->pktd2s;
            e->bytecnts2d = f->bytes2d;
            e->bytecntd2s = f->byted2s;
            e->last_seen = f->cycle;
        }
    return k;
}

void oracle_flow_stats(const oracle_flow_t *ft, uint64_t *live, uint64_t *new_flow, uint64_t *del_flow) {
    if (live) *live = ft->live;
    if (new_flow) *new_flow = ft->new_flow;
    if (del_flow) *del_flow = ft->del_flow;
}

/* ---- UDP: dataplane/src/decode/decode-udp.c:16-71 ---- */
static int decode_udp(omb_t *m, const uint8_t *pkt, uint16_t len) {
    if (len < 8) {
        cnt(m, PPE_C_UDP_HEADERLEN_ERR);
        set_status(m, PPE_ST_UDP_HEADER_ERR);
        return DEC_DROP;
    }
    m->r->mset |= ORACLE_M_L4H;  /* transport_header, decode-udp.c:24 */
    m->r->l4off = (uint32_t)(pkt - m->frame);
    const uint32_t uh_len = rd16(m, pkt + 4);
    if (len < uh_len || len != uh_len) {
        cnt(m, PPE_C_UDP_PKTLEN_ERR);
        set_status(m, PPE_ST_UDP_LEN_ERR);
        return DEC_DROP;
    }
    m->r->sport = rd16(m, pkt);
    m->r->dport = rd16(m, pkt + 2);
    m->r->paylen = (uint16_t)(len - 8);
    m->r->mset |= ORACLE_M_L4;   /* sport, dport, payload, payload_len: decode-udp.c:38-45 */
    m->r->payoff = m->r->l4off + 8u;
    cnt(m, PPE_C_UDP_RX_OK);
    flow_handle_packet(m);
    return DEC_OK;
}

/* dataplane/src/decode/decode-tcp.c:18-131 — only the window-scale option is recorded (:61-70: the first valid one,
 * a duplicate is ignored), as its byte offset from the TCP header `th`; no verdict effect.  The reference reads the
 * whole option space (it lies inside the packet: hlen <= len, :149); here the frame holds `avail` bytes, so a parse
 * that needs a byte past them before it has found the option records opt_past (what the kernel reports as
 * PPE_TUPLE_OPT_PAST for a narrower header window).  The first valid option is final, so the parse stops there. */
static void decode_tcp_options(omb_t *m, const uint8_t *th, const uint8_t *pkt, uint16_t len) {
    uint16_t plen = len;
    while (plen) {
        const uint32_t off = (uint32_t)(pkt - m->frame);
        if (off >= m->avail) { m->r->opt_past = 1; return; }
        const uint8_t t = pkt[0];
        if (t == 0) break;          /* EOL */
        if (t == 1) { pkt++; plen--; continue; }  /* NOP */
        if (plen < 2) break;
        if (off + 1 >= m->avail) { m->r->opt_past = 1; return; }
        const uint8_t ol = pkt[1];
        if (ol > plen || ol < 2) return;  /* invalid length: return -1 (:43-46) */
        if (t == 3 && ol == 3) {    /* m->tcpvars.ws = &m->TCP_OPTS[0] (:63-70) */
            m->r->tcp_ws = (uint32_t)(pkt - th);
            m->r->mset |= ORACLE_M_WS;
            return;
        }
        pkt += ol;
        plen = (uint16_t)(plen - ol);
    }
}

/* ---- TCP: dataplane/src/decode/decode-tcp.c:135-222 ---- */
static int decode_tcp(omb_t *m, const uint8_t *pkt, uint16_t len) {
    if (len < 20) {
        cnt(m, PPE_C_TCP_HEADERLEN_ERR);
        set_status(m, PPE_ST_TCP_HEADER_ERR);
        return DEC_DROP;
    }
    m->r->mset |= ORACLE_M_L4H;  /* transport_header, decode-tcp.c:146 */
    m->r->l4off = (uint32_t)(pkt - m->frame);
    const uint8_t hlen = (uint8_t)((rd8(m, pkt + 12) >> 4) << 2);
    if (len < hlen) {
        cnt(m, PPE_C_TCP_PKTLEN_ERR);
        set_status(m, PPE_ST_TCP_LEN_ERR);
        return DEC_DROP;
    }
    const uint8_t opt_len = (uint8_t)(hlen - 20);
    if (opt_len > 40) {
        cnt(m, PPE_C_TCP_PKTLEN_ERR);
        set_status(m, PPE_ST_TCP_LEN_ERR);
        return DEC_DROP;
    }
    m->r->flags |= PPE_F_TCP;
    if (rd8(m, pkt + 13) & 0x02) m->r->flags |= PPE_F_SYN;  /* land / SYN-flood monitors pass at default config */
    if (opt_len > 0) decode_tcp_options(m, pkt, pkt + 20, opt_len);
    m->r->sport = rd16(m, pkt);
    m->r->dport = rd16(m, pkt + 2);
    m->r->paylen = (uint16_t)(len - hlen);
    m->r->mset |= ORACLE_M_L4;   /* sport, dport, payload, payload_len: decode-tcp.c:179-187 */
    m->r->payoff = m->r->l4off + hlen;
    cnt(m, PPE_C_TCP_RX_OK);
    flow_handle_packet(m);
    return DEC_OK;
}

/* ---- IPv4: dataplane/src/decode/decode-ipv4.c:27-247 ---- */
static int decode_ipv4(omb_t *m, const uint8_t *pkt, uint16_t len) {
    oracle_result_t *r = m->r;
    if (len < 20) {
        cnt(m, PPE_C_IPV4_HEADERLEN_ERR);
        set_status(m, PPE_ST_IPV4_HEADER_ERR);
        return DEC_DROP;
    }
    const uint32_t verhl = rd8(m, pkt);
    if ((verhl >> 4) != 4) {
        cnt(m, PPE_C_IPV4_VERSION_ERR);
        set_status(m, PPE_ST_IPV4_VERSION_ERR);
        return DEC_DROP;
    }
    r->mset |= ORACLE_M_L3;       /* network_header, decode-ipv4.c:42 */
    r->l3off = (uint32_t)(pkt - m->frame);
    const uint32_t hl = (verhl & 0x0f) << 2;
    if (hl < 20) {
        cnt(m, PPE_C_IPV4_HEADERLEN_ERR);
        set_status(m, PPE_ST_IPV4_HEADER_ERR);
        return DEC_DROP;
    }
    const uint32_t ip_len = rd16(m, pkt + 2);
    if (ip_len < hl || len < ip_len) {
        cnt(m, PPE_C_IPV4_PKTLEN_ERR);
        set_status(m, PPE_ST_IPV4_LEN_ERR);
        return DEC_DROP;
    }
    r->sip = rd32(m, pkt + 12);
    r->dip = rd32(m, pkt + 16);
    r->proto = rd8(m, pkt + 9);
    r->mset |= ORACLE_M_IP;       /* ipv4.sip / dip, proto: decode-ipv4.c:62-63, 97 */
    const uint32_t ip_off = rd16(m, pkt + 6);
    if (((ip_off & 0x1fff) > 0 || ((ip_off & 0x2000) >> 13) == 1) && r->proto != 89) {
        r->flags |= PPE_F_FRAG;
        const uint16_t frag_len = (uint16_t)(len - hl);
        r->mset |= ORACLE_M_FRAG;  /* decode-ipv4.c:106-109 */
        r->frag_id = rd16(m, pkt + 4);
        r->frag_off = (uint16_t)((ip_off & 0x1fff) << 3);
        r->frag_len = frag_len;
        if (frag_len == 0) {
            cnt(m, PPE_C_FRAG_FRAGLEN_ERR);
            set_status(m, PPE_ST_FRAG_LEN_ERR);
            return DEC_DROP;
        }
        /* Defrag(): stateful, out of scope — the packet is handed to the host (PUNT); Defrag returning NULL
         * makes DecodeIPV4 return DECODE_OK with no output call */
        cnt(m, PPE_C_FRAG_PUNT);
        set_status(m, PPE_ST_FRAG);
        r->action = PPE_ACT_PUNT;
        m->decided = 1;
        return DEC_OK;
    }
    const uint16_t l4len = (uint16_t)(ip_len - hl);
    switch (r->proto) {
        case 6:
            cnt(m, PPE_C_IPV4_RX_OK);
            if (decode_tcp(m, pkt + hl, l4len) != DEC_OK) out_drop(m);
            return DEC_OK;
        case 17:
            cnt(m, PPE_C_IPV4_RX_OK);
            /* DP_Attack_UdpPacketMonitor passes at default config */
            if (decode_udp(m, pkt + hl, l4len) != DEC_OK) out_drop(m);
            return DEC_OK;
        default:
            cnt(m, PPE_C_IPV4_UNSUPPORT);
            set_status(m, PPE_ST_IPV4_UNSUPPORT);
            unsupport_proto_handle(m);
            return DEC_OK;
    }
}

/* ---- VLAN: dataplane/src/decode/decode-vlan.c:23-89 ---- */
static int decode_vlan(omb_t *m, const uint8_t *pkt, uint16_t len) {
    if (len < 4) {
        cnt(m, PPE_C_VLAN_HEADERLEN_ERR);
        set_status(m, PPE_ST_VLAN_HEADER_ERR);
        return DEC_DROP;
    }
    if (m->vlan_idx >= 1) {
        cnt(m, PPE_C_VLAN_LAYER_EXCEED);
        set_status(m, PPE_ST_VLAN_LAYER_EXCEED);
        return DEC_DROP;
    }
    const uint32_t proto = rd16(m, pkt + 2);
    m->vlan_idx = 1;
    m->r->flags |= PPE_F_VLAN;
    m->r->mset |= ORACLE_M_VLAN;  /* vlanh, vlan_idx: decode-vlan.c:41, 46 */
    switch (proto) {
        case 0x0800:
            cnt(m, PPE_C_VLAN_RX_OK);
            return decode_ipv4(m, pkt + 4, (uint16_t)(len - 4));
        case 0x8100:
        case 0x9100:
            cnt(m, PPE_C_VLAN_RX_OK);
            return decode_vlan(m, pkt + 4, (uint16_t)(len - 4));
        default:
            cnt(m, PPE_C_VLAN_UNSUPPORT);
            set_status(m, PPE_ST_VLAN_UNSUPPORT);
            unsupport_proto_handle(m);
            return DEC_OK;
    }
}

/* ---- Ethernet: dataplane/src/decode/decode-ethernet.c:23-115 ---- */
static int decode_ethernet(omb_t *m, const uint8_t *pkt, uint16_t len) {
    if (len < 14) {
        cnt(m, PPE_C_L2_HEADERLEN_ERR);
        set_status(m, PPE_ST_L2_HEADER_ERR);
        return DEC_DROP;
    }
    int dz = 1, sz = 1;
    for (int i = 0; i < 6; i++) {
        m->dmac[i] = (uint8_t)rd8(m, pkt + i);
        m->smac[i] = (uint8_t)rd8(m, pkt + 6 + i);
        dz &= m->dmac[i] == 0;
        sz &= m->smac[i] == 0;
    }
    if (dz || sz) {
        cnt(m, PPE_C_L2_HEADERLEN_ERR);
        set_status(m, PPE_ST_L2_HEADER_ERR);
        return DEC_DROP;
    }
    m->r->mset |= ORACLE_M_ETH;   /* ethh, eth_dst, eth_src: decode-ethernet.c:57, 71-72 */
    switch (rd16(m, pkt + 12)) {
        case 0x0800:
            cnt(m, PPE_C_L2_RX_OK);
            return decode_ipv4(m, pkt + 14, (uint16_t)(len - 14));
        case 0x8100:
        case 0x9100:
            cnt(m, PPE_C_L2_RX_OK);
            return decode_vlan(m, pkt + 14, (uint16_t)(len - 14));
        default:
            cnt(m, PPE_C_L2_UNSUPPORT);
            set_status(m, PPE_ST_L2_UNSUPPORT);
            unsupport_proto_handle(m);
            return DEC_OK;
    }
}

void oracle_classify(const uint8_t *pkt, uint32_t avail, uint32_t len, uint64_t ts, const oracle_cfg_t *cfg,
                     oracle_result_t *out) {
    memset(out, 0, sizeof *out);
    out->status = 0xffu;
    out->acl_hit = -1;
    out->action = PPE_ACT_DROP;
    omb_t m;
    memset(&m, 0, sizeof m);
    m.frame = pkt;
    m.avail = avail;
    m.ts = ts;
    m.cfg = cfg;
    m.r = out;
    m.totallen = len;
    out->counters |= 1u << PPE_C_PKTS;
    /* Decode(): dataplane/src/decode/decode.c:19-28, len = (uint16_t)pkt_totallen */
    if (decode_ethernet(&m, pkt, (uint16_t)len) != DEC_OK) out_drop(&m);
    switch (out->action) {
        case PPE_ACT_FW: cnt(&m, PPE_C_OUT_FW); break;
        case PPE_ACT_DROP: cnt(&m, PPE_C_OUT_DROP); break;
        default: cnt(&m, PPE_C_OUT_PUNT); break;
    }
}

/* ---- batch + threads (the CPU baseline: run-to-completion shards, like per-core mainloop, main.c:250) ---- */
typedef struct {
    const uint8_t *hdr;
    uint32_t stride;
    const uint32_t *len;
    const uint64_t *ts;
    uint32_t lo, hi;
    const oracle_cfg_t *cfg;
    int use_tree;
    oracle_flow_t *flow;
    uint32_t *verdict, *flow_hash, *tuple, *reach;
    int32_t *acl_hit;
    uint64_t counters[32];
} shard_t;

static void *run_shard(void *arg) {
    shard_t *s = (shard_t *)arg;
    t_use_tree = s->use_tree;
    t_flow = s->flow;
    t_now = s->cfg->now_seconds;
    memset(s->counters, 0, sizeof s->counters);
    for (uint32_t i = s->lo; i < s->hi; i++) {
        oracle_result_t r;
        const uint32_t len = s->len[i];
        const uint32_t avail = len < s->stride ? len : s->stride;
        oracle_classify(s->hdr + (size_t)i * s->stride, avail, len, s->ts ? s->ts[i] : s->cfg->now_seconds, s->cfg,
                        &r);
        if (s->verdict) s->verdict[i] = r.status | (r.action << 8) | (r.flags << 16);
        if (s->flow_hash) s->flow_hash[i] = r.flow_hash;
        if (s->acl_hit) s->acl_hit[i] = r.acl_hit;
        if (s->reach) s->reach[i] = r.reach;
        if (s->tuple) {
            s->tuple[4 * (size_t)i + 0] = r.sip;
            s->tuple[4 * (size_t)i + 1] = r.dip;
            /* ppe_hip.h ppe_result_t.tuple (ABI 5): a fragment's word 2 / length field carry its Defrag fields */
            const int fr = (r.mset & ORACLE_M_FRAG) != 0;
            s->tuple[4 * (size_t)i + 2] = fr ? (r.frag_id | (r.frag_off << 16)) : (r.sport | (r.dport << 16));
            s->tuple[4 * (size_t)i + 3] = r.proto | (((r.flags & PPE_F_VLAN) ? 1u : 0u) << 8) | (r.tcp_ws << 9) |
                                          (r.opt_past ? PPE_TUPLE_OPT_PAST : 0u) | ((fr ? r.frag_len : r.paylen) << 16);
        }
        for (int c = 0; c < 32; c++)
            if (r.counters & (1u << c)) s->counters[c]++;
        s->counters[PPE_C_RX_BYTES] += len;  /* STAT_RECV_PB_ADD(m->pkt_totallen), oct-rxtx.c:213 */
    }
    return NULL;
}

/* CPU pinning of the shard threads (the reference pins one mainloop pthread per core, main.c:422-425,
 * dataplane/src/platform/oct-thread.c:18-55): thread t runs on g_pin[t % g_npin]; none when g_npin == 0 */
static int g_pin[1024];
static int g_npin = 0;

int oracle_set_pin_cpus(const int *cpus, int n) {
    if (n < 0 || n > 1024) return -1;
    for (int i = 0; i < n; i++) g_pin[i] = cpus[i];
    g_npin = n;
    return 0;
}

static void pin_attr(pthread_attr_t *at, int t) {
    if (g_npin <= 0) return;
    cpu_set_t cs;
    CPU_ZERO(&cs);
    CPU_SET(g_pin[t % g_npin], &cs);
    pthread_attr_setaffinity_np(at, sizeof cs, &cs);
}

int oracle_classify_batch(const uint8_t *hdr, uint32_t stride, const uint32_t *len, const uint64_t *ts, uint32_t n,
                          const oracle_cfg_t *cfg, int nthreads, int use_tree, uint32_t *verdict,
                          uint32_t *flow_hash, int32_t *acl_hit, uint32_t *tuple, uint32_t *reach,
                          uint64_t *counters) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 512) nthreads = 512;
    shard_t *sh = (shard_t *)calloc((size_t)nthreads, sizeof(shard_t));
    pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
    if (!sh || !th) {
        free(sh);
        free(th);
        return -1;
    }
    const uint32_t per = (n + (uint32_t)nthreads - 1) / (uint32_t)nthreads;
    for (int t = 0; t < nthreads; t++) {
        shard_t *s = &sh[t];
        s->hdr = hdr;
        s->stride = stride;
        s->len = len;
        s->ts = ts;
        s->lo = (uint32_t)t * per < n ? (uint32_t)t * per : n;
        s->hi = s->lo + per < n ? s->lo + per : n;
        s->cfg = cfg;
        s->use_tree = use_tree;
        s->verdict = verdict;
        s->flow_hash = flow_hash;
        s->acl_hit = acl_hit;
        s->tuple = tuple;
        s->reach = reach;
        if (nthreads == 1 && g_npin == 0) {
            run_shard(s);
        } else {
            pthread_attr_t at;
            pthread_attr_init(&at);
            pin_attr(&at, t);
            pthread_create(&th[t], &at, run_shard, s);
            pthread_attr_destroy(&at);
        }
    }
    if (nthreads > 1 || g_npin > 0)
        for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
    if (counters) {
        memset(counters, 0, 32 * sizeof(uint64_t));
        for (int t = 0; t < nthreads; t++)
            for (int c = 0; c < 32; c++) counters[c] += sh[t].counters[c];
    }
    free(sh);
    free(th);
    return 0;
}

/* The batch through one core's flow table, in index order (one shard: the table is per core). */
int oracle_flow_classify_batch(oracle_flow_t *ft, const uint8_t *hdr, uint32_t stride, const uint32_t *len,
                               const uint64_t *ts, uint32_t n, const oracle_cfg_t *cfg, int use_tree,
                               uint32_t *verdict, uint32_t *flow_hash, int32_t *acl_hit, uint32_t *tuple,
                               uint64_t *counters) {
    shard_t s;
    memset(&s, 0, sizeof s);
    s.hdr = hdr;
    s.stride = stride;
    s.len = len;
    s.ts = ts;
    s.lo = 0;
    s.hi = n;
    s.cfg = cfg;
    s.use_tree = use_tree;
    s.flow = ft;
    s.verdict = verdict;
    s.flow_hash = flow_hash;
    s.acl_hit = acl_hit;
    s.tuple = tuple;
    run_shard(&s);
    t_flow = NULL;
    if (counters) memcpy(counters, s.counters, sizeof s.counters);
    return 0;
}
