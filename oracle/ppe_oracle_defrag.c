/*
 * ppe_oracle_defrag.c — TEST INFRASTRUCTURE ONLY.  Sequential CPU restatement of the reference's IPv4 reassembly
 * (dataplane/src/decode/decode-defrag.c) for one core, used by tests/ and bench.py's cpu_baseline leg as the checker
 * of ppe_defrag (libppe_hip.so never links or calls it).
 *
 * Pinning: decode-defrag.c needs the Cavium SDK, the FPA / mem_pool allocators and the hlist / jhash headers, which
 * cannot be built here without stand-ins (forbidden), and the reference ships no defrag tests or fixtures.  PARITY
 * UNPINNED by reference outputs: this restatement is pinned by hand-derived known answers
 * (tests/test_oracle_defrag.py), each citing the reference line it exercises.
 *
 * Follows, per fragment in arrival order:
 *   Defrag                 decode-defrag.c:449-487   find the FCB of (sip, dip, ip_id) or create it (cap fcb_max)
 *   Frag_defrag_begin      decode-defrag.c:412-446   HW2SW copy (frame <= frag_buf), DELETE check, cache_max check
 *   Frag_defrag_process    decode-defrag.c:292-406   last-fragment / total checks, chain position (the scan compares
 *                                                    a chained fragment's frag_len with the new offset, :344-349),
 *                                                    overlap checks, insert, FIRST_IN, completion test
 *   Frag_defrag_reasm      decode-defrag.c:222-289   head frame + later payloads, ip_len, ip_off = 0, checksum
 *   Frag_defrag_setup      decode-defrag.c:164-219   buffer of total + L2 + ihl*4 bytes (<= reasm_buf), ICMP 1000
 *   Frag_defrag_timeout    decode-defrag.c:490-551   free DELETE FCBs and those idle past the timeout
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "ppe_oracle.h"

#define OD_FIRST_IN 1u
#define OD_LAST_IN 2u
#define OD_COMPLETE 4u
#define OD_DELETE 8u
#define OD_BUCKETS 1024u   /* FRAG_BUCKET_NUM (decode-defrag.h:86) */

typedef struct od_frag {
    struct od_frag *next;
    uint8_t *frame;          /* HW2SW copy */
    uint32_t totlen;
    uint32_t offset, flen, l2, ihl4, proto;
    uint64_t id;
} od_frag_t;

typedef struct od_fcb {
    struct od_fcb *hnext;    /* bucket chain (hlist_add_head order) */
    od_frag_t *fragments, *tail;
    uint64_t cycle;
    uint32_t sip, dip, id;
    uint32_t status;         /* OD_COMPLETE | OD_DELETE */
    int total_fraglen, meat;
    uint32_t cache_num;
    uint32_t last_in;
} od_fcb_t;

struct oracle_defrag {
    uint32_t fcb_max, cache_max, frag_buf, reasm_buf;
    od_fcb_t *bucket[OD_BUCKETS];
    uint64_t running, new_fcb, del_fcb, st[PPE_DF__COUNT], teardrop, timeout_drop, datagrams;
};

static uint32_t be16(const uint8_t *p) { return ((uint32_t)p[0] << 8) | p[1]; }
static uint32_t be32(const uint8_t *p) { return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3]; }

oracle_defrag_t *oracle_defrag_create(uint32_t fcb_max, uint32_t cache_max, uint32_t frag_buf, uint32_t reasm_buf) {
    oracle_defrag_t *d = calloc(1, sizeof(*d));
    if (!d) return NULL;
    d->fcb_max = fcb_max ? fcb_max : 1024;
    d->cache_max = cache_max ? cache_max : 8;
    d->frag_buf = frag_buf ? frag_buf : 2024;
    d->reasm_buf = reasm_buf ? reasm_buf : 8168;
    return d;
}

static void free_frags(od_frag_t *f) {
    while (f) {
        od_frag_t *n = f->next;
        free(f->frame);
        free(f);
        f = n;
    }
}

void oracle_defrag_destroy(oracle_defrag_t *d) {
    if (!d) return;
    for (uint32_t b = 0; b < OD_BUCKETS; ++b) {
        od_fcb_t *f = d->bucket[b];
        while (f) {
            od_fcb_t *n = f->hnext;
            free_frags(f->fragments);
            free(f);
            f = n;
        }
    }
    free(d);
}

static uint32_t bucket_of(uint32_t sip, uint32_t dip, uint32_t id) {
    uint32_t h = sip * 2654435761u ^ dip * 2246822519u ^ id * 3266489917u;
    return (h ^ (h >> 16)) & (OD_BUCKETS - 1);
}

/* The parse DecodeEthernet / DecodeVLAN / DecodeIPV4Packet / DecodeIPV4 perform before Defrag; 0 = not a fragment
 * Defrag would see. */
static int parse(const uint8_t *p, uint32_t tot, od_frag_t *f, uint32_t *sip, uint32_t *dip, uint32_t *id,
                 uint32_t *mf) {
    const uint32_t L = tot & 0xffffu;   /* Decode: (uint16_t)pkt_totallen (decode.c:25) */
    if (L < 14) return 0;
    int z0 = 1, z1 = 1;
    for (int b = 0; b < 6; ++b) {
        if (p[b]) z0 = 0;
        if (p[6 + b]) z1 = 0;
    }
    if (z0 || z1) return 0;
    uint32_t l2 = 14, et = be16(p + 12);
    if (et == 0x8100u || et == 0x9100u) {
        if (L - 14 < 4 || be16(p + 16) != 0x0800u) return 0;
        l2 = 18;
    } else if (et != 0x0800u) {
        return 0;
    }
    if (L < l2 + 20) return 0;
    const uint8_t *ip = p + l2;
    const uint32_t l3 = L - l2, ihl4 = (ip[0] & 15u) * 4u, iplen = be16(ip + 2), offw = be16(ip + 6);
    if ((ip[0] >> 4) != 4u || ihl4 < 20 || iplen < ihl4 || l3 < iplen) return 0;
    if (!((offw & 0x1fffu) || (offw & 0x2000u)) || ip[9] == 89u) return 0;   /* IPV4_IS_FRAGMENT, not OSPF */
    const uint32_t flen = (l3 - ihl4) & 0xffffu;
    if (flen == 0) return 0;                                                 /* STAT_FRAG_LEN_ERR upstream */
    f->totlen = tot;
    f->offset = (offw & 0x1fffu) << 3;
    f->flen = flen;
    f->l2 = l2;
    f->ihl4 = ihl4;
    f->proto = ip[9];
    *sip = be32(ip + 12);
    *dip = be32(ip + 16);
    *id = be16(ip + 4);
    *mf = (offw >> 13) & 1u;
    return 1;
}

/* IPV4CalculateChecksum (decode-ipv4.h:117-163) over big-endian 16-bit words, skipping the checksum word */
static uint32_t ip_csum(const uint8_t *h, uint32_t hlen) {
    uint32_t cs = 0;
    for (uint32_t o = 0; o < 20; o += 2)
        if (o != 10) cs += be16(h + o);
    for (uint32_t o = 20; o < hlen; o += 2) cs += be16(h + o);
    cs = (cs >> 16) + (cs & 0xffffu);
    cs += cs >> 16;
    return (~cs) & 0xffffu;
}

uint32_t oracle_defrag_batch(oracle_defrag_t *d, const uint8_t *pkt, const uint64_t *off, const uint32_t *len,
                             const uint64_t *ids, uint32_t n, uint64_t now, uint32_t *status, uint32_t *dgram_of,
                             uint8_t *dgram_pkt, uint32_t *dgram_len, uint64_t *dgram_frags) {
    uint32_t nd = 0;
    for (uint32_t i = 0; i < n; ++i) {
        const uint8_t *p = pkt + off[i];
        od_frag_t tmp;
        memset(&tmp, 0, sizeof(tmp));
        uint32_t sip, dip, id, mf;
        if (dgram_of) dgram_of[i] = 0xffffffffu;
        if (!parse(p, len[i], &tmp, &sip, &dip, &id, &mf)) {
            status[i] = PPE_DF_NOT_FRAG;
            d->st[PPE_DF_NOT_FRAG]++;
            continue;
        }
        tmp.id = ids ? ids[i] : i;
        /* Defrag: FragFind, else fcb_create + fcb_insert */
        const uint32_t b = bucket_of(sip, dip, id);
        od_fcb_t *fcb = d->bucket[b];
        while (fcb && !(fcb->id == id && fcb->sip == sip && fcb->dip == dip)) fcb = fcb->hnext;
        if (!fcb) {
            if (d->running >= d->fcb_max) {   /* fetch-and-add, fail at DEFRAG_FCB_MAX (decode-defrag.c:76-82) */
                status[i] = PPE_DF_FCB_FULL;
                d->st[PPE_DF_FCB_FULL]++;
                continue;
            }
            d->running++;
            d->new_fcb++;
            fcb = calloc(1, sizeof(*fcb));
            fcb->sip = sip;
            fcb->dip = dip;
            fcb->id = id;
            fcb->hnext = d->bucket[b];
            d->bucket[b] = fcb;
        }
        fcb->cycle = now;   /* FCB_UPDATE_TIMESTAMP (FragFind :139, Defrag :472) */
        /* Frag_defrag_begin */
        if (tmp.totlen > d->frag_buf) {            /* PACKET_HW2SW: MEM_2K_ALLOC(pkt_totallen) fails */
            status[i] = PPE_DF_HW2SW_ERR;
            d->st[PPE_DF_HW2SW_ERR]++;
            continue;
        }
        if (fcb->status & OD_DELETE) {
            status[i] = PPE_DF_DELETED;
            d->st[PPE_DF_DELETED]++;
            continue;
        }
        if (fcb->cache_num >= d->cache_max) {
            status[i] = PPE_DF_CACHE_FULL;
            d->st[PPE_DF_CACHE_FULL]++;
            continue;
        }
        /* Frag_defrag_process */
        const int offset = (int)tmp.offset, end = offset + (int)tmp.flen;
        int err = 0, tear = 0;
        if (fcb->last_in & OD_COMPLETE) err = 1;   /* never set on last_in in the reference (:299-300) */
        if (!err) {
            if (!mf) {
                if (end < fcb->total_fraglen || (fcb->last_in & OD_LAST_IN)) err = 1;
                else {
                    fcb->last_in |= OD_LAST_IN;
                    fcb->total_fraglen = end;
                }
            } else if (end > fcb->total_fraglen) {
                if (fcb->last_in & OD_LAST_IN) err = 1;
                else fcb->total_fraglen = end;
            }
        }
        od_frag_t *prev = NULL, *next = NULL;
        if (!err) {
            prev = fcb->tail;
            if (!prev || (int)prev->offset < offset) {
                next = NULL;
            } else {
                prev = NULL;
                for (next = fcb->fragments; next; next = next->next) {
                    if ((int)next->flen >= offset) break;   /* sic: frag_len, decode-defrag.c:346 */
                    prev = next;
                }
            }
            if (prev && (int)(prev->offset + prev->flen) - offset > 0) err = tear = 1;
            if (!err && next && (int)next->offset - end < 0) err = tear = 1;
        }
        if (err) {
            status[i] = PPE_DF_DEFRAG_ERR | (tear ? PPE_DF_TEARDROP : 0u);
            d->st[PPE_DF_DEFRAG_ERR]++;
            d->teardrop += (uint64_t)tear;
            continue;
        }
        od_frag_t *f = malloc(sizeof(*f));
        *f = tmp;
        f->frame = malloc(tmp.totlen ? tmp.totlen : 1);
        memcpy(f->frame, p, tmp.totlen);
        f->next = next;
        if (!next) fcb->tail = f;
        if (prev) prev->next = f;
        else fcb->fragments = f;
        fcb->cache_num++;
        fcb->meat += (int)f->flen;
        if (offset == 0) fcb->last_in |= OD_FIRST_IN;
        if (!(fcb->last_in == (OD_FIRST_IN | OD_LAST_IN) && fcb->meat == fcb->total_fraglen)) {
            status[i] = PPE_DF_CACHED;
            d->st[PPE_DF_CACHED]++;
            continue;
        }
        /* Frag_defrag_reasm */
        od_frag_t *head = fcb->fragments;
        const int icmp = head->proto == 1u;
        if (!icmp && (uint32_t)fcb->total_fraglen + head->l2 + head->ihl4 > d->reasm_buf) {
            status[i] = PPE_DF_SETUP_ERR;   /* MEM_8K_ALLOC fails: the chain stays cached */
            d->st[PPE_DF_SETUP_ERR]++;
            continue;
        }
        uint8_t *out = dgram_pkt ? dgram_pkt + (size_t)nd * d->reasm_buf : NULL;
        uint32_t tl = head->totlen;
        if (out) {
            memset(out, 0, d->reasm_buf);
            memcpy(out, head->frame, head->totlen < d->reasm_buf ? head->totlen : d->reasm_buf);
        }
        uint32_t k = 0;
        for (od_frag_t *q = head; q; q = q->next, ++k) {
            if (dgram_frags) dgram_frags[(size_t)nd * d->cache_max + k] = q->id;
            if (q == head) continue;
            if (!icmp && out) memcpy(out + tl, q->frame + q->totlen - q->flen, q->flen);
            tl += q->flen;
        }
        for (; dgram_frags && k < d->cache_max; ++k) dgram_frags[(size_t)nd * d->cache_max + k] = ~0ull;
        if (out) {
            uint8_t *iph = out + head->l2;
            if (!icmp) {
                const uint32_t iplen = (head->ihl4 + (uint32_t)fcb->total_fraglen) & 0xffffu;
                iph[2] = (uint8_t)(iplen >> 8);
                iph[3] = (uint8_t)iplen;
            }
            iph[6] = iph[7] = 0;
            if (!icmp) {
                const uint32_t cs = ip_csum(iph, head->ihl4);
                iph[10] = (uint8_t)(cs >> 8);
                iph[11] = (uint8_t)cs;
            }
        }
        if (dgram_len) dgram_len[nd] = tl;
        if (dgram_of) dgram_of[i] = nd;
        nd++;
        /* the chain moves to the reassembled mbuf (:268-276); the FCB is marked complete and deleted */
        free_frags(fcb->fragments);
        fcb->fragments = fcb->tail = NULL;
        fcb->status |= OD_COMPLETE | OD_DELETE;
        status[i] = PPE_DF_REASM;
        d->st[PPE_DF_REASM]++;
        d->datagrams++;
    }
    return nd;
}

uint32_t oracle_defrag_age(oracle_defrag_t *d, uint64_t now, uint64_t timeout, uint64_t *dropped, uint32_t max,
                           uint32_t *n_freed) {
    uint32_t nd = 0, nf = 0;
    for (uint32_t b = 0; b < OD_BUCKETS; ++b) {
        od_fcb_t **pp = &d->bucket[b];
        while (*pp) {
            od_fcb_t *f = *pp;
            if ((now > f->cycle && now - f->cycle > timeout) || (f->status & OD_DELETE)) {
                *pp = f->hnext;
                for (od_frag_t *q = f->fragments; q; q = q->next) {
                    if (dropped && nd < max) dropped[nd] = q->id;
                    nd++;
                }
                free_frags(f->fragments);
                free(f);
                nf++;
            } else {
                pp = &f->hnext;
            }
        }
    }
    d->running -= nf;
    d->del_fcb += nf;
    d->timeout_drop += nd;
    if (n_freed) *n_freed = nf;
    return nd;
}

/* out: running, new_fcb, del_fcb, st[PPE_DF__COUNT], teardrop, timeout_drop, datagrams */
void oracle_defrag_stats(const oracle_defrag_t *d, uint64_t *out) {
    out[0] = d->running;
    out[1] = d->new_fcb;
    out[2] = d->del_fcb;
    for (int k = 0; k < PPE_DF__COUNT; ++k) out[3 + k] = d->st[k];
    out[3 + PPE_DF__COUNT] = d->teardrop;
    out[4 + PPE_DF__COUNT] = d->timeout_drop;
    out[5 + PPE_DF__COUNT] = d->datagrams;
}
