/*
 * ppe_kernels.hip — the MI355X (gfx950) decode + 5-tuple ACL classify kernel.
 *
 * One lane per packet, one 64-packet tile per wavefront, persistent grid (each workgroup walks tiles
 * blockIdx*4+wave, +4*gridDim, ...).  Per packet:
 *   1. load the first 64 B of the header window (4 × 16-B loads) + the wire length;
 *   2. decode Ethernet → [VLAN] → IPv4 → UDP|TCP exactly as the reference dataplane (big-endian field values,
 *      the reference's check order and uint16/uint8 arithmetic — citations inline);
 *   3. flow_hashfn (TluHash ×3, dataplane/src/flow/tluhash.h:7-35);
 *   4. on the flow-miss path: syn_check, then the ACL decision-tree walk (image staged in LDS when it fits);
 *   5. SoA verdict / hash / hit stores, wave-ballot compaction of FW/DROP indices per tile, and per-reason
 *      counters reduced by ballot+popcount into one LDS word per reason, then one plain add per workgroup into
 *      that workgroup's own counter slot (no global atomics).
 * No MFMA: integer bitfield / compare work bound by HBM bandwidth.
 */
#include <hip/hip_runtime.h>

#include "ppe_hip.h"
#include "ppe_image.h"
#include "ppe_internal.h"

namespace {

__device__ __forceinline__ uint32_t be16_lo(uint32_t w) { return ((w & 0xffu) << 8) | ((w >> 8) & 0xffu); }
__device__ __forceinline__ uint32_t be16_hi(uint32_t w) { return ((w >> 8) & 0xff00u) | (w >> 24); }
__device__ __forceinline__ uint32_t bswap16(uint32_t x) { return ((x & 0xffu) << 8) | ((x >> 8) & 0xffu); }

// dataplane/src/flow/tluhash.h:7-23 (one Jenkins lookup2 mix with c = 0)
__device__ __forceinline__ uint32_t tlu_hash(uint32_t u1, uint32_t u2) {
    uint32_t a = u2 + 0x9e3779b9u, b = u1 + 0x9e3779b9u, c = 0;
    a -= b; a -= c; a ^= (c >> 13);
    b -= c; b -= a; b ^= (a << 8);
    c -= a; c -= b; c ^= (b >> 13);
    a -= b; a -= c; a ^= (c >> 12);
    b -= c; b -= a; b ^= (a << 16);
    c -= a; c -= b; c ^= (b >> 5);
    a -= b; a -= c; a ^= (c >> 3);
    b -= c; b -= a; b ^= (a << 10);
    c -= a; c -= b; c ^= (b >> 15);
    return c;
}

// dataplane/src/flow/tluhash.h:26-35
__device__ __forceinline__ uint32_t flow_hashfn(uint32_t proto, uint32_t sip, uint32_t dip, uint32_t sport,
                                                uint32_t dport) {
    return tlu_hash(sip, sport) ^ tlu_hash(dip, dport) ^ tlu_hash(proto, 0);
}

struct Pkt {
    uint32_t st, act, flags, cb;
    uint32_t sip, dip, sport, dport, proto, paylen;
    uint32_t acl;  // 1: flow miss path reached the ACL
};

#define CB(x) (1u << (x))

// Decode of one packet.  w[0..15] = first 64 bytes (little-endian dwords), row = the packet's window in global
// memory (for fields past byte 63), stride = window size.
__device__ __forceinline__ void decode(const uint32_t (&w)[16], uint32_t len32, const uint8_t *row,
                                       uint32_t stride, uint32_t unsup_act, uint32_t syn_check, Pkt &k) {
    const uint32_t len = len32 & 0xffffu;  // Decode passes (uint16_t)pkt_totallen, decode.c:22
    k.cb = CB(PPE_C_PKTS);
    k.flags = 0;
    k.acl = 0;
    k.sip = k.dip = k.sport = k.dport = k.proto = k.paylen = 0;
    k.act = PPE_ACT_DROP;

    // ---- Ethernet: dataplane/src/decode/decode-ethernet.c:23-115 ----
    if (len < 14) {  // :29-34
        k.st = PPE_ST_L2_HEADER_ERR; k.cb |= CB(PPE_C_L2_HEADERLEN_ERR); return;
    }
    const bool dst_zero = (w[0] == 0u) && ((w[1] & 0xffffu) == 0u);  // :38-44
    const bool src_zero = ((w[1] >> 16) == 0u) && (w[2] == 0u);      // :45-51
    if (dst_zero || src_zero) {
        k.st = PPE_ST_L2_HEADER_ERR; k.cb |= CB(PPE_C_L2_HEADERLEN_ERR); return;
    }
    const uint32_t etype = be16_lo(w[3]);
    uint32_t v, l3len;
    if (etype == 0x0800u) {  // :75-79
        k.cb |= CB(PPE_C_L2_RX_OK);
        v = 0;
        l3len = len - 14u;
    } else if (etype == 0x8100u || etype == 0x9100u) {  // :96-101 → decode-vlan.c:23-89
        k.cb |= CB(PPE_C_L2_RX_OK);
        const uint32_t vlen = len - 14u;
        if (vlen < 4u) {  // decode-vlan.c:28-33
            k.st = PPE_ST_VLAN_HEADER_ERR; k.cb |= CB(PPE_C_VLAN_HEADERLEN_ERR); return;
        }
        k.flags |= PPE_F_VLAN;  // vlan_idx = 1, decode-vlan.c:46
        const uint32_t itype = be16_lo(w[4]);
        if (itype == 0x0800u) {  // :49-53
            k.cb |= CB(PPE_C_VLAN_RX_OK);
            v = 1;
            l3len = vlen - 4u;
        } else if (itype == 0x8100u || itype == 0x9100u) {  // :70-75 recurse: len check, then vlan_idx >= 1
            k.cb |= CB(PPE_C_VLAN_RX_OK);
            if (vlen - 4u < 4u) {
                k.st = PPE_ST_VLAN_HEADER_ERR; k.cb |= CB(PPE_C_VLAN_HEADERLEN_ERR);
            } else {
                k.st = PPE_ST_VLAN_LAYER_EXCEED; k.cb |= CB(PPE_C_VLAN_LAYER_EXCEED);
            }
            return;
        } else {  // :76-84 unsupported → Decode_unsupport_proto_handle (decode.c:31-45)
            k.st = PPE_ST_VLAN_UNSUPPORT; k.cb |= CB(PPE_C_VLAN_UNSUPPORT); k.act = unsup_act; return;
        }
    } else {  // :102-111
        k.st = PPE_ST_L2_UNSUPPORT; k.cb |= CB(PPE_C_L2_UNSUPPORT); k.act = unsup_act; return;
    }

    // ---- IPv4: dataplane/src/decode/decode-ipv4.c:27-79, 86-247.  L3 starts at byte 14 + 4v = 4*(3+v) + 2.
    // D[i] = dword (3 + v + i) of the window, i.e. the dwords covering the L3/L4 headers.  Blended with a mask
    // rather than `v ? w[4+i] : w[3+i]`, which the compiler turns into a dynamic index (scratch).
    const uint32_t vm = 0u - v;
    uint32_t D[10];
#pragma unroll
    for (int i = 0; i < 10; ++i) D[i] = (w[3 + i] & ~vm) | (w[4 + i] & vm);
    if (l3len < 20u) {  // :30-34
        k.st = PPE_ST_IPV4_HEADER_ERR; k.cb |= CB(PPE_C_IPV4_HEADERLEN_ERR); return;
    }
    const uint32_t verhl = (D[0] >> 16) & 0xffu;
    if ((verhl >> 4) != 4u) {  // :36-40
        k.st = PPE_ST_IPV4_VERSION_ERR; k.cb |= CB(PPE_C_IPV4_VERSION_ERR); return;
    }
    const uint32_t hlen = (verhl & 0xfu) << 2;
    if (hlen < 20u) {  // :44-48
        k.st = PPE_ST_IPV4_HEADER_ERR; k.cb |= CB(PPE_C_IPV4_HEADERLEN_ERR); return;
    }
    const uint32_t iplen = be16_lo(D[1]);
    if (iplen < hlen || l3len < iplen) {  // :50-60
        k.st = PPE_ST_IPV4_LEN_ERR; k.cb |= CB(PPE_C_IPV4_PKTLEN_ERR); return;
    }
    k.sip = __builtin_bswap32((D[3] >> 16) | (D[4] << 16));  // :62 src_addr at L3+12
    k.dip = __builtin_bswap32((D[4] >> 16) | (D[5] << 16));  // :63 dst_addr at L3+16
    k.proto = D[2] >> 24;                                     // :97 ip_proto at L3+9
    const uint32_t ipoff = be16_lo(D[2]);                     // ip_off at L3+6
    if ((ipoff & 0x3fffu) != 0u && k.proto != 89u) {          // IPV4_IS_FRAGMENT && !OSPF, :102
        k.flags |= PPE_F_FRAG;
        if (((l3len - hlen) & 0xffffu) == 0u) {  // frag_len == 0, :109-114
            k.st = PPE_ST_FRAG_LEN_ERR; k.cb |= CB(PPE_C_FRAG_FRAGLEN_ERR); return;
        }
        k.st = PPE_ST_FRAG; k.cb |= CB(PPE_C_FRAG_PUNT); k.act = PPE_ACT_PUNT; return;  // Defrag → host
    }
    const bool is_tcp = k.proto == 6u, is_udp = k.proto == 17u;
    if (!is_tcp && !is_udp) {  // :233-243
        k.st = PPE_ST_IPV4_UNSUPPORT; k.cb |= CB(PPE_C_IPV4_UNSUPPORT); k.act = unsup_act; return;
    }
    k.cb |= CB(PPE_C_IPV4_RX_OK);
    const uint32_t l4len = (iplen - hlen) & 0xffffu;
    const uint32_t l4off = 14u + 4u * v + hlen;
    const bool fast = hlen == 20u;  // L4 at byte 34+4v: fields from registers
    uint32_t sport, dport, x;
    if (is_udp) {
        // ---- UDP: dataplane/src/decode/decode-udp.c:16-49 ----
        if (l4len < 8u) {  // :18-22
            k.st = PPE_ST_UDP_HEADER_ERR; k.cb |= CB(PPE_C_UDP_HEADERLEN_ERR); return;
        }
        if (fast) {
            sport = be16_hi(D[5]);
            dport = be16_lo(D[6]);
            x = be16_hi(D[6]);
        } else {
            if (l4off + 6u > stride) {
                k.st = PPE_ST_WINDOW_PUNT; k.cb |= CB(PPE_C_WINDOW_PUNT); k.act = PPE_ACT_PUNT; return;
            }
            const uint16_t *q = (const uint16_t *)(row + l4off);
            sport = bswap16(q[0]);
            dport = bswap16(q[1]);
            x = bswap16(q[2]);
        }
        if (l4len != x) {  // l4len < uh_len, l4len != uh_len: :26-36
            k.st = PPE_ST_UDP_LEN_ERR; k.cb |= CB(PPE_C_UDP_PKTLEN_ERR); return;
        }
        k.cb |= CB(PPE_C_UDP_RX_OK);
        k.paylen = l4len - 8u;
    } else {
        // ---- TCP: dataplane/src/decode/decode-tcp.c:135-190 ----
        if (l4len < 20u) {  // :140-144
            k.st = PPE_ST_TCP_HEADER_ERR; k.cb |= CB(PPE_C_TCP_HEADERLEN_ERR); return;
        }
        if (fast) {
            sport = be16_hi(D[5]);
            dport = be16_lo(D[6]);
            x = D[8] >> 16;  // byte 12 = th_offx2, byte 13 = th_flags
        } else {
            if (l4off + 14u > stride) {
                k.st = PPE_ST_WINDOW_PUNT; k.cb |= CB(PPE_C_WINDOW_PUNT); k.act = PPE_ACT_PUNT; return;
            }
            const uint16_t *q = (const uint16_t *)(row + l4off);
            sport = bswap16(q[0]);
            dport = bswap16(q[1]);
            x = q[6];
        }
        const uint32_t thl = ((x & 0xffu) >> 4) << 2;  // uint8_t hlen, :148
        if (l4len < thl || ((thl - 20u) & 0xffu) > 40u) {  // :149-160
            k.st = PPE_ST_TCP_LEN_ERR; k.cb |= CB(PPE_C_TCP_PKTLEN_ERR); return;
        }
        k.flags |= PPE_F_TCP;
        if ((x >> 8) & 0x02u) k.flags |= PPE_F_SYN;  // TCP_IS_SYN, decode-tcp.h:313
        k.cb |= CB(PPE_C_TCP_RX_OK);
        k.paylen = l4len - thl;
    }
    k.sport = sport;
    k.dport = dport;
    k.flags |= PPE_F_L4;

    // ---- FlowHandlePacket miss path: dataplane/src/flow/flow.c:204-243 ----
    if (is_tcp && syn_check && !(k.flags & PPE_F_SYN)) {
        k.st = PPE_ST_FLOW_TCP_NO_SYN_FIRST;
        k.cb |= CB(PPE_C_FLOW_TCP_NO_SYN_FIRST) | CB(PPE_C_FLOW_PROC_FAIL);
        return;
    }
    k.acl = 1;  // status decided by the ACL
}

// First-match decision-tree lookup over the classifier image (ppe_image.h).  `im` points either into LDS or to
// global memory; after inlining the address space is inferred from the caller.
// The 5-tuple arrives as scalars (not struct fields): a select between fields of an in-memory struct is folded
// into a dynamically indexed load, which sends the whole struct to scratch.
__device__ __forceinline__ void acl_lookup(const uint32_t *__restrict__ im, uint32_t off_leaf, uint32_t off_rules,
                                           uint32_t off_resid, uint32_t default_action, const uint32_t sip,
                                           const uint32_t dip, const uint32_t sport, const uint32_t dport,
                                           const uint32_t proto, uint32_t dmac_lo, uint32_t dmac_hi,
                                           uint32_t smac_lo, uint32_t smac_hi, uint64_t ts, int32_t &hit,
                                           uint32_t &action) {
    const uint2 *nodes = (const uint2 *)(im + PPE_IMG_HDR_WORDS);
    uint2 nd = nodes[0];
#pragma unroll 1
    for (int it = 0; it < PPE_MAX_DEPTH && (nd.y & 7u) != PPE_NODE_LEAF; ++it) {
        const uint32_t d = nd.y & 7u;
        uint32_t key = proto;
        key = d == PPE_DIM_SIP ? sip : key;
        key = d == PPE_DIM_DIP ? dip : key;
        key = d == PPE_DIM_SPORT ? sport : key;
        key = d == PPE_DIM_DPORT ? dport : key;
        nd = nodes[(nd.y >> 3) + (key > nd.x ? 1u : 0u)];
    }
    hit = -1;
    action = default_action;
    if ((nd.y & 7u) != PPE_NODE_LEAF) return;  // unreachable for a builder-made image
    const uint32_t cnt = nd.y >> 3;
    const uint32_t *lf = im + off_leaf + nd.x;
#pragma unroll 1
    for (uint32_t j = 0; j < cnt; ++j) {
        const uint32_t e = lf[j];
        const uint32_t slot = e & ~PPE_LEAF_CERTAIN;
        const uint4 *rp = (const uint4 *)(im + off_rules + 8u * slot);
        const uint4 a = rp[0], b = rp[1];
        bool m = (e & PPE_LEAF_CERTAIN) != 0u;
        if (!m) {
            m = sip >= a.x && sip <= a.y && dip >= a.z && dip <= a.w &&
                sport >= (b.x & 0xffffu) && sport <= (b.x >> 16) &&
                dport >= (b.y & 0xffffu) && dport <= (b.y >> 16) &&
                proto >= (b.z & 0xffu) && proto <= ((b.z >> 8) & 0xffu);
            const uint32_t rs = b.w >> 29;
            if (m && rs) {
                const uint4 *xp = (const uint4 *)(im + off_resid + 8u * slot);
                const uint4 c = xp[0], t = xp[1];
                if (rs & PPE_RESID_DMAC) m = m && c.x == dmac_lo && c.y == dmac_hi;
                if (rs & PPE_RESID_SMAC) m = m && c.z == smac_lo && c.w == smac_hi;
                if (rs & PPE_RESID_TIME) {
                    const uint64_t t0 = (uint64_t)t.x | ((uint64_t)t.y << 32);
                    const uint64_t t1 = (uint64_t)t.z | ((uint64_t)t.w << 32);
                    m = m && ts >= t0 && ts <= t1;
                }
            }
        }
        if (m) {
            hit = (int32_t)(b.w & 0x1fffffffu);
            action = b.z >> 16;
            return;
        }
    }
}

template <bool LDS_IMG>
__global__ __launch_bounds__(PPE_BLOCK) void ppe_classify_kernel(ppe_kargs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    uint32_t *lcnt = smem;       // [32] per-reason counters of this workgroup
    uint32_t *limg = smem + 32;  // staged classifier image
    const uint32_t tid = threadIdx.x;
    if (tid < 32) lcnt[tid] = 0;
    if (LDS_IMG) {
        const uint4 *src = (const uint4 *)a.img;
        uint4 *dst = (uint4 *)limg;
        const uint32_t n4 = (a.img_words + 3u) >> 2;
        for (uint32_t i = tid; i < n4; i += PPE_BLOCK) dst[i] = src[i];
    }
    __syncthreads();
    const uint32_t *im = LDS_IMG ? (const uint32_t *)limg : a.img;
    const uint32_t off_leaf = a.img[PPE_IMG_W_OFFLEAF];
    const uint32_t off_rules = a.img[PPE_IMG_W_OFFRULES];
    const uint32_t off_resid = a.img[PPE_IMG_W_OFFRESID];

    const uint32_t lane = tid & 63u;
    const uint32_t ntiles = (a.n + 63u) >> 6;
    const uint32_t stride_waves = gridDim.x * (PPE_BLOCK / 64);
    const uint32_t unsup_act = a.unsup_fw ? (uint32_t)PPE_ACT_FW : (uint32_t)PPE_ACT_DROP;
    uint32_t my_cnt = 0;  // lane b (< PPE_C__COUNT) accumulates counter b of this wave

    for (uint32_t tile = blockIdx.x * (PPE_BLOCK / 64) + (tid >> 6); tile < ntiles; tile += stride_waves) {
        const uint32_t p = (tile << 6) + lane;
        const bool valid = p < a.n;
        uint32_t w[16];
        uint32_t len = 0;
        const uint8_t *row = a.hdr + (size_t)p * a.stride;
        if (valid) {
            const uint4 *r4 = (const uint4 *)row;
            const uint4 q0 = r4[0], q1 = r4[1], q2 = r4[2], q3 = r4[3];
            w[0] = q0.x; w[1] = q0.y; w[2] = q0.z; w[3] = q0.w;
            w[4] = q1.x; w[5] = q1.y; w[6] = q1.z; w[7] = q1.w;
            w[8] = q2.x; w[9] = q2.y; w[10] = q2.z; w[11] = q2.w;
            w[12] = q3.x; w[13] = q3.y; w[14] = q3.z; w[15] = q3.w;
            len = a.len[p];
        } else {
#pragma unroll
            for (int i = 0; i < 16; ++i) w[i] = 0;
        }

        Pkt k;
        decode(w, len, row, a.stride, unsup_act, a.syn_check, k);
        if (!valid) k.acl = 0;

        uint32_t fh = 0;
        int32_t hit = -1;
        if (k.flags & PPE_F_L4) fh = flow_hashfn(k.proto, k.sip, k.dip, k.sport, k.dport);
        if (k.acl) {
            const uint64_t ts = a.ts ? a.ts[p] : a.now;
            uint32_t act;
            // dmac = bytes 0-5, smac = bytes 6-11 (EthernetHdr, decode-ethernet.h:23-27)
            acl_lookup(im, off_leaf, off_rules, off_resid, a.default_action, k.sip, k.dip, k.sport, k.dport,
                       k.proto, w[0], w[1] & 0xffffu,
                       (w[1] >> 16) | (w[2] << 16), w[2] >> 16, ts, hit, act);
            k.flags |= PPE_F_ACL;
            if (act == ACL_RULE_ACTION_DROP) {  // flow.c:232-237
                k.st = PPE_ST_ACL_DROP;
                k.act = PPE_ACT_DROP;
                k.cb |= CB(PPE_C_ACL_DROP) | CB(PPE_C_FLOW_PROC_FAIL);
            } else {  // flow.c:238-243, FlowHandlePacket :309
                k.st = PPE_ST_ACL_FW;
                k.act = PPE_ACT_FW;
                k.cb |= CB(PPE_C_ACL_FW) | CB(PPE_C_FLOW_PROC_OK);
            }
        }
        k.cb |= k.act == PPE_ACT_FW ? CB(PPE_C_OUT_FW) : (k.act == PPE_ACT_DROP ? CB(PPE_C_OUT_DROP) : CB(PPE_C_OUT_PUNT));

        if (valid) {
            if (a.verdict) a.verdict[p] = k.st | (k.act << 8) | (k.flags << 16);
            if (a.fhash) a.fhash[p] = fh;
            if (a.hit) a.hit[p] = hit;
            if (a.tuple) {
                uint4 t;
                t.x = k.sip;
                t.y = k.dip;
                t.z = k.sport | (k.dport << 16);
                t.w = k.proto | (((k.flags & PPE_F_VLAN) ? 1u : 0u) << 8) | (k.paylen << 16);
                ((uint4 *)a.tuple)[p] = t;
            }
        }

        // ---- wave-ballot compaction of FW / DROP indices into this tile's 64-slot segment ----
        const bool is_fw = valid && k.act == PPE_ACT_FW;
        const bool is_drop = valid && k.act == PPE_ACT_DROP;
        const uint64_t bfw = __ballot(is_fw);
        const uint64_t bdr = __ballot(is_drop);
        const uint64_t bpu = __ballot(valid && k.act == PPE_ACT_PUNT);
        if (a.fw_idx && is_fw) {
            const uint32_t pos =
                __builtin_amdgcn_mbcnt_hi((uint32_t)(bfw >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bfw, 0u));
            a.fw_idx[(tile << 6) + pos] = p + a.idx_base;
        }
        if (a.drop_idx && is_drop) {
            const uint32_t pos =
                __builtin_amdgcn_mbcnt_hi((uint32_t)(bdr >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bdr, 0u));
            a.drop_idx[(tile << 6) + pos] = p + a.idx_base;
        }
        if (a.tile_cnt && lane == 0)
            a.tile_cnt[tile] = (uint32_t)__popcll(bfw) | ((uint32_t)__popcll(bdr) << 8) |
                               ((uint32_t)__popcll(bpu) << 16);

        // ---- per-reason counters: one ballot per reason, lane b keeps reason b ----
        const uint32_t cb = valid ? k.cb : 0u;
#pragma unroll
        for (int b = 0; b < PPE_C__COUNT; ++b) {
            const uint32_t c = (uint32_t)__popcll(__ballot((cb >> b) & 1u));
            my_cnt += lane == (uint32_t)b ? c : 0u;
        }
    }

    if (lane < PPE_C__COUNT && my_cnt) atomicAdd(&lcnt[lane], my_cnt);
    __syncthreads();
    if (tid < PPE_C__COUNT) a.cslots[(size_t)blockIdx.x * PPE_CSLOT_WORDS + tid] += lcnt[tid];
}

// ACL-only lookup over pre-decoded tuples (the DP_Acl_Lookup(mbuf) entry, dataplane/src/flow/flow.c:232):
// tuple = {sip, dip, sport | dport << 16, proto}, macs = {dmac lo, dmac hi, smac lo, smac hi} (optional).
template <bool LDS_IMG>
__global__ __launch_bounds__(PPE_BLOCK) void ppe_acl_tuple_kernel(ppe_tuple_kargs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    const uint32_t tid = threadIdx.x;
    if (LDS_IMG) {
        const uint4 *src = (const uint4 *)a.img;
        uint4 *dst = (uint4 *)smem;
        const uint32_t n4 = (a.img_words + 3u) >> 2;
        for (uint32_t i = tid; i < n4; i += PPE_BLOCK) dst[i] = src[i];
        __syncthreads();
    }
    const uint32_t *im = LDS_IMG ? (const uint32_t *)smem : a.img;
    const uint32_t off_leaf = a.img[PPE_IMG_W_OFFLEAF];
    const uint32_t off_rules = a.img[PPE_IMG_W_OFFRULES];
    const uint32_t off_resid = a.img[PPE_IMG_W_OFFRESID];
    for (uint32_t i = blockIdx.x * PPE_BLOCK + tid; i < a.n; i += gridDim.x * PPE_BLOCK) {
        const uint4 t = ((const uint4 *)a.tuple)[i];
        uint4 m = make_uint4(0, 0, 0, 0);
        if (a.macs) m = ((const uint4 *)a.macs)[i];
        const uint64_t ts = a.ts ? a.ts[i] : a.now;
        int32_t hit;
        uint32_t act;
        acl_lookup(im, off_leaf, off_rules, off_resid, a.default_action, t.x, t.y, t.z & 0xffffu, t.z >> 16,
                   t.w & 0xffu, m.x, m.y, m.z, m.w, ts, hit, act);
        if (a.hit) a.hit[i] = hit;
        if (a.action) a.action[i] = act;
    }
}

}  // namespace

extern "C" int ppe_launch_classify(const ppe_kargs *a, uint32_t grid, int lds_img, void *stream) {
    const size_t base = 32 * sizeof(uint32_t);
    if (lds_img) {
        const size_t shmem = base + (((size_t)a->img_words * 4u + 15u) & ~(size_t)15u);
        hipLaunchKernelGGL(ppe_classify_kernel<true>, dim3(grid), dim3(PPE_BLOCK), shmem, (hipStream_t)stream, *a);
    } else {
        hipLaunchKernelGGL(ppe_classify_kernel<false>, dim3(grid), dim3(PPE_BLOCK), base, (hipStream_t)stream, *a);
    }
    return (int)hipGetLastError();
}

extern "C" int ppe_launch_acl_tuples(const ppe_tuple_kargs *a, uint32_t grid, int lds_img, void *stream) {
    if (lds_img) {
        const size_t shmem = ((size_t)a->img_words * 4u + 15u) & ~(size_t)15u;
        hipLaunchKernelGGL(ppe_acl_tuple_kernel<true>, dim3(grid), dim3(PPE_BLOCK), shmem, (hipStream_t)stream, *a);
    } else {
        hipLaunchKernelGGL(ppe_acl_tuple_kernel<false>, dim3(grid), dim3(PPE_BLOCK), 0, (hipStream_t)stream, *a);
    }
    return (int)hipGetLastError();
}
