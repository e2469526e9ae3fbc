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
#include <hip/hip_ext.h>

#include "ppe_hip.h"
#include "ppe_image.h"
#include "ppe_internal.h"

// Diagnostic ablation builds only (make ablate): bit 0 skip the ACL walk, bit 1 skip counters, bit 2 skip the
// compaction, bit 3 skip the flow hash.  The product build has PPE_ABLATE == 0.
#ifndef PPE_ABLATE
#define PPE_ABLATE 0
#endif
// Diagnostic builds only (make variant NAME=trace VFLAGS=-DPPE_TRACE=1): lane 0 of every wave writes shader-clock
// timestamps (s_memrealtime, 100 MHz) of its phases to kargs.trace, 32 words per wave (tools/trace_analyze.py):
//   [0] kernel entry  [1] image staged  [2 + 5i + k] tile iteration i < 4: k 0 loop top, 1 window in registers,
//   2 decoded + hashed, 3 ACL done, 4 outputs + counters issued   [22] after the loop  [31] tiles processed
#ifndef PPE_TRACE
#define PPE_TRACE 0
#endif
#define TRACE_AT(idx)                                                                      \
    do {                                                                                   \
        if (PPE_TRACE) {                                                                   \
            const uint64_t t_ = __builtin_amdgcn_s_memrealtime();                            \
            if (lane == 0 && a.trace) a.trace[(size_t)twave * 32u + (idx)] = t_;          \
        }                                                                                  \
    } while (0)

namespace {

typedef __attribute__((address_space(1))) const void *gptr_t;
typedef __attribute__((address_space(3))) void *lptr_t;

__device__ __forceinline__ uint32_t be16_lo(uint32_t w) { return ((w & 0xffu) << 8) | ((w >> 8) & 0xffu); }
__device__ __forceinline__ uint32_t be16_hi(uint32_t w) { return ((w >> 8) & 0xff00u) | (w >> 24); }
__device__ __forceinline__ uint32_t bswap16(uint32_t x) { return ((x & 0xffu) << 8) | ((x >> 8) & 0xffu); }

// dataplane/src/flow/tluhash.h:7-23 (one Jenkins lookup2 mix with c = 0)
__host__ __device__ constexpr uint32_t tlu_hash(uint32_t u1, uint32_t u2) {
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

// dataplane/src/flow/tluhash.h:26-35.  Only TCP/UDP packets reach the flow engine, so the protocol term
// TluHash(proto, 0) is one of two compile-time constants.
constexpr uint32_t kProtoHashTcp = tlu_hash(6u, 0u);
constexpr uint32_t kProtoHashUdp = tlu_hash(17u, 0u);
__device__ __forceinline__ uint32_t flow_hashfn_l4(bool tcp, uint32_t sip, uint32_t dip, uint32_t sport,
                                                   uint32_t dport) {
    return tlu_hash(sip, sport) ^ tlu_hash(dip, dport) ^ (tcp ? kProtoHashTcp : kProtoHashUdp);
}

#define CB(x) (1u << (x))
#define ST_ACL 0xffu  // decode passed: the ACL decides

// counter index of each terminal status (enum ppe_status → enum ppe_counter), 5 bits per entry
__device__ __forceinline__ uint32_t reason_counter(uint32_t st) {
    constexpr uint64_t K0 =  // st 0..11
        ((uint64_t)PPE_C_ACL_FW << 0) | ((uint64_t)PPE_C_ACL_DROP << 5) | ((uint64_t)PPE_C_L2_HEADERLEN_ERR << 10) |
        ((uint64_t)PPE_C_L2_UNSUPPORT << 15) | ((uint64_t)PPE_C_VLAN_HEADERLEN_ERR << 20) |
        ((uint64_t)PPE_C_VLAN_LAYER_EXCEED << 25) | ((uint64_t)PPE_C_VLAN_UNSUPPORT << 30) |
        ((uint64_t)PPE_C_IPV4_HEADERLEN_ERR << 35) | ((uint64_t)PPE_C_IPV4_VERSION_ERR << 40) |
        ((uint64_t)PPE_C_IPV4_PKTLEN_ERR << 45) | ((uint64_t)PPE_C_FRAG_FRAGLEN_ERR << 50) |
        ((uint64_t)PPE_C_FRAG_PUNT << 55);
    constexpr uint64_t K1 =  // st 12..18
        ((uint64_t)PPE_C_IPV4_UNSUPPORT << 0) | ((uint64_t)PPE_C_UDP_HEADERLEN_ERR << 5) |
        ((uint64_t)PPE_C_UDP_PKTLEN_ERR << 10) | ((uint64_t)PPE_C_TCP_HEADERLEN_ERR << 15) |
        ((uint64_t)PPE_C_TCP_PKTLEN_ERR << 20) | ((uint64_t)PPE_C_FLOW_TCP_NO_SYN_FIRST << 25) |
        ((uint64_t)PPE_C_WINDOW_PUNT << 30);
    const bool lo = st < 12u;
    return (uint32_t)(((lo ? K0 : K1) >> (5u * (lo ? st : st - 12u))) & 31u);
}

// Synchronous global loads for the rare paths (IPv4 options, time-window rules).  Inline asm with its own wait: the
// compiler then tracks no pending VMEM result across the tile loop, so it never puts a conservative vmcnt(0) -
// which would also wait for the next tile's in-flight LDS-DMA - at the top of the loop.
__device__ __forceinline__ void ld_l4_sync(const uint8_t *q, uint32_t &a, uint32_t &b, uint32_t &c, uint32_t &d) {
    asm volatile(
        "global_load_ushort %0, %4, off\n\t"
        "global_load_ushort %1, %4, off offset:2\n\t"
        "global_load_ushort %2, %4, off offset:4\n\t"
        "global_load_ushort %3, %4, off offset:12\n\t"
        "s_waitcnt vmcnt(0)"
        : "=&v"(a), "=&v"(b), "=&v"(c), "=&v"(d)
        : "v"(q)
        : "memory");
}
__device__ __forceinline__ void ld_mac_sync(const uint8_t *q, uint32_t &a, uint32_t &b, uint32_t &c) {
    typedef uint32_t v3u __attribute__((ext_vector_type(3)));
    v3u v;
    asm volatile("global_load_dwordx3 %0, %1, off\n\ts_waitcnt vmcnt(0)" : "=&v"(v) : "v"(q) : "memory");
    a = v.x;
    b = v.y;
    c = v.z;
}
__device__ __forceinline__ uint64_t ld_u64_sync(const uint64_t *q) {
    uint64_t v;
    asm volatile("global_load_dwordx2 %0, %1, off\n\ts_waitcnt vmcnt(0)" : "=&v"(v) : "v"(q) : "memory");
    return v;
}

// Where a residual MAC rule gets the packet's MACs: re-read from the header window (classify kernel: rare path, keeps
// the MACs out of registers during the tree walk) or given by value (tuple kernel).
struct MacFromWindow {
    const uint8_t *hdr;
    uint32_t p, stride;
    __device__ __forceinline__ void get(uint32_t &dlo, uint32_t &dhi, uint32_t &slo, uint32_t &shi) const {
        uint32_t w0, w1, w2;  // dmac = bytes 0-5, smac = bytes 6-11 (EthernetHdr, decode-ethernet.h:23-27)
        ld_mac_sync(hdr + (size_t)p * stride, w0, w1, w2);
        dlo = w0;
        dhi = w1 & 0xffffu;
        slo = (w1 >> 16) | (w2 << 16);
        shi = w2 >> 16;
    }
};
struct MacValues {
    uint32_t dlo, dhi, slo, shi;
    __device__ __forceinline__ void get(uint32_t &a, uint32_t &b, uint32_t &c, uint32_t &d) const {
        a = dlo;
        b = dhi;
        c = slo;
        d = shi;
    }
};

// Per-reason counters are a function of the final (status, VLAN / TCP / L4 flags) of a packet, so the kernel only
// counts packets per bin key = status | VLAN << 5 | TCP << 6 | L4 << 7 (one LDS add per packet) and expands each
// non-empty bin into counter increments once per workgroup.  The rules (same as the reference's pktstat updates):
//   every packet: PKTS and its terminal reason (decode-statistic.h:239-327; ACL_FW / ACL_DROP for the ACL path)
//   L2_RX_OK unless the Ethernet layer failed; VLAN_RX_OK for a parsed tag that was not of an unsupported type;
//   IPV4_RX_OK when the packet reached the TCP/UDP decoder; UDP_RX_OK / TCP_RX_OK when it reached the flow engine;
//   FLOW_PROC_OK / _FAIL by the flow engine's outcome; OUT_FW / OUT_DROP / OUT_PUNT by the action.
#define PPE_NBINS 256u
__device__ __forceinline__ uint32_t bin_counters(uint32_t key, uint64_t act_table) {
    const uint32_t st = key & 31u;
    const bool vl = (key >> 5) & 1u, tcp = (key >> 6) & 1u, l4 = (key >> 7) & 1u;
    uint32_t cb = CB(PPE_C_PKTS) | CB(reason_counter(st));
    if (st != PPE_ST_L2_HEADER_ERR && st != PPE_ST_L2_UNSUPPORT) cb |= CB(PPE_C_L2_RX_OK);
    if (vl && st != PPE_ST_VLAN_UNSUPPORT) cb |= CB(PPE_C_VLAN_RX_OK);
    const bool l4_in = st == PPE_ST_ACL_FW || st == PPE_ST_ACL_DROP || st == PPE_ST_UDP_HEADER_ERR ||
                       st == PPE_ST_UDP_LEN_ERR || st == PPE_ST_TCP_HEADER_ERR || st == PPE_ST_TCP_LEN_ERR ||
                       st == PPE_ST_FLOW_TCP_NO_SYN_FIRST || st == PPE_ST_WINDOW_PUNT;
    if (l4_in) cb |= CB(PPE_C_IPV4_RX_OK);
    if (l4 && !tcp) cb |= CB(PPE_C_UDP_RX_OK);
    if (tcp) cb |= CB(PPE_C_TCP_RX_OK);
    if (st == PPE_ST_FLOW_TCP_NO_SYN_FIRST || st == PPE_ST_ACL_DROP) cb |= CB(PPE_C_FLOW_PROC_FAIL);
    if (st == PPE_ST_ACL_FW) cb |= CB(PPE_C_FLOW_PROC_OK);
    const uint32_t act = (uint32_t)(act_table >> (2u * st)) & 3u;
    cb |= act == PPE_ACT_FW ? CB(PPE_C_OUT_FW) : (act == PPE_ACT_DROP ? CB(PPE_C_OUT_DROP) : CB(PPE_C_OUT_PUNT));
    return cb;
}

struct Dec {
    uint32_t st, flags;
    uint32_t sip, dip, sport, dport, proto, paylen;
};

// Decode of one packet, straight-line: every check of the reference is evaluated, then the terminal status is
// chosen by applying the checks in REVERSE order of the reference's control flow, so the first failing check
// (the one the reference returns on) wins.  w[0..15] = first 64 bytes (little-endian dwords); row = the packet's
// window in global memory (read only for L4 headers behind IPv4 options).
__device__ __forceinline__ Dec decode(const uint32_t (&w)[16], uint32_t len32, const uint8_t *hdr, uint32_t p, uint32_t stride,
                                      uint32_t syn_check) {
    Dec k;
    const uint32_t len = len32 & 0xffffu;  // Decode passes (uint16_t)pkt_totallen, decode.c:22
    // ---- Ethernet: dataplane/src/decode/decode-ethernet.c:23-115 ----
    const bool bad_len = len < 14u;                               // :29-34
    const bool dz = (w[0] | (w[1] & 0xffffu)) == 0u;              // :38-44 dst MAC all zero
    const bool sz = ((w[1] >> 16) | w[2]) == 0u;                  // :45-51 src MAC all zero
    const uint32_t etype = be16_lo(w[3]);
    const bool is_ip = etype == 0x0800u;                          // :75
    const bool is_vl = (etype | 0x1000u) == 0x9100u;              // 0x8100 or 0x9100, :96-97
    const bool l2_ok = !(bad_len || dz || sz) && (is_ip || is_vl);
    // ---- VLAN: dataplane/src/decode/decode-vlan.c:23-89 ----
    const uint32_t vlen = len - 14u;
    const uint32_t itype = be16_lo(w[4]);
    const bool v_ip = itype == 0x0800u, v_vl = (itype | 0x1000u) == 0x9100u;
    const uint32_t v = is_vl ? 1u : 0u;
    const uint32_t l3len = vlen - 4u * v;
    // ---- IPv4: dataplane/src/decode/decode-ipv4.c:27-247.  L3 starts at byte 14 + 4v = 4*(3+v) + 2.
    // D[i] = dword (3 + v + i); a mask blend, not `v ? w[4+i] : w[3+i]` (folded into a dynamic index → scratch)
    const uint32_t vm = 0u - v;
    uint32_t D[10];
#pragma unroll
    for (int i = 0; i < 10; ++i) D[i] = (w[3 + i] & ~vm) | (w[4 + i] & vm);
    const uint32_t verhl = (D[0] >> 16) & 0xffu;
    const uint32_t hlen = (verhl & 0xfu) << 2;
    const uint32_t iplen = be16_lo(D[1]);
    const uint32_t sip = __builtin_bswap32((D[3] >> 16) | (D[4] << 16));  // src_addr, L3+12
    const uint32_t dip = __builtin_bswap32((D[4] >> 16) | (D[5] << 16));  // dst_addr, L3+16
    const uint32_t proto = D[2] >> 24;                                     // ip_proto, L3+9
    const uint32_t ipoff = be16_lo(D[2]);                                  // ip_off, L3+6
    const bool l3_in = l2_ok && (is_ip || (vlen >= 4u && v_ip));
    const bool ip_ok = l3_in && l3len >= 20u && (verhl >> 4) == 4u && hlen >= 20u && iplen >= hlen && l3len >= iplen;
    const bool frag = (ipoff & 0x3fffu) != 0u && proto != 89u;             // IPV4_IS_FRAGMENT && !OSPF, :102
    const bool is_tcp = proto == 6u, is_udp = proto == 17u;
    const bool l4_in = ip_ok && !frag && (is_tcp || is_udp);
    const uint32_t l4len = (iplen - hlen) & 0xffffu;
    const uint32_t l4off = 14u + 4u * v + hlen;
    const bool fast = hlen == 20u;  // L4 at byte 34+4v: every field below byte 52, in registers
    const bool win_short = !fast && (l4off + (is_tcp ? 14u : 6u) > stride);
    uint32_t sport = be16_hi(D[5]), dport = be16_lo(D[6]);
    uint32_t x = is_tcp ? (D[8] >> 16) : be16_hi(D[6]);  // TCP: offx2 | flags << 8;  UDP: uh_len
    if (l4_in && !fast && !win_short) {  // IPv4 options: L4 header at a data-dependent offset
        uint32_t h0, h1, h2, h6;
        ld_l4_sync(hdr + (size_t)p * stride + l4off, h0, h1, h2, h6);
        sport = bswap16(h0);
        dport = bswap16(h1);
        x = is_tcp ? h6 : bswap16(h2);
    }
    // ---- UDP: dataplane/src/decode/decode-udp.c:16-49;  TCP: dataplane/src/decode/decode-tcp.c:135-190 ----
    const uint32_t thl = ((x & 0xffu) >> 4) << 2;  // uint8_t hlen, decode-tcp.c:148
    const bool syn = ((x >> 8) & 0x02u) != 0u;     // TCP_IS_SYN, decode-tcp.h:313
    uint32_t st_tcp = (syn_check && !syn) ? (uint32_t)PPE_ST_FLOW_TCP_NO_SYN_FIRST : ST_ACL;  // flow.c:204-214
    st_tcp = (l4len < thl || ((thl - 20u) & 0xffu) > 40u) ? (uint32_t)PPE_ST_TCP_LEN_ERR : st_tcp;  // :149-160
    st_tcp = win_short ? (uint32_t)PPE_ST_WINDOW_PUNT : st_tcp;
    st_tcp = l4len < 20u ? (uint32_t)PPE_ST_TCP_HEADER_ERR : st_tcp;  // :140-144
    uint32_t st_udp = l4len != x ? (uint32_t)PPE_ST_UDP_LEN_ERR : ST_ACL;  // :26-36
    st_udp = win_short ? (uint32_t)PPE_ST_WINDOW_PUNT : st_udp;
    st_udp = l4len < 8u ? (uint32_t)PPE_ST_UDP_HEADER_ERR : st_udp;  // :18-22
    uint32_t st = is_tcp ? st_tcp : (is_udp ? st_udp : (uint32_t)PPE_ST_IPV4_UNSUPPORT);  // decode-ipv4.c:233-243
    st = frag ? ((((l3len - hlen) & 0xffffu) == 0u) ? (uint32_t)PPE_ST_FRAG_LEN_ERR : (uint32_t)PPE_ST_FRAG) : st;
    st = (iplen < hlen || l3len < iplen) ? (uint32_t)PPE_ST_IPV4_LEN_ERR : st;  // decode-ipv4.c:50-60
    st = hlen < 20u ? (uint32_t)PPE_ST_IPV4_HEADER_ERR : st;                    // :44-48
    st = (verhl >> 4) != 4u ? (uint32_t)PPE_ST_IPV4_VERSION_ERR : st;           // :36-40
    st = l3len < 20u ? (uint32_t)PPE_ST_IPV4_HEADER_ERR : st;                   // :30-34
    // VLAN tag (decode-vlan.c): len check, then the inner type; a second tag recurses: len check, vlan_idx >= 1
    uint32_t st_v = v_ip ? st
                         : (v_vl ? ((vlen - 4u < 4u) ? (uint32_t)PPE_ST_VLAN_HEADER_ERR
                                                     : (uint32_t)PPE_ST_VLAN_LAYER_EXCEED)
                                 : (uint32_t)PPE_ST_VLAN_UNSUPPORT);
    st_v = vlen < 4u ? (uint32_t)PPE_ST_VLAN_HEADER_ERR : st_v;
    st = is_vl ? st_v : (is_ip ? st : (uint32_t)PPE_ST_L2_UNSUPPORT);
    st = (bad_len || dz || sz) ? (uint32_t)PPE_ST_L2_HEADER_ERR : st;

    const bool l4_ok = st == ST_ACL || st == PPE_ST_FLOW_TCP_NO_SYN_FIRST;  // reached FlowHandlePacket
    k.st = st;
    k.flags = (l2_ok && is_vl && vlen >= 4u ? PPE_F_VLAN : 0u) | (l4_ok ? PPE_F_L4 : 0u) |
              (l4_ok && is_tcp ? PPE_F_TCP : 0u) | (l4_ok && is_tcp && syn ? PPE_F_SYN : 0u) |
              (ip_ok && frag ? PPE_F_FRAG : 0u);
    k.sip = ip_ok ? sip : 0u;
    k.dip = ip_ok ? dip : 0u;
    k.proto = ip_ok ? proto : 0u;
    k.sport = l4_ok ? sport : 0u;
    k.dport = l4_ok ? dport : 0u;
    k.paylen = l4_ok ? (is_tcp ? l4len - thl : l4len - 8u) : 0u;
    return k;
}

// Image staging modes of the classify kernel:
//   IMG_GLOBAL  the whole classifier image is read from global memory (L1/L2/MALL-cached)
//   IMG_LDS     the whole image is staged in LDS
//   IMG_SPLIT   a prefix is staged: tree nodes [0, lds_nodes) (BFS order: the top of the tree) and, when it fits,
//               the leaf lists; deeper nodes, leaf lists that did not fit and the rule records come from global
#define IMG_GLOBAL 0
#define IMG_LDS 1
#define IMG_SPLIT 2

// key of dimension d held in registers (walks that read nodes from global memory); d == PPE_NODE_LEAF gives 0
__device__ __forceinline__ uint32_t node_key(uint32_t d, uint32_t sip, uint32_t dip, uint32_t sport, uint32_t dport,
                                             uint32_t proto) {
    uint32_t key = 0u;
    key = d == PPE_DIM_PROTO ? proto : key;
    key = d == PPE_DIM_SIP ? sip : key;
    key = d == PPE_DIM_DIP ? dip : key;
    key = d == PPE_DIM_SPORT ? sport : key;
    key = d == PPE_DIM_DPORT ? dport : key;
    return key;
}

#define NODE_IS_LEAF(nd) (PPE_NODE_DIM((nd).y) == PPE_NODE_LEAF)
#define NODE_CHILD(nd, key) (((nd).y >> PPE_NODE_CHILD_SHIFT) + ((key) > (nd).x ? 1u : 0u))

// Per-lane walk keys in LDS (IMG_LDS): each wave owns KEY_SLOTS x 64 words, slot d = dimension d of every lane
// ([slot][lane]: a read with per-lane slots is bank-conflict free), slot PPE_NODE_LEAF = 0.  A level then costs one
// LDS read for the key instead of a 5-way register select.
#define KEY_SLOTS 6u
#define KEY_WAVE_WORDS (KEY_SLOTS * 64u)
// Classifier geometry for one launch (host-computed from the image header, ppe_image.h).
struct AclGeo {
    uint32_t lds_iters;   // walk levels whose nodes are all staged in LDS (IMG_LDS: max_depth, IMG_GLOBAL: 0)
    uint32_t max_depth;   // deepest leaf
    uint32_t max_leaf;    // longest leaf candidate list
    uint32_t off_leaf, off_rules, off_resid;
    uint32_t leaf_lds;    // leaf lists in LDS (IMG_LDS always; IMG_SPLIT when they fit)
    uint32_t default_action;
};

// One level of the walk for every lane, keys from LDS: a leaf's dimension is the zero key slot, so a lane already at a
// leaf stays there (ppe_image.h): a wave-uniform trip count, no per-lane exit, no exec-mask bookkeeping per level.
__device__ __forceinline__ void walk_level_lds(const uint2 *nodes, const uint32_t *keys, uint2 &nd) {
    const uint32_t key = *(const uint32_t *)((const char *)keys + (nd.y & 0x700u));          // slot dim, this lane
    const uint32_t off = ((nd.y >> 8) & ~7u) + (key > nd.x ? 8u : 0u);                       // child byte offset
    nd = *(const uint2 *)((const char *)nodes + off);
}

// Scan a leaf's candidate list in priority order; the first rule that matches wins (lowest index).  max_leaf
// uniform iterations: a lane whose list is shorter, or that has matched, keeps reading a valid entry and ignores it.
// `lf`, `rules` and `resid` may each point into LDS or global memory (address space inferred after inlining).
template <class Mac>
__device__ __forceinline__ void leaf_scan(uint2 nd, uint32_t max_leaf, const uint32_t *__restrict__ lf,
                                          const uint32_t *__restrict__ rules, const uint32_t *__restrict__ resid,
                                          uint32_t sip, uint32_t dip, uint32_t sport, uint32_t dport, uint32_t proto,
                                          const Mac &mac, const uint64_t *tsp, uint32_t p, uint64_t now,
                                          int32_t &hit, uint32_t &action) {
    uint32_t first = nd.x, cnt = nd.y & 0xffu;
    if (max_leaf >= PPE_LEAF_CNT_ESC && cnt == PPE_LEAF_CNT_ESC) cnt = lf[first++];  // long list: escaped count
    bool done = false;
#pragma unroll 1
    for (uint32_t j = 0; j < max_leaf; ++j) {
        const bool live = !done && j < cnt;
        const uint32_t e = lf[live ? first + j : 0u];  // entry 0 exists whenever max_leaf > 0
        const uint32_t slot = e & ~PPE_LEAF_CERTAIN;
        const uint4 *rp = (const uint4 *)(rules + 8u * slot);
        const uint4 a = rp[0], b = rp[1];
        const bool box = sip >= a.x && sip <= a.y && dip >= a.z && dip <= a.w &&
                         sport >= (b.x & 0xffffu) && sport <= (b.x >> 16) &&
                         dport >= (b.y & 0xffffu) && dport <= (b.y >> 16) &&
                         proto >= (b.z & 0xffu) && proto <= ((b.z >> 8) & 0xffu);
        bool m = live && ((e & PPE_LEAF_CERTAIN) != 0u || box);
        const uint32_t rs = b.w >> 29;
        if (m && rs && (e & PPE_LEAF_CERTAIN) == 0u) {  // residual MAC / time fields: rare
            const uint4 *xp = (const uint4 *)(resid + 8u * slot);
            const uint4 c = xp[0], t = xp[1];
            if (rs & (PPE_RESID_DMAC | PPE_RESID_SMAC)) {
                uint32_t dmac_lo, dmac_hi, smac_lo, smac_hi;
                mac.get(dmac_lo, dmac_hi, smac_lo, smac_hi);
                if (rs & PPE_RESID_DMAC) m = m && c.x == dmac_lo && c.y == dmac_hi;
                if (rs & PPE_RESID_SMAC) m = m && c.z == smac_lo && c.w == smac_hi;
            }
            if (rs & PPE_RESID_TIME) {  // the packet timestamp is only fetched for time-window rules
                const uint64_t ts = tsp ? ld_u64_sync(tsp + p) : now;
                const uint64_t t0 = (uint64_t)t.x | ((uint64_t)t.y << 32);
                const uint64_t t1 = (uint64_t)t.z | ((uint64_t)t.w << 32);
                m = m && ts >= t0 && ts <= t1;
            }
        }
        hit = m ? (int32_t)(b.w & 0x1fffffffu) : hit;
        action = m ? b.z >> 16 : action;
        done = done || m;
    }
}

// First-match decision-tree lookup over the classifier image.  The 5-tuple arrives as scalars (not struct fields):
// a select between fields of an in-memory struct is folded into a dynamically indexed load, which sends the whole
// struct to scratch.  Levels [0, lds_iters) read the staged top of the tree from LDS, the rest from global memory.
template <int MODE, class Mac>
__device__ __forceinline__ void acl_lookup(const uint32_t *__restrict__ gimg, const uint32_t *__restrict__ limg,
                                           const uint32_t *keys, const AclGeo &g, const uint32_t sip,
                                           const uint32_t dip, const uint32_t sport, const uint32_t dport,
                                           const uint32_t proto, const Mac &mac, const uint64_t *tsp, uint32_t p,
                                           uint64_t now, int32_t &hit, uint32_t &action) {
    const uint2 *gn = (const uint2 *)(gimg + PPE_IMG_HDR_WORDS);
    const uint2 *ln = (const uint2 *)(limg + PPE_IMG_HDR_WORDS);
    uint32_t it = 0;
    uint2 nd;
    if (MODE == IMG_GLOBAL) {
        nd = gn[0];
    } else if (MODE == IMG_LDS) {
        nd = ln[0];
#pragma unroll 2
        for (; it < g.max_depth; ++it) walk_level_lds(ln, keys, nd);
    } else {  // IMG_SPLIT: the staged top of the tree, keys selected in registers
        nd = ln[0];
#pragma unroll 1
        for (; it < g.lds_iters; ++it) nd = ln[NODE_CHILD(nd, node_key(PPE_NODE_DIM(nd.y), sip, dip, sport, dport, proto))];
    }
    if (MODE != IMG_LDS) {  // below the staged top: per-lane exit (a finished lane must not keep reading L2/HBM)
#pragma unroll 1
        for (; it < g.max_depth && !NODE_IS_LEAF(nd); ++it)
            nd = gn[NODE_CHILD(nd, node_key(PPE_NODE_DIM(nd.y), sip, dip, sport, dport, proto))];
    }
    hit = -1;
    action = g.default_action;
    // every lane is at a leaf now (max_depth = the deepest leaf of the builder's tree)
    if (MODE == IMG_LDS)
        leaf_scan(nd, g.max_leaf, limg + g.off_leaf, limg + g.off_rules, limg + g.off_resid, sip, dip, sport, dport,
                  proto, mac, tsp, p, now, hit, action);
    else if (MODE == IMG_SPLIT && g.leaf_lds)
        leaf_scan(nd, g.max_leaf, limg + g.off_leaf, gimg + g.off_rules, gimg + g.off_resid, sip, dip, sport, dport,
                  proto, mac, tsp, p, now, hit, action);
    else
        leaf_scan(nd, g.max_leaf, gimg + g.off_leaf, gimg + g.off_rules, gimg + g.off_resid, sip, dip, sport, dport,
                  proto, mac, tsp, p, now, hit, action);
}

// Copy the classifier image into LDS with LDS-DMA (global_load_lds_dwordx4): every 1-KB piece of the image is in
// flight at once, no VGPR round trip.  Each wave-instruction writes 64 × 16 B at a wave-uniform LDS base, so the
// LDS region is padded to a multiple of 1 KB and the (clamped) tail lanes write into the padding.
template <int BLOCK>
__device__ __forceinline__ void stage_image(const uint32_t *img, uint32_t *lds, uint32_t words, uint32_t tid) {
    const uint32_t n4 = (words + 3u) >> 2;
    const uint32_t lane = tid & 63u;
    for (uint32_t base = (tid >> 6) * 64u; base < n4; base += BLOCK) {
        const uint32_t i = min(base + lane, n4 - 1u);
        __builtin_amdgcn_global_load_lds((gptr_t)(img + 4u * i), (lptr_t)(lds + 4u * base), 16, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// LDS-DMA packet pipeline (PIPE): each wave owns one 3.5-KB LDS slot.  While tile t is classified from registers,
// tile t+1 is already on its way from HBM into the slot via global_load_lds (no VGPRs held, no wait), so the next
// HBM fetch overlaps this tile's decode / tree walk.  Slot layout (bytes): [0, 3072) the first 48 B of each of the 64
// windows (48-B rows: ds_read_b128 per lane is bank-conflict free), [3072, 3328) bytes 48..51 of each window,
// [3328, 3584) the 64 wire lengths.  Bytes 52..63 are never needed on the fast path (hlen == 20); IPv4-options
// packets read their L4 header from the window in global memory, as without the pipeline.
#define PIPE_SLOT_BYTES 3584u
#define PIPE_W12_OFF 3072u
#define PIPE_LEN_OFF 3328u

// Issue the five DMA ops of tile `t` into the slot at LDS byte address `slot` (wave-uniform).  Lane l of op k (< 3)
// fetches 16-B chunk (64k+l) % 3 of packet (64k+l) / 3; op 3 fetches bytes 48..51, op 4 the length.  In asm, like
// pipe_read: compiler-visible LDS-DMA makes the compiler (a) hoist the per-lane 64-bit addresses out of the tile loop
// (spilled to scratch, and every scratch reload then waits for the DMA in flight) and (b) track the DMA as pending
// VMEM.  Full tiles use the saddr form (uniform 64-bit tile base + 32-bit lane offset); M0 is saved and restored
// because the compiler reserves it.  No instruction offsets: an LDS-DMA op adds its offset to the LDS address too.
__device__ __forceinline__ uint32_t launder(uint32_t x) {  // opaque copy: stops loop-invariant hoisting
    uint32_t y;
    asm volatile("v_mov_b32 %0, %1" : "=v"(y) : "v"(x));
    return y;
}

__device__ __forceinline__ void pipe_issue(const ppe_kargs &a, uint32_t t, uint32_t slot, uint32_t lane_) {
    const uint32_t base = t << 6;
    const uint32_t lane = launder(lane_);
    uint32_t off[3];
#pragma unroll
    for (uint32_t k = 0; k < 3; ++k) {
        const uint32_t idx = 64u * k + lane;
        const uint32_t pk = (idx * 0xAAABu) >> 17;  // idx / 3 for idx < 192
        off[k] = pk * a.stride + 16u * (idx - 3u * pk);
    }
    uint32_t m0save;
    if (base + 64u <= a.n) {  // full tile
        const uint8_t *tb = a.hdr + (size_t)base * a.stride;
        const uint32_t *lb = a.len + base;
        asm volatile(
            "s_mov_b32 %[sv], m0\n\t"
            "s_mov_b32 m0, %[s0]\n\t"
            "s_nop 0\n\t"
            "global_load_lds_dwordx4 %[o0], %[tb]\n\t"
            "s_add_u32 m0, %[s0], 0x400\n\t"
            "s_nop 0\n\t"
            "global_load_lds_dwordx4 %[o1], %[tb]\n\t"
            "s_add_u32 m0, %[s0], 0x800\n\t"
            "s_nop 0\n\t"
            "global_load_lds_dwordx4 %[o2], %[tb]\n\t"
            "s_add_u32 m0, %[s0], 0xc00\n\t"
            "s_nop 0\n\t"
            "global_load_lds_dword %[o3], %[tb]\n\t"
            "s_add_u32 m0, %[s0], 0xd00\n\t"
            "s_nop 0\n\t"
            "global_load_lds_dword %[ol], %[lb]\n\t"
            "s_mov_b32 m0, %[sv]"
            : [sv] "=&s"(m0save)
            : [s0] "s"(slot), [o0] "v"(off[0]), [o1] "v"(off[1]), [o2] "v"(off[2]), [o3] "v"(lane * a.stride + 48u),
              [ol] "v"(lane * 4u), [tb] "s"(tb), [lb] "s"(lb)
            : "memory");
        return;
    }
    // the batch's partial last tile: clamp to the last packet, 64-bit per-lane addresses
    const uint32_t last = a.n - 1u;
    const uint8_t *g[4];
#pragma unroll
    for (uint32_t k = 0; k < 3; ++k) {
        const uint32_t idx = 64u * k + lane;
        const uint32_t pk = (idx * 0xAAABu) >> 17;
        g[k] = a.hdr + (size_t)min(base + pk, last) * a.stride + (off[k] - pk * a.stride);
    }
    const uint32_t p = min(base + lane, last);
    g[3] = a.hdr + (size_t)p * a.stride + 48u;
    const uint32_t *gl = a.len + p;
    asm volatile(
        "s_mov_b32 %[sv], m0\n\t"
        "s_mov_b32 m0, %[s0]\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %[g0], off\n\t"
        "s_add_u32 m0, %[s0], 0x400\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %[g1], off\n\t"
        "s_add_u32 m0, %[s0], 0x800\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %[g2], off\n\t"
        "s_add_u32 m0, %[s0], 0xc00\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dword %[g3], off\n\t"
        "s_add_u32 m0, %[s0], 0xd00\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dword %[gl], off\n\t"
        "s_mov_b32 m0, %[sv]"
        : [sv] "=&s"(m0save)
        : [s0] "s"(slot), [g0] "v"(g[0]), [g1] "v"(g[1]), [g2] "v"(g[2]), [g3] "v"(g[3]), [gl] "v"(gl)
        : "memory");
}

// Wait for every outstanding VMEM op of this wave (the slot's DMA, issued one tile earlier, and the previous tile's
// stores), then read this lane's packet from the slot.  In asm: the compiler cannot see which LDS bytes the DMA
// writes and would otherwise wait for it before every LDS access to the slot.
__device__ __forceinline__ void pipe_read(uint32_t slot, uint32_t lane, uint4 &q0, uint4 &q1, uint4 &q2, uint32_t &w12,
                                          uint32_t &len) {
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
    v4u r0, r1, r2;
    const uint32_t row = slot + 48u * lane, col = slot + 4u * lane;
    asm volatile(
        "s_waitcnt vmcnt(0)\n\t"
        "ds_read_b128 %0, %5\n\t"
        "ds_read_b128 %1, %5 offset:16\n\t"
        "ds_read_b128 %2, %5 offset:32\n\t"
        "ds_read_b32 %3, %6 offset:3072\n\t"
        "ds_read_b32 %4, %6 offset:3328\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&v"(r0), "=&v"(r1), "=&v"(r2), "=&v"(w12), "=&v"(len)
        : "v"(row), "v"(col)
        : "memory");
    q0 = make_uint4(r0.x, r0.y, r0.z, r0.w);
    q1 = make_uint4(r1.x, r1.y, r1.z, r1.w);
    q2 = make_uint4(r2.x, r2.y, r2.z, r2.w);
}

// PF: how the next tile's window is fetched while this one is classified
#define PF_NONE 0  // loaded at the top of its own iteration
#define PF_REG 1   // register double buffer: the next tile's loads are issued before this tile's compute
#define PF_LDS 2   // LDS-DMA slot (PIPE, above)
#define PF_HOIST 3 // as PF_NONE, but the first tile's loads are issued before the image staging

template <int MODE, int PF, int BLOCK>
__global__ __launch_bounds__(BLOCK, 8) void ppe_classify_kernel(ppe_kargs a) {
    constexpr bool PIPE = PF == PF_LDS;
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    // a separate LDS object from the image: the compiler then knows the slot DMA never aliases image reads
    __shared__ __attribute__((aligned(16))) uint32_t ring[PIPE ? BLOCK / 64 : 1][PIPE ? PIPE_SLOT_BYTES / 4 : 1];
    uint32_t *bins = smem;                   // [PPE_NBINS] packets per (status, flags) bin of this workgroup
    uint32_t *lcnt = smem + PPE_NBINS;       // [32] per-reason counters of this workgroup
    // IMG_LDS: per-wave walk keys (KEY_WAVE_WORDS per wave), then the staged classifier image
    constexpr uint32_t KEYW = MODE == IMG_LDS ? (BLOCK / 64) * KEY_WAVE_WORDS : 0u;
    uint32_t *lkeys = smem + PPE_NBINS + 32;
    uint32_t *limg = lkeys + KEYW;
    const uint32_t tid = threadIdx.x;
    const uint32_t lane = tid & 63u;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const uint32_t ntiles = (a.n + 63u) >> 6;
    const uint32_t stride_waves = gridDim.x * (BLOCK / 64);
    uint32_t tile = blockIdx.x * (BLOCK / 64) + wv;
    const uint32_t slot = PIPE ? (uint32_t)(uintptr_t)(lptr_t)&ring[wv][0] : 0u;
    const uint32_t twave = blockIdx.x * (BLOCK / 64) + wv;
    uint32_t titer = 0;
    bool titer_any = false;  // a tile was processed already (PF_HOIST: the first one was loaded in the prologue)
    TRACE_AT(0);
    if (PIPE && tile < ntiles) pipe_issue(a, tile, slot, lane);  // in flight during the image staging
    // current tile's window: bytes 0..51 (w[0..12]) and the wire length
    uint4 q0, q1, q2;
    uint32_t w12, qlen;
    // clamped (unconditional) loads of tile t's window into q*: a past-the-end lane re-reads the last packet
    auto load_tile = [&](uint32_t t) {
        const uint32_t pc = min((t << 6) + lane, a.n - 1u);
        const uint4 *r4 = (const uint4 *)(a.hdr + (size_t)pc * a.stride);
        q0 = r4[0]; q1 = r4[1]; q2 = r4[2];
        w12 = ((const uint32_t *)r4)[12];
        qlen = a.len[pc];
    };
    if (PF == PF_HOIST && tile < ntiles) load_tile(tile);  // first window in flight during the image staging

    for (uint32_t i = tid; i < PPE_NBINS + 32u; i += BLOCK) smem[i] = 0;
    uint32_t *keys = lkeys + (MODE == IMG_LDS ? wv * KEY_WAVE_WORDS + lane : 0u);  // this lane's slot 0
    if (MODE == IMG_LDS) keys[64u * PPE_NODE_LEAF] = 0u;                           // the leaves' zero key
    if (MODE != IMG_GLOBAL) stage_image<BLOCK>(a.img, limg, a.lds_words, tid);
    __syncthreads();
    TRACE_AT(1);
    const AclGeo geo = {a.lds_iters, a.max_depth, a.max_leaf, a.off_leaf, a.off_rules, a.off_resid, a.leaf_lds,
                        a.default_action};

    // action of each terminal status, 2 bits per status: FW for ACL_FW, PUNT for fragments / short windows, the
    // configured action for unsupported protocols (Decode_unsupport_proto_handle, decode.c:31-45), else DROP
    uint64_t act_table = 0;
#pragma unroll
    for (uint32_t st = 0; st < PPE_ST__COUNT; ++st) {
        const uint64_t ac = st == PPE_ST_ACL_FW ? PPE_ACT_FW
                          : (st == PPE_ST_L2_UNSUPPORT || st == PPE_ST_VLAN_UNSUPPORT || st == PPE_ST_IPV4_UNSUPPORT)
                              ? (a.unsup_fw ? PPE_ACT_FW : PPE_ACT_DROP)
                          : (st == PPE_ST_FRAG || st == PPE_ST_WINDOW_PUNT) ? PPE_ACT_PUNT : PPE_ACT_DROP;
        act_table |= ac << (2u * st);
    }

    if (PIPE && tile < ntiles) {
        pipe_read(slot, lane, q0, q1, q2, w12, qlen);
        if (tile + stride_waves < ntiles) pipe_issue(a, tile + stride_waves, slot, lane);
    }
    if (PF == PF_REG && tile < ntiles) load_tile(tile);
    for (; tile < ntiles; tile += stride_waves) {
        const uint32_t p = (tile << 6) + lane;
        const bool valid = p < a.n;
        if (PPE_TRACE && titer < 4) TRACE_AT(2 + 5 * titer);
        if (PF == PF_NONE || (PF == PF_HOIST && titer_any)) load_tile(tile);
        titer_any = true;
        if (PPE_TRACE) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (PPE_TRACE && titer < 4) TRACE_AT(3 + 5 * titer);
        const uint32_t w[16] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w,
                                q2.x, q2.y, q2.z, q2.w, w12, 0u, 0u, 0u};
        const uint32_t len = valid ? qlen : 0u;
        if (PF == PF_REG && tile + stride_waves < ntiles) load_tile(tile + stride_waves);
        Dec k = decode(w, len, a.hdr, p, a.stride, a.syn_check);

        uint32_t fh = 0, act;
        int32_t hit = -1;
        if (!(PPE_ABLATE & 8) && (k.flags & PPE_F_L4)) fh = flow_hashfn_l4(k.proto == 6u, k.sip, k.dip, k.sport, k.dport);
        if (PPE_TRACE && titer < 4) {
            asm volatile("" ::"v"(fh), "v"(k.st));  // decoded + hashed before the stamp
            TRACE_AT(4 + 5 * titer);
        }
        if ((PPE_ABLATE & 1) && valid && k.st == ST_ACL) {
            k.st = PPE_ST_ACL_FW;
            k.flags |= PPE_F_ACL;
        }
        if (!(PPE_ABLATE & 1) && valid && k.st == ST_ACL) {
            uint32_t rule_act;
            const MacFromWindow mac = {a.hdr, p, a.stride};
            if (MODE == IMG_LDS) {
                keys[0] = k.sip;
                keys[64] = k.dip;
                keys[128] = k.sport;
                keys[192] = k.dport;
                keys[256] = k.proto;
            }
            acl_lookup<MODE>(a.img, limg, keys, geo, k.sip, k.dip, k.sport, k.dport, k.proto, mac, a.ts, p, a.now, hit,
                             rule_act);
            const bool drop = rule_act == ACL_RULE_ACTION_DROP;  // flow.c:232-243, FlowHandlePacket :309
            k.st = drop ? (uint32_t)PPE_ST_ACL_DROP : (uint32_t)PPE_ST_ACL_FW;
            k.flags |= PPE_F_ACL;
        }
        const uint32_t st = k.st;
        act = (uint32_t)(act_table >> (2u * st)) & 3u;
        if (PPE_TRACE && titer < 4) {
            asm volatile("" ::"v"(hit), "v"(act));
            TRACE_AT(5 + 5 * titer);
        }

        // next tile: its DMA has had this whole tile's compute to land; take it into registers and start the one
        // after (the stores below are issued after this wait, so it never waits on this tile's own stores)
        if (PIPE && tile + stride_waves < ntiles) pipe_read(slot, lane, q0, q1, q2, w12, qlen);

        if (valid) {
            if (a.verdict) a.verdict[p] = st | (act << 8) | (k.flags << 16);
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

        // ---- wave-ballot compaction of FW / DROP indices into this tile's 64-slot segment of each list ----
        if (!(PPE_ABLATE & 4)) {
            const bool is_fw = valid && act == PPE_ACT_FW;
            const bool is_drop = valid && act == PPE_ACT_DROP;
            const uint64_t bfw = __ballot(is_fw);
            const uint64_t bdr = __ballot(is_drop);
            const uint32_t pfw = __builtin_amdgcn_mbcnt_hi((uint32_t)(bfw >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bfw, 0u));
            const uint32_t pdr = __builtin_amdgcn_mbcnt_hi((uint32_t)(bdr >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bdr, 0u));
            if (a.fw_idx && a.drop_idx) {  // both lists: one store instruction
                uint32_t *dst = is_fw ? a.fw_idx : a.drop_idx;
                if (is_fw || is_drop) dst[(tile << 6) + (is_fw ? pfw : pdr)] = p + a.idx_base;
            } else {
                if (a.fw_idx && is_fw) a.fw_idx[(tile << 6) + pfw] = p + a.idx_base;
                if (a.drop_idx && is_drop) a.drop_idx[(tile << 6) + pdr] = p + a.idx_base;
            }
            const uint32_t nv = (uint32_t)__popcll(__ballot(valid));  // (a ballot outside the lane-0 branch)
            if (a.tile_cnt && lane == 0) {
                const uint32_t nfw = (uint32_t)__popcll(bfw), ndr = (uint32_t)__popcll(bdr);
                a.tile_cnt[tile] = nfw | (ndr << 8) | ((nv - nfw - ndr) << 16);
            }
        }

        // ---- per-reason counters: one LDS add per packet into its (status, flags) bin ----
        if (!(PPE_ABLATE & 2) && valid)
            atomicAdd(&bins[st | ((k.flags & PPE_F_VLAN) ? 32u : 0u) | ((k.flags & PPE_F_TCP) ? 64u : 0u) |
                            ((k.flags & PPE_F_L4) ? 128u : 0u)],
                      1u);
        if (PPE_TRACE && titer < 4) TRACE_AT(6 + 5 * titer);
        ++titer;
        // the slot was emptied by pipe_read above; refill it with the tile after next (issued here, where little
        // is live, rather than right after the read)
        if (PIPE && tile + 2u * stride_waves < ntiles) pipe_issue(a, tile + 2u * stride_waves, slot, lane);
    }

    TRACE_AT(22);
    if (PPE_TRACE && lane == 0 && a.trace) a.trace[(size_t)twave * 32u + 31u] = titer;
    __syncthreads();
    for (uint32_t b = tid; b < PPE_NBINS; b += BLOCK) {  // expand the bins into counter increments
        const uint32_t c = bins[b];
        if (c) {
            for (uint32_t cb = bin_counters(b, act_table); cb; cb &= cb - 1u) atomicAdd(&lcnt[__builtin_ctz(cb)], c);
        }
    }
    __syncthreads();
    if (tid < PPE_C__COUNT) a.cslots[(size_t)blockIdx.x * PPE_CSLOT_WORDS + tid] += lcnt[tid];
}

// ACL-only lookup over pre-decoded tuples (the DP_Acl_Lookup(mbuf) entry, dataplane/src/flow/flow.c:232):
// tuple = {sip, dip, sport | dport << 16, proto}, macs = {dmac lo, dmac hi, smac lo, smac hi} (optional).
template <bool LDS_IMG>
__global__ __launch_bounds__(PPE_BLOCK) void ppe_acl_tuple_kernel(ppe_tuple_kargs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    const uint32_t tid = threadIdx.x;
    constexpr uint32_t KEYW = LDS_IMG ? (PPE_BLOCK / 64) * KEY_WAVE_WORDS : 0u;
    uint32_t *keys = smem + (tid >> 6) * KEY_WAVE_WORDS + (tid & 63u);
    uint32_t *limg = smem + KEYW;
    if (LDS_IMG) {
        keys[64u * PPE_NODE_LEAF] = 0u;
        stage_image<PPE_BLOCK>(a.img, limg, a.img_words, tid);
        __syncthreads();
    }
    const uint32_t depth = a.img[PPE_IMG_W_MAXDEPTH];
    const AclGeo geo = {LDS_IMG ? depth : 0u, depth, a.img[PPE_IMG_W_MAXLEAF], a.img[PPE_IMG_W_OFFLEAF],
                        a.img[PPE_IMG_W_OFFRULES], a.img[PPE_IMG_W_OFFRESID], LDS_IMG ? 1u : 0u, a.default_action};
    for (uint32_t i = blockIdx.x * PPE_BLOCK + tid; i < a.n; i += gridDim.x * PPE_BLOCK) {
        const uint4 t = ((const uint4 *)a.tuple)[i];
        uint4 m = make_uint4(0, 0, 0, 0);
        if (a.macs) m = ((const uint4 *)a.macs)[i];
        int32_t hit;
        uint32_t act;
        const MacValues mac = {m.x, m.y, m.z, m.w};
        if (LDS_IMG) {
            keys[0] = t.x;
            keys[64] = t.y;
            keys[128] = t.z & 0xffffu;
            keys[192] = t.z >> 16;
            keys[256] = t.w & 0xffu;
        }
        if (LDS_IMG)
            acl_lookup<IMG_LDS>(a.img, limg, keys, geo, t.x, t.y, t.z & 0xffffu, t.z >> 16, t.w & 0xffu, mac, a.ts, i, a.now,
                                hit, act);
        else
            acl_lookup<IMG_GLOBAL>(a.img, limg, keys, geo, t.x, t.y, t.z & 0xffffu, t.z >> 16, t.w & 0xffu, mac, a.ts, i,
                                   a.now, hit, act);
        if (a.hit) a.hit[i] = hit;
        if (a.action) a.action[i] = act;
    }
}

}  // namespace

template <int M, int P, int B>
static int launch_t(const ppe_kargs *a, uint32_t grid, size_t shmem, hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
    // hipExtLaunchKernelGGL's events are the dispatch packet's own start/end timestamps (what rocprofv3 reports),
    // unlike hipEventRecord markers around the launch
    hipExtLaunchKernelGGL((ppe_classify_kernel<M, P, B>), dim3(grid), dim3(B), shmem, s, e0, e1, 0, *a);
    return (int)hipGetLastError();
}

template <int M, int P, int B>
static int occ_t(size_t shmem) {
    int nb = 0;
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, ppe_classify_kernel<M, P, B>, B, shmem) == hipSuccess
               ? nb : -1;
}

static size_t classify_shmem(uint32_t lds_words, int mode, int block) {
    const size_t base = (PPE_NBINS + 32u) * sizeof(uint32_t);  // counter bins + per-reason counters
    if (mode == IMG_GLOBAL) return base;
    const size_t keys = mode == IMG_LDS ? (size_t)(block / 64) * KEY_WAVE_WORDS * 4u : 0u;
    return base + keys + (((size_t)lds_words * 4u + 1023u) & ~(size_t)1023u);
}

#define PPE_DISPATCH_B(FN, M, P, ...)                                \
    do {                                                             \
        if (block == 1024) return FN<M, P, 1024>(__VA_ARGS__);       \
        if (block == 512) return FN<M, P, 512>(__VA_ARGS__);         \
        return FN<M, P, 256>(__VA_ARGS__);                           \
    } while (0)
#define PPE_DISPATCH_P(FN, M, ...)                                   \
    do {                                                             \
        if (pipe == PF_LDS) PPE_DISPATCH_B(FN, M, PF_LDS, __VA_ARGS__); \
        if (pipe == PF_REG) PPE_DISPATCH_B(FN, M, PF_REG, __VA_ARGS__); \
        if (pipe == PF_HOIST) PPE_DISPATCH_B(FN, M, PF_HOIST, __VA_ARGS__); \
        PPE_DISPATCH_B(FN, M, PF_NONE, __VA_ARGS__);                 \
    } while (0)
#define PPE_DISPATCH_Q(FN, M, ...)                                   \
    do {                                                             \
        if (pipe == PF_REG) PPE_DISPATCH_B(FN, M, PF_REG, __VA_ARGS__); \
        if (pipe == PF_HOIST) PPE_DISPATCH_B(FN, M, PF_HOIST, __VA_ARGS__); \
        PPE_DISPATCH_B(FN, M, PF_NONE, __VA_ARGS__);                 \
    } while (0)
// the LDS-DMA pipeline is built for the whole-image-in-LDS variant only: with tree nodes or rules read from global
// memory every such load waits (in-order vmcnt) for the next tile's DMA, which defeats the overlap
#define PPE_DISPATCH(FN, ...)                                        \
    do {                                                             \
        if (mode == IMG_LDS) PPE_DISPATCH_P(FN, IMG_LDS, __VA_ARGS__);     \
        if (mode == IMG_SPLIT) PPE_DISPATCH_Q(FN, IMG_SPLIT, __VA_ARGS__); \
        PPE_DISPATCH_Q(FN, IMG_GLOBAL, __VA_ARGS__);                 \
    } while (0)

extern "C" int ppe_launch_classify(const ppe_kargs *a, uint32_t grid, int mode, int pipe, int block, void *stream,
                                   void *ev_start, void *ev_stop) {
    const size_t shmem = classify_shmem(a->lds_words, mode, block);
    hipStream_t s = (hipStream_t)stream;
    hipEvent_t e0 = (hipEvent_t)ev_start, e1 = (hipEvent_t)ev_stop;
    PPE_DISPATCH(launch_t, a, grid, shmem, s, e0, e1);
}

// resident workgroups per CU for the kernel variant (the persistent grid is sized to exactly fill the chip)
extern "C" int ppe_classify_occupancy(uint32_t lds_words, int mode, int pipe, int block) {
    const size_t shmem = classify_shmem(lds_words, mode, block);
    PPE_DISPATCH(occ_t, shmem);
}

// static LDS of the pipelined kernel (the per-wave DMA slots), for the engine's LDS budget
extern "C" uint32_t ppe_classify_pipe_lds(int block) { return (uint32_t)(block / 64) * PIPE_SLOT_BYTES; }
// dynamic LDS of the whole-image-in-LDS variant beyond counters + image (the per-wave walk keys)
extern "C" uint32_t ppe_classify_keys_lds(int block) { return (uint32_t)(block / 64) * KEY_WAVE_WORDS * 4u; }

extern "C" int ppe_launch_acl_tuples(const ppe_tuple_kargs *a, uint32_t grid, int lds_img, void *stream) {
    if (lds_img) {
        const size_t shmem = (size_t)(PPE_BLOCK / 64) * KEY_WAVE_WORDS * 4u +
                             (((size_t)a->img_words * 4u + 1023u) & ~(size_t)1023u);
        hipLaunchKernelGGL(ppe_acl_tuple_kernel<true>, dim3(grid), dim3(PPE_BLOCK), shmem, (hipStream_t)stream, *a);
    } else {
        hipLaunchKernelGGL(ppe_acl_tuple_kernel<false>, dim3(grid), dim3(PPE_BLOCK), 0, (hipStream_t)stream, *a);
    }
    return (int)hipGetLastError();
}
