/*
 * ppe_kernels.hip — the MI355X (gfx950) decode + 5-tuple ACL classify kernel.
 *
 * One lane per packet, one 64-packet tile per wavefront, persistent grid (wave w of the grid takes tiles w, w + W,
 * ...).  Per packet:
 *   1. load the first 52 B of the header window (3 × 16-B loads + 1 dword) and the wire length;
 *   2. decode Ethernet → [VLAN] → IPv4 → UDP|TCP exactly as the reference dataplane (big-endian field values,
 *      the reference's check order and uint16/uint8 arithmetic — citations inline);
 *   3. flow_hashfn (TluHash ×3, dataplane/src/flow/tluhash.h:7-35);
 *   4. on the flow-miss path: syn_check, then the ACL decision-tree walk (image v3, ppe_image.h: one LDS round trip
 *      and four VALU per level, the classifier staged in LDS when it fits) and the leaf's rule check;
 *   5. SoA verdict / hash / hit stores, wave-ballot compaction of FW/DROP indices per tile, and per-reason counters
 *      (one LDS add per packet into its (status, flags) bin, expanded once per workgroup into that workgroup's own
 *      counter slot — no contended global atomics).
 * No MFMA: integer bitfield / compare work bound by HBM bandwidth and VALU issue.
 *
 * LDS layout of a workgroup (dynamic shared memory, nothing static):
 *   [0, KEYB)              per-wave walk keys: wave w, key slot d, lane l at w * 1536 + d * 256 + 4 l (slot 5 = 0)
 *   [KEYB, KEYB + 1152)    256 counter bins + 32 per-reason counters
 *   [IMGB, ...)            the staged classifier image (all of it, or a prefix), 1-KB padded
 * KEYB and IMGB are compile-time constants of the workgroup size, so a node at image byte offset o is read from LDS
 * address IMGB + o with IMGB in the instruction's offset field.
 */
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include "ppe_hip.h"
#include "ppe_image.h"
#include "ppe_internal.h"

// Diagnostic ablation builds only (make ablate): bit 0 skip the ACL walk, bit 1 skip counters, bit 2 skip the
// compaction, bit 3 skip the flow hash, bit 4 skip the flow-counter atomics, bit 5 skip the flow last-seen stores.
// The product build has PPE_ABLATE == 0.
#ifndef PPE_ABLATE
#define PPE_ABLATE 0
#endif
// minimum resident waves per SIMD the single-tile classify kernel is compiled for (VGPR budget 512 / this)
#ifndef PPE_WAVES_PER_EU
#define PPE_WAVES_PER_EU 8
#endif

namespace {

typedef __attribute__((address_space(1))) const void *gptr_t;
typedef __attribute__((address_space(3))) void *lptr_t;
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

// ---------------------------------------------------------------------------------------------------------------
// LDS geometry
#define KEY_SLOTS 6u
#define KEY_WAVE_BYTES (KEY_SLOTS * 256u)  // 1536
// KEYS = false: block and cut-list walks keep the keys in registers and have no key slots, so their image starts
// right after the counter bins (24 KB more image per CU at 1024 threads)
// QB: the flow-table kernel's owner-update buckets, between the counter bins and the image
template <int BLOCK, bool KEYS = true, uint32_t QB = 0> struct Lds {
    static constexpr uint32_t KEYB = KEYS ? (BLOCK / 64) * KEY_WAVE_BYTES : 0u;
    static constexpr uint32_t BINS = KEYB;                   // 256 u32 bins, then 32 u32 counters
    static constexpr uint32_t QUEUE = KEYB + PPE_LDS_FIXED;  // 16-B aligned (1152 = 72 × 16)
    static constexpr uint32_t IMGB = QUEUE + QB;
};

// LDS accesses by byte address (the compiler folds constant parts into the instruction offset)
__device__ __forceinline__ uint32_t lds_u32(uint32_t addr) {
    return *(const __attribute__((address_space(3))) uint32_t *)(uintptr_t)addr;
}
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 lds_u128(uint32_t addr) {
    const u32x4 v = *(const __attribute__((address_space(3))) u32x4 *)(uintptr_t)addr;
    return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void lds_st32(uint32_t addr, uint32_t v) {
    *(__attribute__((address_space(3))) uint32_t *)(uintptr_t)addr = v;
}
// global accesses by 32-bit byte offset from a uniform base (the saddr form: no 64-bit address math per lane)
// (explicitly global: a select between two output pointers must not degrade to a flat store, whose out-of-order
// completion makes the compiler wait for vmcnt(0) at the next use of any load)
template <class T> struct GType { typedef T type; };
template <> struct GType<uint4> { typedef uint32_t __attribute__((ext_vector_type(4))) type; };
template <> struct GType<uint2> { typedef uint32_t __attribute__((ext_vector_type(2))) type; };
template <class T> __device__ __forceinline__ T gld(const void *base, uint32_t off) {
    typedef typename GType<T>::type G;
    return __builtin_bit_cast(T, *(const __attribute__((address_space(1))) G *)((const char *)base + off));
}
template <class T> __device__ __forceinline__ void gst(void *base, uint32_t off, T v) {
    typedef typename GType<T>::type G;
    *(__attribute__((address_space(1))) G *)((char *)base + off) = __builtin_bit_cast(G, v);
}
// Per-packet result streams (verdict, hash, hit, compacted lists, tuple): written once, read by the consumer after
// the launch, so they go out with the non-temporal (streaming) policy.  The memory skeleton of this kernel
// (tools/calib/stream_calib2.hip) runs 3-6 % faster with it; non-temporal LOADS of the windows run 25 % slower
// (the 4 partial-line loads of a row would each refetch the line), so the loads keep the default policy.
template <class T> __device__ __forceinline__ void gst_nt(void *base, uint32_t off, T v) {
    typedef typename GType<T>::type G;
    __builtin_nontemporal_store(__builtin_bit_cast(G, v), (__attribute__((address_space(1))) G *)((char *)base + off));
}

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
    constexpr uint64_t K1 =  // st 12..19
        ((uint64_t)PPE_C_IPV4_UNSUPPORT << 0) | ((uint64_t)PPE_C_UDP_HEADERLEN_ERR << 5) |
        ((uint64_t)PPE_C_UDP_PKTLEN_ERR << 10) | ((uint64_t)PPE_C_TCP_HEADERLEN_ERR << 15) |
        ((uint64_t)PPE_C_TCP_PKTLEN_ERR << 20) | ((uint64_t)PPE_C_FLOW_TCP_NO_SYN_FIRST << 25) |
        ((uint64_t)PPE_C_WINDOW_PUNT << 30) | ((uint64_t)PPE_C_FLOW_NODE_NOMEM << 35);
    const bool lo = st < 12u;
    return (uint32_t)(((lo ? K0 : K1) >> (5u * (lo ? st : st - 12u))) & 31u);
}

// Synchronous global loads for the rare paths (IPv4 options, MAC / time-window rules).  Inline asm with its own
// wait, so the compiler tracks no pending VMEM result across the tile loop.
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
__device__ __forceinline__ uint32_t ld_u32_sync(const uint32_t *q) {
    uint32_t v;
    asm volatile("global_load_dword %0, %1, off\n\ts_waitcnt vmcnt(0)" : "=&v"(v) : "v"(q) : "memory");
    return v;
}
__device__ __forceinline__ uint64_t ld_u64_sync(const uint64_t *q) {
    uint64_t v;
    asm volatile("global_load_dwordx2 %0, %1, off\n\ts_waitcnt vmcnt(0)" : "=&v"(v) : "v"(q) : "memory");
    return v;
}

// DecodeTCPOptions (dataplane/src/decode/decode-tcp.c:18-131) over a TCP header's options in the window `row`:
// opt = Dec.tcpopt.  Returns the byte offset of the first valid window-scale option (type 3, length 3) from the TCP
// header, what the reference records as m->tcpvars.ws (:61-70, a duplicate is ignored), or 0; | PPE_TUPLE_OPT_PAST
// >> 9 when no such option was found before the parse needed a byte past the header window (the reference reads
// the whole option space, which lies inside the packet: hlen <= l4len, decode-tcp.c:149; the answer for such a
// packet needs a wider window, e.g. Decode's 144 B).  A recorded option is final (the first one counts), so the parse
// stops there.  Rare path (tuple output only): dword loads with their own wait.
__device__ __forceinline__ uint32_t tcp_ws_offset(const uint8_t *row, uint32_t opt) {
    const uint32_t th = opt & 0xffu, avail = opt >> 16;
    uint32_t plen = (opt >> 8) & 0xffu, pos = th + 20u, dwi = ~0u, dw = 0;
    bool past = false;
    auto byte_at = [&](uint32_t b) -> uint32_t {
        if (b >= avail) {  // (option bytes lie below the wire length: past the window)
            past = true;
            return 0u;
        }
        if ((b >> 2) != dwi) {
            dwi = b >> 2;
            dw = ld_u32_sync((const uint32_t *)row + dwi);
        }
        return (dw >> (8u * (b & 3u))) & 0xffu;
    };
#pragma unroll 1
    while (plen) {
        const uint32_t t = byte_at(pos);
        if (t == 0u) break;  // EOL (or past the window)
        if (t == 1u) {       // NOP
            ++pos;
            --plen;
            continue;
        }
        if (plen < 2u) break;
        const uint32_t ol = byte_at(pos + 1u);
        if (past || ol > plen || ol < 2u) break;  // invalid length: return -1 (the option already recorded stays)
        if (t == 3u && ol == 3u) return pos - th;
        pos += ol;
        plen -= ol;
    }
    return past ? (PPE_TUPLE_OPT_PAST >> 9) : 0u;
}

// Where a residual MAC rule gets the packet's MACs: re-read from the header window (classify kernel: rare path, keeps
// the MACs out of registers during the walk) or given by value (tuple kernel).
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

// Per-reason counters are a function of the final (status, VLAN / L4 / TCP flags) of a packet, so the kernel only
// counts packets per bin key = status | (flags & 7) << 5 (VLAN bit 5, L4 bit 6, TCP bit 7; one LDS add per packet)
// and expands each non-empty bin into counter increments once per workgroup.  The rules (same as the reference's
// pktstat updates):
//   every packet: PKTS and its terminal reason (decode-statistic.h:239-327; ACL_FW / ACL_DROP for the ACL path)
//   L2_RX_OK unless the Ethernet layer failed; VLAN_RX_OK for a parsed tag that was not of an unsupported type;
//   IPV4_RX_OK when the packet reached the TCP/UDP decoder; UDP_RX_OK / TCP_RX_OK when it reached the flow engine;
//   FLOW_PROC_OK / _FAIL by the flow engine's outcome; OUT_FW / OUT_DROP / OUT_PUNT by the action.
#define PPE_NBINS 256u
static_assert(PPE_F_VLAN == 1u && PPE_F_L4 == 2u && PPE_F_TCP == 4u, "bin key layout");
__device__ __forceinline__ uint32_t bin_counters(uint32_t key, uint64_t act_table) {
    const uint32_t st = key & 31u;
    const bool vl = (key >> 5) & 1u, l4 = (key >> 6) & 1u, tcp = (key >> 7) & 1u;
    uint32_t cb = CB(PPE_C_PKTS) | CB(reason_counter(st));
    if (st != PPE_ST_L2_HEADER_ERR && st != PPE_ST_L2_UNSUPPORT) cb |= CB(PPE_C_L2_RX_OK);
    if (vl && st != PPE_ST_VLAN_UNSUPPORT) cb |= CB(PPE_C_VLAN_RX_OK);
    const bool l4_in = st == PPE_ST_ACL_FW || st == PPE_ST_ACL_DROP || st == PPE_ST_UDP_HEADER_ERR ||
                       st == PPE_ST_UDP_LEN_ERR || st == PPE_ST_TCP_HEADER_ERR || st == PPE_ST_TCP_LEN_ERR ||
                       st == PPE_ST_FLOW_TCP_NO_SYN_FIRST || st == PPE_ST_WINDOW_PUNT || st == PPE_ST_FLOW_NOMEM;
    if (l4_in) cb |= CB(PPE_C_IPV4_RX_OK);
    if (l4 && !tcp) cb |= CB(PPE_C_UDP_RX_OK);
    if (tcp) cb |= CB(PPE_C_TCP_RX_OK);
    if (st == PPE_ST_FLOW_TCP_NO_SYN_FIRST || st == PPE_ST_ACL_DROP || st == PPE_ST_FLOW_NOMEM)
        cb |= CB(PPE_C_FLOW_PROC_FAIL);
    if (st == PPE_ST_FLOW_NOMEM) cb |= CB(PPE_C_ACL_FW);  // counted before FlowAdd failed (flow.c:240)
    if (st == PPE_ST_ACL_FW) cb |= CB(PPE_C_FLOW_PROC_OK);
    const uint32_t act = (uint32_t)(act_table >> (2u * st)) & 3u;
    cb |= act == PPE_ACT_FW ? CB(PPE_C_OUT_FW) : (act == PPE_ACT_DROP ? CB(PPE_C_OUT_DROP) : CB(PPE_C_OUT_PUNT));
    return cb;
}

struct Dec {
    uint32_t st, flags;
    uint32_t sip, dip, sport, dport, proto, paylen;
    uint32_t tcpopt;  // TCP with options: window byte offset of the TCP header | option bytes << 8 | avail << 16
};

// Decode of one packet, straight-line: every check of the reference is evaluated, then the terminal status is
// chosen by applying the checks in REVERSE order of the reference's control flow, so the first failing check
// (the one the reference returns on) wins.  w[0..12] = first 52 bytes (little-endian dwords); hdr / p = the packet's
// window in global memory (read only for L4 headers behind IPv4 options).
// TUP (kernels that may write the tuple output): a fragment's sport / dport / paylen carry what DecodeIPV4 records
// for Defrag instead (decode-ipv4.c:106-109): ip_id, the fragment offset in bytes and frag_len (ppe_hip.h tuple).
template <bool TUP = true>
__device__ __forceinline__ Dec decode(const uint32_t (&w)[13], uint32_t len32, const uint8_t *hdr, uint32_t p,
                                      uint32_t stride, uint32_t syn_check) {
    Dec k;
    const uint32_t len = len32 & 0xffffu;  // Decode passes (uint16_t)pkt_totallen, decode.c:22
    // ---- Ethernet: dataplane/src/decode/decode-ethernet.c:23-115 ----
    const bool bad_len = len < 14u;                               // :29-34
    const bool dz = (w[0] | (w[1] & 0xffffu)) == 0u;              // :38-44 dst MAC all zero
    const bool sz = ((w[1] >> 16) | w[2]) == 0u;                  // :45-51 src MAC all zero
    const uint32_t etype = w[3] & 0xffffu;                        // bytes 12-13, little-endian view
    const bool is_ip = etype == 0x0008u;                          // ETHERNET_TYPE_IP 0x0800, :75
    const bool is_vl = (etype | 0x0010u) == 0x0091u;              // 0x8100 or 0x9100, :96-97
    const bool l2_bad = bad_len | dz | sz;
    const bool l2_ok = !l2_bad & (is_ip | is_vl);
    // ---- VLAN: dataplane/src/decode/decode-vlan.c:23-89 ----
    const uint32_t vlen = len - 14u;
    const uint32_t itype = w[4] & 0xffffu;
    const bool v_ip = itype == 0x0008u, v_vl = (itype | 0x0010u) == 0x0091u;
    const uint32_t v = is_vl ? 1u : 0u;
    const uint32_t l3len = vlen - 4u * v;
    // ---- IPv4: dataplane/src/decode/decode-ipv4.c:27-247.  L3 starts at byte 14 + 4v = 4*(3+v) + 2.
    // D[i] = dword (3 + v + i); a VLAN-free wave takes w[3 + i] as is (wave-uniform branch)
    uint32_t D[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) D[i] = w[3 + i];
    if (__builtin_amdgcn_ballot_w64(is_vl) != 0) {
#pragma unroll
        for (int i = 0; i < 9; ++i) D[i] = is_vl ? w[4 + i] : w[3 + i];
    }
    const uint32_t verhl = (D[0] >> 16) & 0xffu;
    const uint32_t hlen = (verhl & 0xfu) << 2;
    const uint32_t iplen = be16_lo(D[1]);
    const uint32_t sip = __builtin_bswap32((D[3] >> 16) | (D[4] << 16));  // src_addr, L3+12
    const uint32_t dip = __builtin_bswap32((D[4] >> 16) | (D[5] << 16));  // dst_addr, L3+16
    const uint32_t proto = D[2] >> 24;                                     // ip_proto, L3+9
    const uint32_t ipoff = be16_lo(D[2]);                                  // ip_off, L3+6
    const bool l3_in = l2_ok & (is_ip | ((vlen >= 4u) & v_ip));
    const bool ip_ok = l3_in & (l3len >= 20u) & ((verhl >> 4) == 4u) & (hlen >= 20u) & (iplen >= hlen) &
                       (l3len >= iplen);
    const bool frag = ((ipoff & 0x3fffu) != 0u) & (proto != 89u);         // IPV4_IS_FRAGMENT && !OSPF, :102
    const bool is_tcp = proto == 6u, is_udp = proto == 17u;
    const bool l4_in = ip_ok & !frag & (is_tcp | is_udp);
    const uint32_t l4len = (iplen - hlen) & 0xffffu;
    const uint32_t l4off = 14u + 4u * v + hlen;
    const bool fast = hlen == 20u;  // L4 at byte 34+4v: every field below byte 52, in registers
    const bool win_short = !fast & (l4off + (is_tcp ? 14u : 6u) > stride);
    uint32_t sport = be16_hi(D[5]), dport = be16_lo(D[6]);
    uint32_t x = is_tcp ? (D[8] >> 16) : be16_hi(D[6]);  // TCP: offx2 | flags << 8;  UDP: uh_len
    if (l4_in & !fast & !win_short) {  // IPv4 options: L4 header at a data-dependent offset
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
    st_tcp = ((l4len < thl) | (((thl - 20u) & 0xffu) > 40u)) ? (uint32_t)PPE_ST_TCP_LEN_ERR : st_tcp;  // :149-160
    st_tcp = win_short ? (uint32_t)PPE_ST_WINDOW_PUNT : st_tcp;
    st_tcp = l4len < 20u ? (uint32_t)PPE_ST_TCP_HEADER_ERR : st_tcp;  // :140-144
    uint32_t st_udp = l4len != x ? (uint32_t)PPE_ST_UDP_LEN_ERR : ST_ACL;  // :26-36
    st_udp = win_short ? (uint32_t)PPE_ST_WINDOW_PUNT : st_udp;
    st_udp = l4len < 8u ? (uint32_t)PPE_ST_UDP_HEADER_ERR : st_udp;  // :18-22
    uint32_t st = is_tcp ? st_tcp : (is_udp ? st_udp : (uint32_t)PPE_ST_IPV4_UNSUPPORT);  // decode-ipv4.c:233-243
    st = frag ? ((((l3len - hlen) & 0xffffu) == 0u) ? (uint32_t)PPE_ST_FRAG_LEN_ERR : (uint32_t)PPE_ST_FRAG) : st;
    st = ((iplen < hlen) | (l3len < iplen)) ? (uint32_t)PPE_ST_IPV4_LEN_ERR : st;  // decode-ipv4.c:50-60
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
    st = l2_bad ? (uint32_t)PPE_ST_L2_HEADER_ERR : st;

    const bool l4_ok = (st == ST_ACL) | (st == PPE_ST_FLOW_TCP_NO_SYN_FIRST);  // reached FlowHandlePacket
    // DecodeTCPOptions (decode-tcp.c:175-177) runs for every TCP header that passed its length checks; only the
    // tuple output reports what it records (the window-scale option), so the PART kernel never reads this
    k.tcpopt = (l4_ok & is_tcp & (thl > 20u)) ? l4off | ((thl - 20u) << 8) | (min(len, stride) << 16) : 0u;
    k.st = st;
    k.flags = ((l2_ok & is_vl & (vlen >= 4u)) ? PPE_F_VLAN : 0u) | (l4_ok ? PPE_F_L4 : 0u) |
              ((l4_ok & is_tcp) ? PPE_F_TCP : 0u) | ((l4_ok & is_tcp & syn) ? PPE_F_SYN : 0u) |
              ((ip_ok & frag) ? PPE_F_FRAG : 0u);
    // zeroed by masks, not selects: ROCm 7.2 miscompiles the select form (dport zeroed for NO_SYN packets;
    // profiles/r3_select_miscompile.md, tools/repro_select_miscompile.sh)
    const uint32_t ipm = ip_ok ? ~0u : 0u, l4m = l4_ok ? ~0u : 0u;
    k.sip = sip & ipm;
    k.dip = dip & ipm;
    k.proto = proto & ipm;
    k.sport = sport & l4m;
    k.dport = dport & l4m;
    k.paylen = (is_tcp ? l4len - thl : l4len - 8u) & l4m;
    if constexpr (TUP) {  // fragments (status FRAG / FRAG_LEN_ERR): defrag_id, frag_offset, frag_len
        const uint32_t fm = (ip_ok & frag) ? ~0u : 0u;
        k.sport |= be16_hi(D[1]) & fm;                       // ip_id, L3+4
        k.dport |= ((ipoff & 0x1fffu) << 3) & fm;            // IPV4_GET_IPOFFSET << 3, uint16
        k.paylen |= ((l3len - hlen) & 0xffffu) & fm;         // len - ihl, uint16
    }
    return k;
}

// Image staging modes:
//   IMG_GLOBAL  the whole classifier image is read from global memory (L1/L2/MALL-cached)
//   IMG_LDS     the whole image is staged in LDS
//   IMG_SPLIT   a prefix [0, lds_words) is staged: header, the top of the BFS tree (every node of the first
//               lds_iters levels) and, when the prefix reaches them, the leaf lists and the rule records
#define IMG_GLOBAL 0
#define IMG_LDS 1
#define IMG_SPLIT 2

// Classifier geometry for one launch (host-computed from the image header, ppe_image.h).
struct AclGeo {
    uint32_t lds_iters;   // IMG_SPLIT: walk levels read from LDS
    uint32_t max_depth;   // deepest leaf: levels 0..max_depth, max_depth + 1 node reads
    uint32_t max_leaf;    // longest leaf candidate list
    uint32_t root_ks;     // the root's key slot << 8
    uint32_t off_leaf, off_rules, off_resid;  // words
    uint32_t lds_words;   // staged prefix (words)
    uint32_t default_action;
    uint32_t jump;        // jump root (image word PPE_IMG_W_JUMP): dim | shift << 8 | bits << 16, 0 = none
    uint32_t off_nodes;   // words (the jump table is [PPE_IMG_HDR_WORDS, off_nodes))
    // multi-tile walks (2-level blocks, ppe_image.h block section)
    uint32_t lds_blocks;  // blocks [0, lds_blocks) in LDS
    uint32_t bsec_lds, blk_lds;  // LDS byte offsets from the staged image base: block jump table, block 0
    uint32_t off_bsec, off_blocks, max_bdepth;
    // compact leaves (image v6): record / index-table word offsets (0 = none), and their LDS byte offsets from the
    // staged image base (~0u = read from global memory)
    uint32_t off_crec, off_idtab, crec_lds, idtab_lds;
    // cut lists (image v8): header word 0 (sip bits | dip bits << 8 | PPE_CUT_IDS16), word offsets of the length
    // slices / group bases / fingerprints / entry lines, entries per line and its divisor magic, and the LDS byte
    // offsets of the bases, fingerprints and entry lines from the staged image base (the slices are at it; the entry
    // lines only when the mode is IMG_LDS)
    uint32_t cut, cut_slc, cut_gbase, cut_fp, cut_ent, cut_epl, cut_div, cut_idrel, cut_gbase_lds, cut_fp_lds,
        cut_ent_lds;
};

// One level of the walk, node and key both in flight: the node's child pointer carries the child's key slot, so
// the key read of the next level needs no node read first.  4 VALU: compare, child select, slot select, address.
__device__ __forceinline__ void walk_step(uint4 nd, uint32_t key, uint32_t lanebase, uint32_t &noff, uint32_t &kaddr) {
    const bool gt = key > nd.x;
    noff = gt ? nd.z : nd.y;
    kaddr = lanebase + (gt ? (nd.w >> 16) : (nd.w & 0xffffu));
}

// Tree walk to a leaf; returns the leaf node.  Keys come from this lane's LDS key slots (lanebase).  Levels read
// from the staged image in LDS run a wave-uniform trip count (a lane at a leaf stays there); the rest read global
// memory with a per-lane exit (a finished lane must not keep reading L2 / HBM).
template <int MODE, int IMGB>
__device__ __forceinline__ uint4 acl_walk(const uint32_t *__restrict__ gimg, const AclGeo &g, uint32_t lanebase) {
    uint32_t noff = 4u * PPE_IMG_HDR_WORDS, kaddr = lanebase + g.root_ks;
    if (g.jump) {
        // jump root (image v4): bucket = key[dim] >> shift picks this lane's subtree root and its key slot
        const uint32_t key = lds_u32(lanebase + ((g.jump & 0xffu) << 8));
        const uint32_t jo = 4u * PPE_IMG_HDR_WORDS + 4u * (key >> ((g.jump >> 8) & 0xffu));
        // (IMG_LDS: always staged — no global-load path, whose merge would wait on every outstanding load)
        const uint32_t e = (MODE == IMG_LDS || (MODE == IMG_SPLIT && g.lds_words >= g.off_nodes))
                               ? lds_u32(IMGB + jo) : gld<uint32_t>(gimg, jo);
        noff = e & 0xffffffu;
        kaddr = lanebase + ((e >> 16) & 0xff00u);
    }
    uint4 nd = make_uint4(0u, 0u, 0u, 0u);
    uint32_t it = 0;
    if (MODE != IMG_GLOBAL) {
        const uint32_t n_lds = MODE == IMG_LDS ? g.max_depth + 1u : g.lds_iters;
#pragma unroll 2
        for (; it < n_lds; ++it) {
            const uint32_t key = lds_u32(kaddr);
            nd = lds_u128(IMGB + noff);
            walk_step(nd, key, lanebase, noff, kaddr);
        }
    }
    if (MODE != IMG_LDS) {
        bool at_leaf = it > 0u && nd.x == PPE_LEAF_THR;
#pragma unroll 1
        for (; it <= g.max_depth; ++it) {
            if (!at_leaf) {
                const uint32_t key = lds_u32(kaddr);
                nd = gld<uint4>(gimg, noff);
                walk_step(nd, key, lanebase, noff, kaddr);
                at_leaf = nd.x == PPE_LEAF_THR;
            }
            if (__builtin_amdgcn_ballot_w64(!at_leaf) == 0) break;
        }
    }
    return nd;
}

// Box check of one rule record (ppe_image.h): a field matches iff (key - lo) mod 2^w <= span.  The ports are
// checked together with packed 16-bit arithmetic.
__device__ __forceinline__ bool rule_box(const uint4 a, const uint4 b, uint32_t sip, uint32_t dip, uint32_t ports,
                                         uint32_t proto) {
    const bool s = sip - a.x <= a.y;
    const bool d = dip - a.z <= a.w;
    const u16x2 kp = __builtin_bit_cast(u16x2, ports), lo = __builtin_bit_cast(u16x2, b.x),
                sp = __builtin_bit_cast(u16x2, b.y);
    const u16x2 dd = kp - lo;
    const bool pp = __builtin_bit_cast(uint32_t, __builtin_elementwise_max(dd, sp)) == b.y;
    const bool pr = proto - (b.z & 0xffu) <= ((b.z >> 8) & 0xffu);
    return s & d & pp & pr;
}

// Residual MAC / time-window fields of a rule whose box matched (rare)
template <class Mac>
__device__ __forceinline__ bool resid_match(uint32_t rs, const uint4 c, const uint4 t, const Mac &mac,
                                         const uint64_t *tsp, uint32_t p, uint64_t now) {
    bool m = true;
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
    return m;
}

// Rule record of `slot` from LDS (staged) or global memory
template <int IMGB>
__device__ __forceinline__ void rule_read(bool in_lds, const uint32_t *gimg, uint32_t off, uint4 &a, uint4 &b) {
    if (in_lds) {
        a = lds_u128(IMGB + off);
        b = lds_u128(IMGB + off + 16u);
    } else {
        a = gld<uint4>(gimg, off);
        b = gld<uint4>(gimg, off + 16u);
    }
}

// First-match ACL lookup: walk to the leaf, then check its candidates in priority order.
// hit = the matching rule's index or -1; action = its action word, or the default action on a miss.
template <int MODE, int IMGB, class Mac>
__device__ __forceinline__ void acl_leaf(const uint32_t *__restrict__ gimg, const AclGeo &g, const uint4 nd,
                                         uint32_t sip, uint32_t dip, uint32_t sport, uint32_t dport, uint32_t proto,
                                         const Mac &mac, const uint64_t *tsp, uint32_t p, uint64_t now,
                                         int32_t &hit, uint32_t &action);

template <int MODE, int IMGB, class Mac>
__device__ __forceinline__ void acl_lookup(const uint32_t *__restrict__ gimg, const AclGeo &g, uint32_t lanebase,
                                           uint32_t sip, uint32_t dip, uint32_t sport, uint32_t dport, uint32_t proto,
                                           const Mac &mac, const uint64_t *tsp, uint32_t p, uint64_t now,
                                           int32_t &hit, uint32_t &action) {
    const uint4 nd = acl_walk<MODE, IMGB>(gimg, g, lanebase);
    acl_leaf<MODE, IMGB>(gimg, g, nd, sip, dip, sport, dport, proto, mac, tsp, p, now, hit, action);
}

// The leaf's candidates in priority order (nd = the leaf node reached by the walk).
template <int MODE, int IMGB, class Mac>
__device__ __forceinline__ void acl_leaf(const uint32_t *__restrict__ gimg, const AclGeo &g, const uint4 nd,
                                         uint32_t sip, uint32_t dip, uint32_t sport, uint32_t dport, uint32_t proto,
                                         const Mac &mac, const uint64_t *tsp, uint32_t p, uint64_t now,
                                         int32_t &hit, uint32_t &action) {
    const uint32_t rules_b = 4u * g.off_rules, resid_b = 4u * g.off_resid;
    const bool rules_lds = MODE == IMG_LDS || (MODE == IMG_SPLIT && g.lds_words >= g.off_resid);
    const bool resid_lds = MODE == IMG_LDS;
    const uint32_t ports = sport | (dport << 16);
    if (g.max_leaf <= 1u) {  // payload = the one candidate's slot (or the always-matching sentinel)
        uint4 ra, rb;
        rule_read<IMGB>(rules_lds, gimg, rules_b + 32u * nd.z, ra, rb);
        bool m = rule_box(ra, rb, sip, dip, ports, proto);
        const uint32_t rs = rb.w >> 29;
        if (m && rs) {
            const uint32_t off = resid_b + 32u * nd.z;
            const uint4 c = resid_lds ? lds_u128(IMGB + off) : gld<uint4>(gimg, off);
            const uint4 t = resid_lds ? lds_u128(IMGB + off + 16u) : gld<uint4>(gimg, off + 16u);
            m = resid_match(rs, c, t, mac, tsp, p, now);
        }
        hit = m ? ((int32_t)(rb.w << 3) >> 3) : -1;  // 29-bit signed rule index (the sentinel's is -1)
        action = m ? rb.z >> 16 : g.default_action;
        return;
    }
    // leaf list: payload = first | count << 24; max_leaf iterations at most (a finished or shorter lane keeps
    // reading a valid entry and ignores it)
    const bool leaf_lds = MODE == IMG_LDS || (MODE == IMG_SPLIT && g.lds_words >= g.off_rules);
    const uint32_t leaf_b = 4u * g.off_leaf;
    uint32_t first = nd.z & 0xffffffu, cnt = nd.z >> 24;
    if (cnt == PPE_LEAF_CNT_ESC) {
        cnt = leaf_lds ? lds_u32(IMGB + leaf_b + 4u * first) : gld<uint32_t>(gimg, leaf_b + 4u * first);
        ++first;
    }
    hit = -1;
    action = g.default_action;
    bool done = false;
#pragma unroll 1
    for (uint32_t j = 0; j < g.max_leaf; ++j) {
        const bool live = !done && j < cnt;
        const uint32_t eo = leaf_b + 4u * (live ? first + j : 0u);  // entry 0 exists whenever max_leaf > 1
        const uint32_t slot = leaf_lds ? lds_u32(IMGB + eo) : gld<uint32_t>(gimg, eo);
        uint4 ra, rb;
        rule_read<IMGB>(rules_lds, gimg, rules_b + 32u * slot, ra, rb);
        bool m = live && rule_box(ra, rb, sip, dip, ports, proto);
        const uint32_t rs = rb.w >> 29;
        if (m && rs) {
            const uint32_t off = resid_b + 32u * slot;
            const uint4 c = resid_lds ? lds_u128(IMGB + off) : gld<uint4>(gimg, off);
            const uint4 t = resid_lds ? lds_u128(IMGB + off + 16u) : gld<uint4>(gimg, off + 16u);
            m = resid_match(rs, c, t, mac, tsp, p, now);
        }
        hit = m ? ((int32_t)(rb.w << 3) >> 3) : hit;
        action = m ? rb.z >> 16 : action;
        done = done || m;
        if (__builtin_amdgcn_ballot_w64(!done && j + 1u < cnt) == 0) break;
    }
}

// Compact leaf (image v6, ppe_image.h): `x` = the leaf exit of the block walk (slot and the candidate's flags).  One
// 16-B record read (LDS when staged) and ~20 VALU: the address prefixes by their marker bits, the ports by packed
// 16-bit spans, the protocol by the exit's TCP / UDP bits (only TCP / UDP packets reach the ACL here).  (Issuing
// every tile's record read before the first check needs 4 more VGPRs per tile: spills at 128)
template <int IMGB>
__device__ __forceinline__ uint4 crec_load(const uint32_t *__restrict__ gimg, const AclGeo &g, uint32_t x) {
    const uint32_t ro = 16u * (x & PPE_CX_SLOT);
    return g.crec_lds != ~0u ? lds_u128(IMGB + g.crec_lds + ro) : gld<uint4>(gimg, 4u * g.off_crec + ro);
}
template <int IMGB>
__device__ __forceinline__ void crec_check(const uint32_t *__restrict__ gimg, const AclGeo &g, uint32_t x,
                                           const uint4 r, uint32_t sip, uint32_t dip, uint32_t sport, uint32_t dport,
                                           bool tcp, int32_t &hit, bool &drop) {
    const uint32_t slot = x & PPE_CX_SLOT;
    // (a /32 compares every bit; else the bits above the marker: ~((lowbit << 1) - 1), 0 for a /0)
    const uint32_t ms = (x & PPE_CX_S32) ? ~0u : ~(((r.x & (0u - r.x)) << 1) - 1u);
    const uint32_t md = (x & PPE_CX_D32) ? ~0u : ~(((r.y & (0u - r.y)) << 1) - 1u);
    const u16x2 kp = __builtin_bit_cast(u16x2, sport | (dport << 16)), lo = __builtin_bit_cast(u16x2, r.z),
                sp = __builtin_bit_cast(u16x2, r.w);
    const bool pp = __builtin_bit_cast(uint32_t, __builtin_elementwise_max(kp - lo, sp)) == r.w;
    const bool m = (((sip ^ r.x) & ms) == 0u) & (((dip ^ r.y) & md) == 0u) & pp &
                   ((x & (tcp ? PPE_CX_TCP : PPE_CX_UDP)) != 0u);
    uint32_t id = slot;
    if (g.off_idtab)  // unused rule entries before this one: the slot's rule index from the table
        id = g.idtab_lds != ~0u ? lds_u32(IMGB + g.idtab_lds + 4u * slot) : gld<uint32_t>(gimg, 4u * g.off_idtab + 4u * slot);
    hit = (m & !(x & PPE_CX_NOHIT)) ? (int32_t)id : -1;
    drop = m ? (x & PPE_CX_DROP) != 0u : g.default_action == ACL_RULE_ACTION_DROP;
}
template <int IMGB>
__device__ __forceinline__ void acl_leaf_compact(const uint32_t *__restrict__ gimg, const AclGeo &g, uint32_t x,
                                                 uint32_t sip, uint32_t dip, uint32_t sport, uint32_t dport,
                                                 bool tcp, int32_t &hit, bool &drop) {
    crec_check<IMGB>(gimg, g, x, crec_load<IMGB>(gimg, g, x), sip, dip, sport, dport, tcp, hit, drop);
}

// Cut-list lookup (image v8, ppe_image.h): the bucket of the key's top sip / dip bits; its group's length slices
// and base (LDS when staged) give the bucket's list; the entries' 4-bit fingerprints (LDS) drop the entries whose
// fixed sip / dip bit below the cut differs from the key's; the rest are independent 16-B reads (LDS, or L2 for large
// sets), two per round, checked in priority order.  The matching entry carries the verdict (its DROP flag); its rule
// id, for the hit output, sits in the same 128-B line (requested right behind the entry, it joins the entry's miss).  Only TCP / UDP keys reach
// it (the classify path).
// one entry against the key's bucket-relative addresses (ks = sip << b0, kd = dip << b1): each prefix matches iff the
// bits above its marker (the lowest set bit above the flag bits: 0-1 in the sip word, 0 in the dip word) equal the
// key's; ports by packed 16-bit spans
__device__ __forceinline__ bool cut_match(const uint4 r, uint32_t ks, uint32_t kd, uint32_t ports, bool tcp) {
    const uint32_t sm = r.x & ~3u, dm = r.y & ~1u;
    const uint32_t ms = ~(((sm & (0u - sm)) << 1) - 1u), md = ~(((dm & (0u - dm)) << 1) - 1u);
    const u16x2 kp = __builtin_bit_cast(u16x2, ports), lo = __builtin_bit_cast(u16x2, r.z),
                sp = __builtin_bit_cast(u16x2, r.w);
    const bool pp = __builtin_bit_cast(uint32_t, __builtin_elementwise_max(kp - lo, sp)) == r.w;
    return (((ks ^ sm) & ms) == 0u) & (((kd ^ dm) & md) == 0u) & pp & (((tcp ? r.x : r.y) & 1u) != 0u);
}
// MODE: IMG_GLOBAL everything from global memory; IMG_SPLIT slices, bases and fingerprints in LDS, entries and ids
// from global (L2); IMG_LDS all of it in LDS
#ifndef PPE_CUT_SPEC
#define PPE_CUT_SPEC 1
#endif
// candidate entries read per round: from L2, 4 (about 1 wave in 3 has a lane with a third candidate after the
// fingerprints, which would cost it a second round trip at 2: C3 ring step -1.5 %, r5p); from LDS, 2 (4: +1 %)
#ifndef PPE_CUT_W_L2
#define PPE_CUT_W_L2 4
#endif
#ifndef PPE_CUT_W_LDS
#define PPE_CUT_W_LDS 2
#endif
template <int MODE, int IMGB>
__device__ __forceinline__ void acl_cut(const uint32_t *__restrict__ gimg, const AclGeo &g, uint32_t sip, uint32_t dip,
                                        uint32_t ports, bool tcp, int32_t &hit, bool &drop) {
    constexpr bool L = MODE != IMG_GLOBAL;
    // IMG_LDS images have the dense layout (the stage plan gives an image with ids in its lines the L2-entry plan):
    // entry e at 16 e, its id at cut_idrel + iw e, no line arithmetic
    constexpr bool DENSE = MODE == IMG_LDS;
    const uint32_t b0 = g.cut & 0xffu, b1 = (g.cut >> 8) & 0xffu;  // (2..14 each)
    const uint32_t bk = ((sip >> (32u - b0)) << b1) | (dip >> (32u - b1));
    const uint32_t gi = bk >> 5, k = bk & 31u;
    const uint4 sl = L ? lds_u128(IMGB + 16u * gi) : gld<uint4>(gimg, 4u * g.cut_slc + 16u * gi);
    const uint32_t base = L ? lds_u32(IMGB + g.cut_gbase_lds + 4u * gi) : gld<uint32_t>(gimg, 4u * g.cut_gbase + 4u * gi);
    const uint32_t m = (1u << k) - 1u;
    const uint32_t cnt = ((sl.x >> k) & 1u) | (((sl.y >> k) & 1u) << 1) | (((sl.z >> k) & 1u) << 2) |
                         (((sl.w >> k) & 1u) << 3);
    const uint32_t first = base + __popc(sl.x & m) + 2u * __popc(sl.y & m) + 4u * __popc(sl.z & m) +
                           8u * __popc(sl.w & m);
    // the list's fingerprints (a window of at least 9 from the aligned dword pair: a longer list's tail is unfiltered)
    const uint32_t fo = 4u * (first >> 3);
    const uint32_t f0 = L ? lds_u32(IMGB + g.cut_fp_lds + fo) : gld<uint32_t>(gimg, 4u * g.cut_fp + fo);
    const uint32_t f1 = L ? lds_u32(IMGB + g.cut_fp_lds + fo + 4u) : gld<uint32_t>(gimg, 4u * g.cut_fp + fo + 4u);
    const uint64_t F = (((uint64_t)f1 << 32) | f0) >> (4u * (first & 7u));
    const uint64_t kn = (uint64_t)(((sip >> (31u - b0)) & 1u) | (((dip >> (31u - b1)) & 1u) << 2)) * 0x1111111111111111ull;
    const uint64_t M = (F ^ kn) & (F >> 1) & 0x5555555555555555ull;  // a fixed bit that differs
    const uint64_t fail = (M | (M >> 2)) & 0x1111111111111111ull;
    uint64_t P = ((1ull << (4u * cnt)) - 1u) & 0x1111111111111111ull & ~fail;  // candidate j at bit 4 j
    const uint32_t ks = sip << b0, kd = dip << b1;
    // entry e: line e / epl (e / epl = umulhi(e, div)), slot e mod epl; byte offset from the entry section
    const uint32_t epl = g.cut_epl;
    auto ebyte = [&](uint32_t e) {
        if constexpr (DENSE) return 16u * e;
        const uint32_t ln = __umulhi(e, g.cut_div);
        return 128u * ln + 16u * (e - ln * epl);
    };
    bool found = false, edrop = false;  // a match; its DROP flag
    uint32_t eb = 0;                    // its byte offset
    const bool i16 = (g.cut & PPE_CUT_IDS16) != 0u;
    const uint32_t iw = i16 ? 2u : 4u;
    // the id's byte offset (after the line's epl entries by slot, or in the id array by entry: dense eb = 16 e)
    auto ibyte = [&](uint32_t b) {
        if constexpr (DENSE) return g.cut_idrel + iw * (b >> 4);
        return (g.cut & PPE_CUT_LINES) ? (b & ~127u) + 16u * epl + iw * ((b & 127u) >> 4) : g.cut_idrel + iw * (b >> 4);
    };
    // entry lines from L2: each candidate's id word is requested right behind its entry, from the same line (the
    // second request joins the first's miss: no L2 request of its own, and no dependent id round after a match)
    const bool spec = PPE_CUT_SPEC && MODE != IMG_LDS && (g.cut & PPE_CUT_LINES) != 0u;
    constexpr int W = MODE == IMG_LDS ? PPE_CUT_W_LDS : PPE_CUT_W_L2;
    uint32_t idw = 0;  // (spec) the match's id word
#pragma unroll 1
    for (uint32_t round = 0; round < 8u; ++round) {
        bool a[W];
        a[0] = !found && P != 0u;
        if (__builtin_amdgcn_ballot_w64(a[0]) == 0) break;
        uint32_t be[W], iv[W];
        uint4 r[W];
#pragma unroll
        for (int c = 0; c < W; ++c) {  // the next W candidates, in priority order
            if (c) a[c] = a[c - 1] && P != 0u;
            const uint32_t j = a[c] ? (uint32_t)__builtin_ctzll(P) >> 2 : 0u;
            P = a[c] ? P & (P - 1u) : P;
            be[c] = ebyte(first + j);
        }
#pragma unroll
        for (int c = 0; c < W; ++c) {
            iv[c] = 0u;
            if constexpr (MODE == IMG_LDS) {
                // every lane reads (an idle one entry `first`, or past it: inside the staged section, ignored), so
                // the reads need no exec-mask branches
                r[c] = lds_u128(IMGB + g.cut_ent_lds + be[c]);
            } else {
                r[c] = make_uint4(0u, 0u, 0u, 0u);
                if (a[c]) {
                    r[c] = gld<uint4>(gimg, 4u * g.cut_ent + be[c]);
                    if (spec) iv[c] = gld<uint32_t>(gimg, 4u * g.cut_ent + (ibyte(be[c]) & ~3u));
                }
            }
        }
#pragma unroll
        for (int c = 0; c < W; ++c) {  // the first match wins (bitwise: no branch per candidate)
            const bool m = a[c] & !found & cut_match(r[c], ks, kd, ports, tcp);
            eb = m ? be[c] : eb;
            idw = m ? iv[c] : idw;
            edrop = m ? (r[c].x & 2u) != 0u : edrop;
            found = found || m;
        }
    }
    drop = found ? edrop : g.default_action == ACL_RULE_ACTION_DROP;
    hit = -1;
    if (found) {  // the rule index
        const uint32_t ib = ibyte(eb);
        if (!spec)
            idw = MODE == IMG_LDS ? lds_u32(IMGB + g.cut_ent_lds + (ib & ~3u)) : gld<uint32_t>(gimg, 4u * g.cut_ent + (ib & ~3u));
        hit = (int32_t)(i16 ? (idw >> (8u * (ib & 2u))) & 0xffffu : idw);
    }
}

// 5-way key select by key slot (multi-tile walks keep the keys in registers)
// Block walks take the packed key {sip, dip, sport | dport << 16, meta} (meta: proto at bits 16-23; the multi-tile
// kernel keeps the status and flags in its low bits), 4 registers per tile instead of 5 + the decode's copies.
__device__ __forceinline__ uint32_t key_sel(uint32_t d, const uint32_t (&k)[4]) {
    return d == 0u ? k[0] : d == 1u ? k[1] : d == 2u ? (k[2] & 0xffffu) : d == 3u ? (k[2] >> 16)
         : d == 4u ? ((k[3] >> 16) & 0xffu) : 0u;
}

// One 2-level block step (ppe_image.h block section): position 0 → b0; position 1 + b0 → b1; exit 2 b0 + b1 (a leaf
// position passes through: threshold ~0)
__device__ __forceinline__ uint32_t block_step(const uint4 lo, const uint4 hi, const uint32_t (&key)[4]) {
    const bool b0 = key_sel(lo.w & 15u, key) > lo.x;
    const uint32_t t1 = b0 ? lo.z : lo.y;
    const uint32_t k1 = (lo.w >> (b0 ? 8u : 4u)) & 15u;
    const bool b1 = key_sel(k1, key) > t1;
    return b0 ? (b1 ? hi.w : hi.z) : (b1 ? hi.y : hi.x);
}
// leaf payload in node form: slot / sentinel, or first | count << 24 for leaf lists (compact images: slot | flags,
// acl_leaf_compact)
__device__ __forceinline__ uint32_t block_leaf_payload(const AclGeo &g, uint32_t x) {
    return g.max_leaf <= 1u ? (x & ~PPE_BLK_LEAF) : ((x & 0x7fffffu) | (((x >> 23) & 0xffu) << 24));
}

// Multi-tile walk over the image's 2-level blocks (PF_MULTI; ppe_image.h block section): the lanes of MT tiles walk
// in lockstep, each step one 32-B block read per lane (LDS for the staged block levels, else L2 / HBM) resolving two
// tree levels, so a deep walk through an L2-resident tree takes half the dependent round trips of a node walk.  Keys
// come from registers; a lane stops reading at its leaf.  Returns, per tile, a node whose .z is the leaf payload in
// the node format acl_leaf reads.
template <int MODE, int IMGB, int MT>
__device__ __forceinline__ void acl_walk_blocks_mt(const uint32_t *__restrict__ gimg, const AclGeo &g,
                                                   const uint32_t (&key)[MT][4], const bool (&need)[MT],
                                                   uint4 (&nd)[MT]) {
    constexpr uint32_t BB = 32u;  // block bytes
    uint32_t blk[MT];
    bool done[MT];
#pragma unroll
    for (int t = 0; t < MT; ++t) {
        blk[t] = 0u;  // single tree: root block 0
        if (g.jump) {  // bucket → root block (the block jump table is staged with the blocks)
            const uint32_t kk = key_sel(g.jump & 0xffu, key[t]);
            const uint32_t jo = 4u * (kk >> ((g.jump >> 8) & 0xffu));
            blk[t] = MODE != IMG_GLOBAL ? lds_u32(IMGB + g.bsec_lds + jo) : gld<uint32_t>(gimg, 4u * g.off_bsec + jo);
        }
        done[t] = !need[t];
        nd[t] = make_uint4(PPE_LEAF_THR, 0u, 0u, 0u);
    }
    if constexpr (MODE == IMG_LDS) {
        // whole image in LDS, branchless: every lane reads a block each step (a finished one its last block again)
        // and the updates are selects, so the wave trades per-tile exec-mask bookkeeping (scalar instructions) for a
        // few VALU selects (C2 / C4 step -2 / -2.6 %, profiles/r3_ab_runs.md r3j)
#pragma unroll 1
        for (uint32_t it = 0; it < g.max_bdepth; ++it) {
            uint4 lo[MT], hi[MT];
#pragma unroll
            for (int t = 0; t < MT; ++t) {
                const uint32_t la = IMGB + g.blk_lds + BB * blk[t];
                lo[t] = lds_u128(la);
                hi[t] = lds_u128(la + 16u);
            }
            bool pending = false;
#pragma unroll
            for (int t = 0; t < MT; ++t) {
                const uint32_t x = block_step(lo[t], hi[t], key[t]);
                const bool leaf = (x & PPE_BLK_LEAF) != 0u, act = !done[t];
                nd[t].z = (act & leaf) ? block_leaf_payload(g, x) : nd[t].z;
                blk[t] = (act & !leaf) ? x : blk[t];
                pending = pending | (act & !leaf);
                done[t] = done[t] | leaf;
            }
            if (__builtin_amdgcn_ballot_w64(pending) == 0) break;
        }
        return;
    }
    if constexpr (MODE == IMG_SPLIT) {
        // Two phases: the staged blocks are the breadth-first prefix of the block forest, so a lane that leaves them
        // never returns.  Phase 1 walks the LDS-resident levels without per-tile branches (a lane outside them, or
        // done, reads block 0 and keeps its state); phase 2 walks the rest from L2 with one exec-masked global read
        // per tile and step (no LDS / global branch pair per step).
#pragma unroll 1
        for (uint32_t it = 0; it < g.max_bdepth; ++it) {
            uint4 lo[MT], hi[MT];
            bool inl[MT];
#pragma unroll
            for (int t = 0; t < MT; ++t) {
                inl[t] = !done[t] & (blk[t] < g.lds_blocks);
                const uint32_t la = IMGB + g.blk_lds + BB * (inl[t] ? blk[t] : 0u);
                lo[t] = lds_u128(la);
                hi[t] = lds_u128(la + 16u);
            }
            bool pending = false;
#pragma unroll
            for (int t = 0; t < MT; ++t) {
                const uint32_t x = block_step(lo[t], hi[t], key[t]);
                const bool leaf = (x & PPE_BLK_LEAF) != 0u;
                nd[t].z = (inl[t] & leaf) ? block_leaf_payload(g, x) : nd[t].z;
                blk[t] = (inl[t] & !leaf) ? x : blk[t];
                done[t] = done[t] | (inl[t] & leaf);
                pending = pending | (inl[t] & !leaf & (x < g.lds_blocks));
            }
            if (__builtin_amdgcn_ballot_w64(pending) == 0) break;
        }
    }
    // the levels read from global memory (L2): one exec-masked read per tile and step
    uint32_t it = 0;
#pragma unroll 1
    for (; it < g.max_bdepth; ++it) {
        bool pending = false;
#pragma unroll
        for (int t = 0; t < MT; ++t) pending = pending | !done[t];
        if (__builtin_amdgcn_ballot_w64(pending) == 0) break;
        if constexpr (MT > 1) {  // (the tail: see below)
            uint32_t tot = 0;
#pragma unroll
            for (int t = 0; t < MT; ++t) tot += (uint32_t)__popcll(__builtin_amdgcn_ballot_w64(!done[t]));
            if (tot <= 64u) break;
        }
        uint4 lo[MT], hi[MT];
#pragma unroll
        for (int t = 0; t < MT; ++t) {
            if (!done[t]) {
                const uint32_t ga = 4u * g.off_blocks + BB * blk[t];
                lo[t] = gld<uint4>(gimg, ga);
                hi[t] = gld<uint4>(gimg, ga + 16u);
            }
        }
#pragma unroll
        for (int t = 0; t < MT; ++t) {
            if (!done[t]) {
                const uint32_t x = block_step(lo[t], hi[t], key[t]);
                if (x & PPE_BLK_LEAF) {
                    done[t] = true;
                    nd[t].z = block_leaf_payload(g, x);
                } else {
                    blk[t] = x;
                }
            }
        }
    }
    if constexpr (MT > 1) {
        // The tail: once the lanes still walking in all MT tiles fit one wave, they move into one virtual tile
        // (ds_permute of the key and block index: lane l of tile t goes to lane P_t + its rank among tile t's
        // walking lanes), which walks the remaining levels with one read per step instead of MT, and hands each lane
        // its leaf back (ds_bpermute).  After the first L2 step about 7 % of C3's lanes walk on.
        if (it >= g.max_bdepth) return;
        uint64_t m[MT];
        uint32_t P[MT + 1];
        P[0] = 0u;
#pragma unroll
        for (int t = 0; t < MT; ++t) {
            m[t] = __builtin_amdgcn_ballot_w64(!done[t]);
            P[t + 1] = P[t] + (uint32_t)__popcll(m[t]);
        }
        const uint32_t tot = P[MT];
        if (tot == 0u) return;
        const uint32_t lane = __lane_id();
        uint32_t vkey[4], vblk = 0u, vpay = 0u, vt = 0u;
#pragma unroll
        for (int t = 1; t < MT; ++t) vt += lane >= P[t] ? 1u : 0u;  // the tile this virtual lane comes from
#pragma unroll
        for (int c = 0; c < 4; ++c) vkey[c] = 0u;
        uint32_t dst[MT];
#pragma unroll
        for (int t = 0; t < MT; ++t) {
            const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(m[t] >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m[t], 0u));
            // a lane that does not walk pushes outside tile t's range [P_t, P_t+1) (its value is not taken there)
            const uint32_t outside = P[t + 1] < 64u ? P[t + 1] : (P[t] > 0u ? P[t] - 1u : 0u);
            dst[t] = !done[t] ? P[t] + rank : outside;
            const uint32_t a4 = dst[t] << 2;
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const uint32_t v = (uint32_t)__builtin_amdgcn_ds_permute((int)a4, (int)key[t][c]);
                vkey[c] = vt == (uint32_t)t ? v : vkey[c];
            }
            const uint32_t vb = (uint32_t)__builtin_amdgcn_ds_permute((int)a4, (int)blk[t]);
            vblk = vt == (uint32_t)t ? vb : vblk;
        }
        bool vdone = lane >= tot;
#pragma unroll 1
        for (; it < g.max_bdepth; ++it) {
            if (__builtin_amdgcn_ballot_w64(!vdone) == 0) break;
            if (!vdone) {
                const uint32_t ga = 4u * g.off_blocks + BB * vblk;
                const uint32_t x = block_step(gld<uint4>(gimg, ga), gld<uint4>(gimg, ga + 16u), vkey);
                if (x & PPE_BLK_LEAF) {
                    vdone = true;
                    vpay = block_leaf_payload(g, x);
                } else {
                    vblk = x;
                }
            }
        }
#pragma unroll
        for (int t = 0; t < MT; ++t) {  // each walking lane takes its leaf back from its virtual lane
            const uint32_t pay = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(dst[t] << 2), (int)vpay);
            if (!done[t]) nd[t].z = pay;
        }
    }
}

// Copy the first `words` of the classifier image into LDS at `lds` with LDS-DMA (global_load_lds_dwordx4): every
// 1-KB piece in flight at once, no VGPR round trip.  Each wave-instruction writes 64 × 16 B at a wave-uniform LDS
// base, so the LDS region is padded to a multiple of 1 KB and the (clamped) tail lanes write into the padding.
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

// action of each terminal status, 2 bits per status: FW for ACL_FW, PUNT for fragments / short windows, the
// configured action for unsupported protocols (Decode_unsupport_proto_handle, decode.c:31-45), else DROP
__device__ __forceinline__ uint64_t make_act_table(uint32_t unsup_fw) {
    uint64_t t = 0;
#pragma unroll
    for (uint32_t st = 0; st < PPE_ST__COUNT; ++st) {
        const uint64_t ac = st == PPE_ST_ACL_FW ? PPE_ACT_FW
                          : (st == PPE_ST_L2_UNSUPPORT || st == PPE_ST_VLAN_UNSUPPORT || st == PPE_ST_IPV4_UNSUPPORT)
                              ? (unsup_fw ? PPE_ACT_FW : PPE_ACT_DROP)
                          : (st == PPE_ST_FRAG || st == PPE_ST_WINDOW_PUNT) ? PPE_ACT_PUNT : PPE_ACT_DROP;
        t |= ac << (2u * st);
    }
    return t;
}

// Wave-ballot compaction of a 64-packet tile's FW / DROP indices into the tile's 64-slot segment of each list (or
// the partition layout when fw_idx == drop_idx, or its compact byte form part8), plus the tile count.  Every lane of
// the wave calls it.
// scr: a wave-private 256-B LDS scratch (byte address) or ~0u.  With scratch, the 4-B partition layout's permuted
// store goes through LDS (each lane writes its slot, then reads slot `lane`), so the global store is in lane order.
__device__ __forceinline__ void compact_tile(uint32_t *fw_idx, uint32_t *drop_idx, uint32_t *tile_cnt, uint32_t n,
                                             uint32_t idx_base, uint32_t tile, uint32_t lane, bool valid, uint32_t act,
                                             uint32_t scr = ~0u, uint8_t *part8 = nullptr) {
    const uint32_t p = (tile << 6) + lane;
    const bool is_fw = valid && act == PPE_ACT_FW;
    const bool is_drop = valid && act == PPE_ACT_DROP;
    const uint64_t bfw = __builtin_amdgcn_ballot_w64(is_fw);
    const uint64_t bdr = __builtin_amdgcn_ballot_w64(is_drop);
    const uint32_t pfw = __builtin_amdgcn_mbcnt_hi((uint32_t)(bfw >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bfw, 0u));
    const uint32_t pdr = __builtin_amdgcn_mbcnt_hi((uint32_t)(bdr >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bdr, 0u));
    const uint32_t so = (tile << 8) + 4u * (is_fw ? pfw : pdr);  // byte offset in the tile's segment
    if (part8) {
        // the partition order, one byte per entry: the packet's offset in its tile and its action
        const uint32_t nv = min(n - (tile << 6), 64u);
        const uint32_t ndr = (uint32_t)__popcll(bdr), nfw = (uint32_t)__popcll(bfw);
        const uint32_t slot = is_fw ? pfw : (is_drop ? nv - ndr + pdr : nfw + lane - pfw - pdr);
        const uint32_t e = lane | (act << 6);
        // (each lane stores its byte at its slot: one 64-B byte-store instruction per tile; the same permutation
        // through LDS stored as 16 dwords measured 16.76 against 16.68 us per 1M, r4h)
        if (valid) gst_nt<uint8_t>(part8, (tile << 6) + slot, (uint8_t)e);
    } else if (fw_idx == drop_idx && fw_idx) {
        // partition layout (one shared list): the tile's segment holds every packet of the tile, FW from the
        // front, DROP at the back, PUNT in between, each in ascending order, the action in bits 31:30 —
        // every slot written by one store instruction (whole-line writes, no tile count needed)
        const uint32_t nv = min(n - (tile << 6), 64u);
        const uint32_t ndr = (uint32_t)__popcll(bdr), nfw = (uint32_t)__popcll(bfw);
        const uint32_t slot = is_fw ? pfw : (is_drop ? nv - ndr + pdr : nfw + lane - pfw - pdr);
        if (scr != ~0u) {  // (LDS ops of one wave complete in order: the read sees every lane's write)
            if (valid) lds_st32(scr + 4u * slot, (p + idx_base) | (act << 30));
            const uint32_t v = lds_u32(scr + 4u * lane);
            if (lane < nv) gst_nt<uint32_t>(fw_idx, (tile << 8) + 4u * lane, v);
        } else if (valid) {
            gst_nt<uint32_t>(fw_idx, (tile << 8) + 4u * slot, (p + idx_base) | (act << 30));
        }
    } else if (fw_idx && drop_idx) {  // both lists: one store instruction
        if (is_fw || is_drop) gst_nt<uint32_t>(is_fw ? fw_idx : drop_idx, so, p + idx_base);
    } else {
        if (fw_idx && is_fw) gst_nt<uint32_t>(fw_idx, so, p + idx_base);
        if (drop_idx && is_drop) gst_nt<uint32_t>(drop_idx, so, p + idx_base);
    }
    if (tile_cnt && lane == 0) {
        const uint32_t nv = min(n - (tile << 6), 64u);
        const uint32_t nfw = (uint32_t)__popcll(bfw), ndr = (uint32_t)__popcll(bdr);
        gst_nt<uint32_t>(tile_cnt, 4u * tile, nfw | (ndr << 8) | ((nv - nfw - ndr) << 16));
    }
}

// ---------------------------------------------------------------------------------------------------------------
// Flow table (dataplane/src/flow/flow.c; layout in ppe_internal.h).  Slot state word: EMPTY, TOMB, LIVE | proto,
// or PEND | packet index (claimed during the current batch, key in rec[index]).

__device__ __forceinline__ uint32_t swap_ports(uint32_t ports) { return (ports >> 16) | (ports << 16); }

// FlowMatch (flow.c:81-94) of two keys {sip, dip, ports}: the same 5-tuple in either direction (protocol compared
// by the caller)
__device__ __forceinline__ bool key_match(uint32_t ax, uint32_t ay, uint32_t az, uint32_t bx, uint32_t by,
                                          uint32_t bz) {
    return (ax == bx && ay == by && az == bz) || (ax == by && ay == bx && az == swap_ports(bz));
}

// FlowFind (flow.c:96-115) over the table as it stood at the start of the batch: the slot of the live flow of
// this 5-tuple, or -1.  One 64-B group (PPE_FLOW_GROUP 16-B keys of the probe array) per probe step;
// stops at the first EMPTY slot.
__device__ __forceinline__ int32_t flow_find(const ppe_flowdev &f, uint32_t fh, uint32_t sip, uint32_t dip,
                                             uint32_t ports, uint32_t proto, uint32_t &fsip, uint32_t &fports) {
    const uint32_t live = PPE_FS_LIVE(proto);
    const uint4 *keys = (const uint4 *)f.keys;  // slot s's key: keys[(PPE_FLOW_SLOT_WORDS / 4) s]
    constexpr uint32_t G = PPE_FLOW_GROUP;
    uint32_t g = fh & f.gmask;
#pragma unroll 1
    for (uint32_t it = 0; it <= f.gmask; ++it) {
        uint4 e[G];
#pragma unroll
        for (uint32_t j = 0; j < G; ++j) e[j] = keys[(PPE_FLOW_SLOT_WORDS / 4u) * (G * g + j)];
#pragma unroll
        for (uint32_t j = 0; j < G; ++j) {
            if (e[j].w == live && key_match(e[j].x, e[j].y, e[j].z, sip, dip, ports)) {
                fsip = e[j].x;
                fports = e[j].z;
                return (int32_t)(G * g + j);
            }
            if (e[j].w == PPE_FS_EMPTY) return -1;
        }
        g = (g + 1u) & f.gmask;
    }
    return -1;
}

// FlowGetPacketDirection (flow.c:248-269) + FlowUpdate (flow.c:163-178) + FLOW_UPDATE_TIMESTAMP: the packet's
// direction flag; per-direction packet / byte counters by one memory-side atomic, last-seen time into the counter record
// (whose line the probe has just read).
__device__ __forceinline__ uint32_t flow_account(const ppe_flowdev &f, uint32_t s, uint32_t fsip, uint32_t fports,
                                                 uint32_t sip, uint32_t ports, uint32_t wire_len, uint64_t now) {
    const uint32_t sport = ports & 0xffffu, dport = ports >> 16, fsport = fports & 0xffffu;
    const bool to_server = sport != dport ? fsport == sport : fsip == sip;
    const uint32_t d = sport == fsport ? 0u : 2u;
    if (!(PPE_ABLATE & 16)) {
        // one memory-side atomic per packet: packets and bytes packed in one word.  The lane whose add takes a field
        // past half its range moves the whole word into the wide counters (exchange with 0, then add), so a field
        // never wraps and concurrent folds never count twice.
        unsigned long long *pk = f.packed + (size_t)PPE_FLOW_REC_WORDS * s + (d >> 1);
        const unsigned long long inc = (1ull << PPE_PK_SHIFT) | (unsigned long long)wire_len;
        const unsigned long long nv =
            __hip_atomic_fetch_add(pk, inc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + inc;
        if ((nv >> PPE_PK_SHIFT) >= f.fold_pkts || (nv & ((1ull << PPE_PK_SHIFT) - 1u)) >= f.fold_bytes) {
            const unsigned long long x = __hip_atomic_exchange(pk, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            unsigned long long *w = f.stats + 4ull * s + d;
            __hip_atomic_fetch_add(w, x >> PPE_PK_SHIFT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_fetch_add(w + 1, x & ((1ull << PPE_PK_SHIFT) - 1u), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    // every packet of the batch carries the same batch time (storing only when it differs measured no faster)
    if (!(PPE_ABLATE & 32)) f.packed[(size_t)PPE_FLOW_REC_WORDS * s + PPE_FLOW_REC_LAST] = now;
    return PPE_F_FLOW | (to_server ? 0u : PPE_F_TOCLIENT);
}

// PPE_UPD_LDS: the classify workgroup collects its bucket entries in LDS as 4-B entries {wire length (16 bits), dir,
// slot within the owner (up to 15 bits)} and writes each bucket out as one 64-B segment at its end, instead of one
// scattered 8-B store per found packet (tables of up to 2^23 slots; larger ones keep the 8-B global entries)
#ifndef PPE_UPD_LDS
#define PPE_UPD_LDS 1
#endif
__device__ __forceinline__ bool upd_small(const ppe_flowdev &f) { return PPE_UPD_LDS && f.upd_osh <= 15u; }

// A found packet (classify launch): its direction flag, and its FlowUpdate as an entry in the bucket of its slot's
// owner in this workgroup's column (flow_update_wg applies it in the next launch, with the last-seen time).
// Without a column (update off, or a workgroup past the allocated columns) or with the bucket full: flow_account.
__device__ __forceinline__ uint32_t flow_found(const ppe_flowdev &f, uint32_t *ucur, uint32_t *ubuf, uint32_t s,
                                               uint32_t fsip, uint32_t fports, uint32_t sip, uint32_t ports,
                                               uint32_t wire_len, uint64_t now) {
    if (blockIdx.x < f.upd_wgs && wire_len < (upd_small(f) ? 0x10000u : 0x80000000u)) {
        const uint32_t sport = ports & 0xffffu, dport = ports >> 16, fsport = fports & 0xffffu;
        const bool to_server = sport != dport ? fsport == sport : fsip == sip;
        const uint32_t d = sport == fsport ? 0u : 1u;
        const uint32_t o = s >> f.upd_osh;
        const uint32_t pos = atomicAdd(&ucur[o], 1u);
        if (pos < PPE_UPD_CAP) {
            if (upd_small(f))
                ubuf[o * PPE_UPD_CAP + pos] = wire_len | (d << 16) | ((s & ((1u << f.upd_osh) - 1u)) << 17);
            else
                f.upd[((size_t)o * f.upd_wgs + blockIdx.x) * PPE_UPD_CAP + pos] =
                    (unsigned long long)s | ((unsigned long long)(wire_len | (d << 31)) << 32);
            return PPE_F_FLOW | (to_server ? 0u : PPE_F_TOCLIENT);
        }
    }
    return flow_account(f, s, fsip, fports, sip, ports, wire_len, now);
}

// the batch's creator counter (classify counts its claims into it; finalize reads it)
__device__ __forceinline__ uint32_t fctl_new(uint32_t parity) {
    return parity ? (uint32_t)PPE_FCTL_BATCH_NEW1 : (uint32_t)PPE_FCTL_BATCH_NEW;
}

__device__ __forceinline__ bool rec_match(const uint4 &q, const uint4 &r) {
    return ((q.w ^ r.w) & 0xffu) == 0u && key_match(q.x, q.y, q.z, r.x, r.y, r.z);
}
// flow_hashfn of a record / key (TCP or UDP only reach the flow table); symmetric, so either orientation
__device__ __forceinline__ uint32_t key_hash(uint32_t sip, uint32_t dip, uint32_t ports, uint32_t proto) {
    return flow_hashfn_l4(proto == 6u, sip, dip, ports & 0xffffu, ports >> 16);
}

// A pending record read or written while other workgroups of the same launch may read it: agent-scope 8-B halves
// (sc1: past this CU's L1, and the store out of the writer's XCD L2), MI355X_MICROARCH.md hand-off row 1 with the
// claim's CAS as the per-record signal
__device__ __forceinline__ void rec_store_shared(uint32_t *rec, uint32_t p, const uint4 &r) {
    unsigned long long *q = (unsigned long long *)(rec + 4ull * p);
    __hip_atomic_store(q, (unsigned long long)r.x | ((unsigned long long)r.y << 32), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(q + 1, (unsigned long long)r.z | ((unsigned long long)r.w << 32), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint4 rec_load_shared(const uint32_t *rec, uint32_t p) {
    unsigned long long *q = (unsigned long long *)(rec + 4ull * p);
    const unsigned long long a = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                             b = __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return make_uint4((uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, (uint32_t)(b >> 32));
}

// The claim of a would-be creator (pending, provisional ACL_FW), made by the classify launch as soon as the packet's
// ACL result is known: the first EMPTY slot on the key's probe path becomes PEND | p (CAS), or the packet joins the
// claim of an equal key met on the way; either way it lowers the slot's creator index (atomicMin).  The caller stored
// the packet's record with rec_store_shared and waited for it (s_waitcnt vmcnt(0)) before the CAS publishes the index.
// Concurrent FlowFind probes of the same launch may see a claimed slot as EMPTY or as PEND: both are "not live".
// Returns the slot, or PPE_FLOW_NONE when the probe path holds no EMPTY slot (table full of live / tombstone slots).
__device__ __forceinline__ uint32_t flow_claim(const ppe_flowdev &f, uint32_t p, const uint4 &r, bool &won) {
    uint32_t g = key_hash(r.x, r.y, r.z, r.w & 0xffu) & f.gmask;
#pragma unroll 1
    for (uint32_t it = 0; it <= f.gmask; ++it) {
#pragma unroll 1
        for (uint32_t j = 0; j < PPE_FLOW_GROUP; ++j) {
            const uint32_t s = PPE_FLOW_GROUP * g + j;
            uint32_t *sw = f.keys + (size_t)PPE_FLOW_SLOT_WORDS * s + 3u;
            uint32_t st = __hip_atomic_load(sw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (st == PPE_FS_EMPTY) {
                uint32_t expect = PPE_FS_EMPTY;
                if (__hip_atomic_compare_exchange_strong(sw, &expect, PPE_FS_PEND | p, __ATOMIC_RELAXED,
                                                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                    atomicMin(&f.creator[s], p);
                    won = true;  // one winning CAS per new flow: the batch's creator count
                    return s;
                }
                st = expect;  // claimed meanwhile (by this flow or another)
            }
            if ((st & PPE_FS_PEND) && rec_match(rec_load_shared(f.rec, st & ~PPE_FS_PEND), r)) {
                atomicMin(&f.creator[s], p);
                return s;
            }
        }
        g = (g + 1u) & f.gmask;
    }
    return PPE_FLOW_NONE;
}

// After the classify launch (every claim made): the slot claimed for a pending packet's flow, or PPE_FLOW_NONE.  The
// finalize launch runs this while its creators turn their PEND slots LIVE (one 16-B store of key and state), so an
// equal LIVE key is this batch's claim too (the packet missed the table as it stood before the batch).
__device__ __forceinline__ uint32_t flow_find_claim(const ppe_flowdev &f, const uint4 &r) {
    const uint4 *keys = (const uint4 *)f.keys;
    const uint32_t live = PPE_FS_LIVE(r.w & 0xffu);
    constexpr uint32_t G = PPE_FLOW_GROUP;
    uint32_t g = key_hash(r.x, r.y, r.z, r.w & 0xffu) & f.gmask;
#pragma unroll 1
    for (uint32_t it = 0; it <= f.gmask; ++it) {
        uint4 e[G];
#pragma unroll
        for (uint32_t j = 0; j < G; ++j) e[j] = keys[(PPE_FLOW_SLOT_WORDS / 4u) * (G * g + j)];
#pragma unroll
        for (uint32_t j = 0; j < G; ++j) {
            if (e[j].w == PPE_FS_EMPTY) return PPE_FLOW_NONE;
            if ((e[j].w & PPE_FS_PEND) ? rec_match(((const uint4 *)f.rec)[e[j].w & ~PPE_FS_PEND], r)
                                       : (e[j].w == live && key_match(e[j].x, e[j].y, e[j].z, r.x, r.y, r.z)))
                return G * g + j;
        }
        g = (g + 1u) & f.gmask;
    }
    return PPE_FLOW_NONE;
}

// PF: how a wave fetches and walks its tiles
#define PF_NONE 0   // one tile per wave, its window loaded at the top of its own iteration
#define PF_HOIST 1  // as PF_NONE, but the first tile's loads are issued before the image staging
#define PF_MULTI 3  // split / global images: each wave loads, decodes and walks PPE_MT tiles together (acl_walk_blocks_mt),
                    // 4 waves/SIMD with 128 VGPRs, one 1024-thread workgroup per CU and its whole LDS for the image
#define PF_CUT 5    // images with cut lists (v7): one tile per wave (8 waves/SIMD), the keys in registers, the bucket
                    // groups in LDS, the list entries and ids in LDS (IMG_LDS) or from L2 (IMG_SPLIT) (acl_cut)
#ifndef PPE_MT
#define PPE_MT 4
#endif
// tiles per wave of the multi-tile kernel over a whole-LDS image (software-pipelined round loop: the next round's
// windows need the registers of two more tiles; C2 / C4 step -4.5 / -3 % at 2 tiles against the plain loop at 4, 3
// tiles -1 %, 4 spills; profiles/r3_ab_runs.md r3h)
#define PPE_MT_LDS 2
#ifndef PPE_FLOW_WAVES  // waves per SIMD the FLOW classify kernel is compiled for
#define PPE_FLOW_WAVES 4   // 8 (the stateless kernels' value) measured 3 % slower per F1 batch: profiles/r3_ab_runs.md r4f
#endif
#ifndef PPE_MT_WAVES  // waves per SIMD the PF_MULTI kernel is compiled for (VGPR budget 512 / this)
#define PPE_MT_WAVES 4
#endif

// FLOW: stateful flow-table mode (ppe_classify_flow, one batch): packets whose flow exists are accounted and
// forwarded here; the rest are recorded (and the would-be creators claim their slots) for the resolve / finalize
// kernels below, which complete their tiles (verdict, compaction, counters).
// PART: every batch of the launch has the throughput layout (verdict, flow hash and ACL hit written, one partition
// list, no tile counts, no tuple: ppe_kargs.part_layout), so the output checks are compile-time and the kernel holds
// fewer scalars (C1 step -2..4 %, C4 -3.5 %: fewer SGPR spills to VGPR lanes)
#ifndef PPE_CUT_LDS_WAVES  // waves per SIMD the cut-list kernel over a whole-LDS image is compiled for (A/B)
#define PPE_CUT_LDS_WAVES PPE_WAVES_PER_EU
#endif
#ifndef PPE_CUT_SPLIT_WAVES  // the same for split images (entries from L2)
#define PPE_CUT_SPLIT_WAVES PPE_WAVES_PER_EU
#endif
template <int MODE, int PF, int BLOCK, bool FLOW, bool PART = false>
__global__ __launch_bounds__(BLOCK, (PF == PF_MULTI && !FLOW) ? PPE_MT_WAVES
                                    : FLOW                                       ? PPE_FLOW_WAVES
                                    : (PF == PF_CUT && MODE == IMG_LDS)          ? PPE_CUT_LDS_WAVES
                                    : (PF == PF_CUT && MODE == IMG_SPLIT)        ? PPE_CUT_SPLIT_WAVES
                                                                                 : PPE_WAVES_PER_EU)
void ppe_classify_kernel(ppe_kargs a) {
    // the multi-tile kernel over a whole-LDS image runs the software-pipelined round loop: the next round's windows
    // are requested before the walk (vmcnt retires loads in issue order; the walk and the record check there issue
    // no global loads, so nothing waits for the prefetch early).  Split images keep the plain round loop: their
    // walk's L2 reads would wait behind the prefetched windows (C3 +3 %).
    constexpr bool MT_PIPE = PF == PF_MULTI && !FLOW && MODE == IMG_LDS;
    constexpr int MT = FLOW ? 1 : PF == PF_MULTI ? (MODE == IMG_LDS ? PPE_MT_LDS : PPE_MT) : 1;
    constexpr bool CUT = PF == PF_CUT && !FLOW;
    constexpr bool KEYS = MT == 1 && !CUT;  // node walks: per-wave key slots in LDS
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    using L = Lds<BLOCK, KEYS, FLOW ? 4u * PPE_UPD_OWNERS * (1u + (PPE_UPD_LDS ? PPE_UPD_CAP : 0u)) : 0u>;
    uint32_t *bins = smem + L::BINS / 4u;    // [PPE_NBINS] packets per (status, flags) bin of this workgroup
    uint32_t *lcnt = bins + PPE_NBINS;       // [32] per-reason counters of this workgroup
    uint32_t *ucur = smem + L::QUEUE / 4u;   // FLOW: [PPE_UPD_OWNERS] entries in this workgroup's owner buckets
    uint32_t *ubuf = ucur + PPE_UPD_OWNERS;  // FLOW, PPE_UPD_LDS: [PPE_UPD_OWNERS][PPE_UPD_CAP] the buckets
    const uint32_t tid = threadIdx.x;
    const uint32_t lane = tid & 63u;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const uint32_t nwaves = gridDim.x * (BLOCK / 64);
    const uint32_t twave = blockIdx.x * (BLOCK / 64) + wv;  // this wave's index in the grid
    // Batch groups: the grid's waves split into G = min(waves, batches, max_groups) equal groups; group g takes
    // batches g, g + G, ..., and its Wb waves stride over each of them (wave wi of the group: tiles wi, wi + Wb, ...).
    // One batch → every wave on it, as before; a queue of batches → each wave walks G times more tiles of a batch
    // before its per-batch setup (descriptor, pointer checks, spilled scalars) comes round again (1M-packet batches
    // over 8,192 waves: 16 tiles per setup at G = 8 instead of 2), while only G batches stream at once.  The
    // remainder waves of the division idle.
    const uint32_t ngroups = max(1u, min(min(nwaves, a.nbatch), a.max_groups));
    const uint32_t stride_waves = nwaves / ngroups;              // Wb
    const uint32_t grp = twave / stride_waves;
    const uint32_t wtile = twave - grp * stride_waves;            // wi
    const bool wave_live = grp < ngroups;
    // the batch being processed (kernel-argument descriptor, or the device descriptor ring: scalar loads either way)
    // (the ring is read through the constant address space: uniform addresses there become scalar loads, so the
    // descriptor lives in SGPRs as the kernel-argument one does)
    static_assert(sizeof(ppe_bdesc) == 96, "descriptor = 6 x 16 B");
    auto bdesc = [&](uint32_t bi) -> ppe_bdesc {
        if (!a.ring) return a.batch[bi];
        typedef const __attribute__((address_space(4))) u32x4 *cq_t;
        const cq_t q = (cq_t)(uintptr_t)(a.ring + bi);
        struct { u32x4 w[6]; } d;
#pragma unroll
        for (int k = 0; k < 6; ++k) d.w[k] = q[k];
        return __builtin_bit_cast(ppe_bdesc, d);
    };
    ppe_bdesc B = bdesc(wave_live ? grp : 0u);
    // current tile's window: bytes 0..51 (w[0..12]) and the wire length.  Clamped (unconditional) loads: a lane past
    // the end of the batch re-reads the last packet.  Byte offsets are 32-bit (the engine keeps n * stride < 2^31).
    uint4 q0, q1, q2;
    uint32_t w12 = 0, qlen = 0;
    auto load_tile = [&](uint32_t t) {
        const uint32_t pc = min((t << 6) + lane, B.n - 1u);
        const uint32_t ro = pc * B.stride;
        q0 = gld<uint4>(B.hdr, ro);
        q1 = gld<uint4>(B.hdr, ro + 16u);
        q2 = gld<uint4>(B.hdr, ro + 32u);
        w12 = gld<uint32_t>(B.hdr, ro + 48u);
        qlen = gld<uint32_t>(B.len, 4u * pc);
    };
    // first window in flight during the image staging
    bool have = (PF == PF_HOIST || CUT) && wave_live && wtile < ((B.n + 63u) >> 6);  // (PF_MULTI: at the loop top)
    if (have) load_tile(wtile);

    for (uint32_t i = tid; i < PPE_NBINS + 32u; i += BLOCK) bins[i] = 0;
    if constexpr (FLOW)
        for (uint32_t i = tid; i < PPE_UPD_OWNERS; i += BLOCK) ucur[i] = 0;
    const uint32_t lanebase = wv * KEY_WAVE_BYTES + 4u * lane;  // this lane's key slot 0 (LDS byte address)
    if (KEYS) lds_st32(lanebase + 256u * PPE_NODE_LEAF, 0u);  // the leaves' zero key
    if (MODE != IMG_GLOBAL) stage_image<BLOCK>(a.img + a.stage_src, smem + L::IMGB / 4u, a.stage_words, tid);
    __syncthreads();
    const AclGeo geo = {a.lds_iters, a.max_depth, a.max_leaf, a.root_ks, a.off_leaf, a.off_rules, a.off_resid,
                        a.lds_words, a.default_action, a.jump, a.off_nodes, a.lds_blocks, a.bsec_lds, a.blk_lds,
                        a.off_bsec, a.off_blocks, a.max_bdepth, a.off_crec, a.off_idtab, a.crec_lds, a.idtab_lds,
                        a.cut, a.cut_slc, a.cut_gbase, a.cut_fp, a.cut_ent, a.cut_epl, a.cut_div, a.cut_idrel,
                        a.cut_gbase_lds, a.cut_fp_lds, a.cut_ent_lds};

    const uint64_t act_table = make_act_table(a.unsup_fw);
    // (this batch's creator counter was zeroed by the previous batch's finalize launch)
    if (FLOW && blockIdx.x == 0 && tid == 0) {
        // the table state after the previous batches, for the host's bounds (zero-copy, no stream stall); LIVE is
        // stable here (the previous batch's finalize has completed, this batch's has not started), so it is also
        // the finalize kernel's overflow reference
        const unsigned long long live0 =
            __hip_atomic_load(&a.flow.ctl[PPE_FCTL_LIVE], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        a.flow.ctl[PPE_FCTL_LIVE_AT_BATCH] = live0;
        a.flow.snap[1] = live0;
        a.flow.snap[2] = __hip_atomic_load(&a.flow.ctl[PPE_FCTL_TOMBS], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __threadfence_system();
        __hip_atomic_store(&a.flow.snap[0], a.flow.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }

    unsigned long long rx_bytes = 0;  // STAT_RECV_PB_ADD (oct-rxtx.c:213) of this lane's packets

    // after the ACL: verdict / hash / hit stores, FLOW pending records, compaction, counters
    auto finish = [&](uint32_t tile, uint32_t p, bool valid, const Dec &k, uint32_t fh, int32_t hit, bool pend) {
        const uint32_t st = k.st;
        const uint32_t act = (uint32_t)(act_table >> (2u * st)) & 3u;
        const uint32_t po = 4u * p;  // byte offset of this packet's SoA output words
        if (valid && !FLOW && (B.flags & PPE_BD_PACKED)) {
            // the packed layout (ppe_result_t.packed): hash | status, action, flags, hit + 1 in one 8-B store
            gst_nt<uint2>(B.verdict, 2u * po,
                          make_uint2(fh, st | (act << 5) | ((k.flags & 63u) << 7) | ((uint32_t)(hit + 1) << 13)));
        } else if (valid) {
            if (PART || B.verdict) gst_nt<uint32_t>(B.verdict, po, st | (act << 8) | (k.flags << 16));
            if (PART || B.fhash) gst_nt<uint32_t>(B.fhash, po, fh);
            if (PART || B.hit) gst_nt<int32_t>(B.hit, po, hit);
            if (!PART && B.tuple) {
                uint4 t;
                t.x = k.sip;
                t.y = k.dip;
                t.z = k.sport | (k.dport << 16);
                // bits 9-15: the window-scale option's offset in the TCP header (DecodeTCPOptions), 0 = none
                const uint32_t ws = k.tcpopt ? tcp_ws_offset(B.hdr + (size_t)p * B.stride, k.tcpopt) : 0u;
                t.w = k.proto | (((k.flags & PPE_F_VLAN) ? 1u : 0u) << 8) | (ws << 9) | (k.paylen << 16);
                gst_nt<uint4>(B.tuple, 4u * po, t);
            }
        }

        if (FLOW) {
            // pending packets: key + provisional status (NO_SYN / ACL_DROP / ACL_FW = would create the flow); a would-be
            // creator claims its flow's slot here (flow_claim), its record stored first for the joiners of its claim
            const uint4 rq = make_uint4(k.sip, k.dip, k.sport | (k.dport << 16), k.proto | (st << 8));
            const bool claim = pend && st == PPE_ST_ACL_FW;
            if (claim) rec_store_shared(a.flow.rec, p, rq);
            else if (pend) gst<uint4>(a.flow.rec, 16u * p, rq);
            if (__builtin_amdgcn_ballot_w64(claim)) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                bool won = false;
                if (claim) a.flow.rslot[p] = flow_claim(a.flow, p, rq, won);
                const uint64_t wb = __builtin_amdgcn_ballot_w64(won);
                if (lane == 0 && wb)
                    __hip_atomic_fetch_add(&a.flow.ctl[fctl_new(a.flow.parity)], (unsigned long long)__popcll(wb),
                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            const uint64_t pm = __builtin_amdgcn_ballot_w64(pend);
            if (lane == 0) {
                a.flow.tile_miss[tile] = pm;
                if (pm) {
                    const unsigned long long i = __hip_atomic_fetch_add(&a.flow.ctl[PPE_FCTL_MISS0 + a.flow.parity],
                                                                        1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    a.flow.miss_tiles[i] = tile;
                }
            }
            if (pm != 0) {  // the finalize kernel completes this tile (compaction, pending lanes' counters)
                if (!(PPE_ABLATE & 2) && valid && !pend) atomicAdd(&bins[st | ((k.flags & 7u) << 5)], 1u);
                return;
            }
        }
        // ---- wave-ballot compaction of FW / DROP indices into this tile's 64-slot segment of each list ----
        if (!(PPE_ABLATE & 4)) {
            const bool p8 = (B.flags & PPE_BD_PART8) != 0u;  // (the compact list travels in the tile_cnt field)
            compact_tile(p8 ? nullptr : B.fw_idx, p8 ? nullptr : (PART ? B.fw_idx : B.drop_idx),
                         (PART || p8) ? nullptr : B.tile_cnt, B.n, B.idx_base, tile, lane, valid, act,
                         KEYS ? lanebase - 4u * lane + 256u * PPE_DIM_SIP : ~0u,
                         p8 ? (uint8_t *)B.tile_cnt : nullptr);
        }

        // ---- per-reason counters: one LDS add per packet into its (status, flags) bin ----
        if (!(PPE_ABLATE & 2) && valid) atomicAdd(&bins[st | ((k.flags & 7u) << 5)], 1u);
    };

    // one tile: decode, hash, ACL, stores, compaction, counters.  w = the window's first 52 bytes, wlen = wire length
    auto process = [&](uint32_t tile, const uint32_t (&w)[13], uint32_t wlen) {
        const uint32_t p = (tile << 6) + lane;
        const bool valid = p < B.n;
        if (!(PPE_ABLATE & 2) && valid) rx_bytes += wlen;
        Dec k = decode<!PART>(w, wlen, B.hdr, p, B.stride, a.syn_check);

        uint32_t fh = 0;
        int32_t hit = -1;
        if (!(PPE_ABLATE & 8) && (k.flags & PPE_F_L4)) fh = flow_hashfn_l4(k.proto == 6u, k.sip, k.dip, k.sport, k.dport);
        bool pend = false;  // FLOW: flow not in the table; resolved by the kernels after this one
        if (FLOW && (k.flags & PPE_F_L4)) {  // FlowGetFlowFromHash, flow.c:181-201
            const uint32_t ports = k.sport | (k.dport << 16);
            uint32_t fsip = 0, fports = 0;
            const int32_t s = flow_find(a.flow, fh, k.sip, k.dip, ports, k.proto, fsip, fports);
            if (s >= 0) {  // found: STAT_ACL_FW without an ACL lookup, then FlowHandlePacket's accounting
                if (valid)
                    k.flags |= flow_found(a.flow, ucur, ubuf, (uint32_t)s, fsip, fports, k.sip, ports, wlen, a.now);
                k.st = PPE_ST_ACL_FW;
            } else {
                pend = valid;
            }
        }
        if ((PPE_ABLATE & 1) && k.st == ST_ACL) {
            k.st = PPE_ST_ACL_FW;
            k.flags |= PPE_F_ACL;
        }
        if (!(PPE_ABLATE & 1) && k.st == ST_ACL && CUT) {
            bool drop;
            acl_cut<MODE, L::IMGB>(a.img, geo, k.sip, k.dip, k.sport | (k.dport << 16), k.proto == 6u, hit, drop);
            k.st = drop ? (uint32_t)PPE_ST_ACL_DROP : (uint32_t)PPE_ST_ACL_FW;  // flow.c:232-243
            k.flags |= PPE_F_ACL;
        }
        if (!(PPE_ABLATE & 1) && k.st == ST_ACL && !CUT) {
            uint32_t rule_act;
            const MacFromWindow mac = {B.hdr, p, B.stride};
            lds_st32(lanebase + 256u * PPE_DIM_SIP, k.sip);
            lds_st32(lanebase + 256u * PPE_DIM_DIP, k.dip);
            lds_st32(lanebase + 256u * PPE_DIM_SPORT, k.sport);
            lds_st32(lanebase + 256u * PPE_DIM_DPORT, k.dport);
            lds_st32(lanebase + 256u * PPE_DIM_PROTO, k.proto);
            acl_lookup<MODE, L::IMGB>(a.img, geo, lanebase, k.sip, k.dip, k.sport, k.dport, k.proto, mac, B.ts, p,
                                      a.now, hit, rule_act);
            const bool drop = rule_act == ACL_RULE_ACTION_DROP;  // flow.c:232-243, FlowHandlePacket :309
            k.st = drop ? (uint32_t)PPE_ST_ACL_DROP : (uint32_t)PPE_ST_ACL_FW;
            k.flags |= PPE_F_ACL;
        }
        finish(tile, p, valid, k, fh, hit, pend);
    };

    // multi-tile rounds: per tile the packed key (sip, dip, ports, meta = status | flags << 8 | proto << 16) and, for
    // the tuple output only, payload length and TCP option word; the flow hash is computed after the walk (fewer live
    // registers while the block reads are in flight)
    auto mt_decode = [&](uint32_t t0, const uint4 (&r0)[MT], const uint4 (&r1)[MT], const uint4 (&r2)[MT],
                         const uint32_t (&r3)[MT], const uint32_t (&rl)[MT], uint32_t (&key)[MT][4],
                         uint32_t (&kpay)[MT], uint32_t (&kopt)[MT], bool (&need)[MT]) {
#pragma unroll
        for (int t = 0; t < MT; ++t) {
            const uint32_t p = ((t0 + t) << 6) + lane;
            if (p < B.n) rx_bytes += rl[t];
            const uint32_t w[13] = {r0[t].x, r0[t].y, r0[t].z, r0[t].w, r1[t].x, r1[t].y, r1[t].z, r1[t].w,
                                    r2[t].x, r2[t].y, r2[t].z, r2[t].w, r3[t]};
            Dec d = decode<!PART>(w, rl[t], B.hdr, p, B.stride, a.syn_check);
            if ((PPE_ABLATE & 1) && d.st == ST_ACL) {
                d.st = PPE_ST_ACL_FW;
                d.flags |= PPE_F_ACL;
            }
            need[t] = d.st == ST_ACL;
            key[t][0] = d.sip;
            key[t][1] = d.dip;
            key[t][2] = d.sport | (d.dport << 16);
            key[t][3] = d.st | (d.flags << 8) | (d.proto << 16);
            kpay[t] = d.paylen;
            kopt[t] = d.tcpopt;
        }
    };
    // a multi-tile round's tile t after the walk: hash, verdict, stores, compaction, counters
    auto mt_finish = [&](uint32_t tile, const uint32_t (&key)[4], uint32_t kpay, uint32_t kopt, bool need, int32_t hit,
                         bool drop) {
        const uint32_t p = (tile << 6) + lane;
        Dec k;
        k.sip = key[0];
        k.dip = key[1];
        k.sport = key[2] & 0xffffu;
        k.dport = key[2] >> 16;
        k.st = key[3] & 0xffu;
        k.flags = (key[3] >> 8) & 0xffu;
        k.proto = key[3] >> 16;
        k.paylen = kpay;
        k.tcpopt = kopt;
        const uint32_t fh = (!(PPE_ABLATE & 8) && (k.flags & PPE_F_L4))
                                ? flow_hashfn_l4(k.proto == 6u, k.sip, k.dip, k.sport, k.dport) : 0u;
        if (need) {
            k.st = drop ? (uint32_t)PPE_ST_ACL_DROP : (uint32_t)PPE_ST_ACL_FW;
            k.flags |= PPE_F_ACL;
        }
        finish(tile, p, p < B.n, k, fh, need ? hit : -1, false);
    };
    // a leaf's rule check (non-compact images: leaf lists / residual fields, rare)
    auto mt_leaf = [&](uint32_t tile, const uint32_t (&key)[4], const uint4 &nd, int32_t &hit, bool &drop) {
        uint32_t rule_act;
        const uint32_t p = (tile << 6) + lane;
        const MacFromWindow mac = {B.hdr, p, B.stride};
        acl_leaf<MODE, L::IMGB>(a.img, geo, nd, key[0], key[1], key[2] & 0xffffu, key[2] >> 16, key[3] >> 16, mac,
                                B.ts, p, a.now, hit, rule_act);
        drop = rule_act == ACL_RULE_ACTION_DROP;
    };

    if constexpr (MT > 1 && MT_PIPE) {
        // PF_MULTI over a whole-LDS image, pipelined: wave w takes rounds of MT tiles [MT w, MT w + MT), then + MT W,
        // ... of its group's batches; round r + 1's windows are requested during round r, before its walk
        uint4 r0[MT], r1[MT], r2[MT];
        uint32_t r3[MT], rl[MT];
        auto load_round = [&](const uint8_t *hdr, const uint32_t *lenp, uint32_t n, uint32_t stride, uint32_t t0) {
#pragma unroll
            for (int t = 0; t < MT; ++t) {
                const uint32_t pc = min(((t0 + t) << 6) + lane, n - 1u);
                const uint32_t ro = pc * stride;
                r0[t] = gld<uint4>(hdr, ro);
                r1[t] = gld<uint4>(hdr, ro + 16u);
                r2[t] = gld<uint4>(hdr, ro + 32u);
                r3[t] = gld<uint32_t>(hdr, ro + 48u);
                rl[t] = gld<uint32_t>(lenp, 4u * pc);
            }
        };
        const uint32_t t_first = wtile * MT, t_step = stride_waves * MT;
        // the first round: the group's first batch with a tile for this wave
        uint32_t bi = grp, t0 = t_first;
        bool live = wave_live;
        while (live && t0 >= ((B.n + 63u) >> 6)) {
            bi += ngroups;
            live = bi < a.nbatch;
            if (live) B = bdesc(bi);
        }
        if (live) load_round(B.hdr, B.len, B.n, B.stride, t0);
        while (live) {
            const uint32_t ntiles = (B.n + 63u) >> 6;
            uint32_t key[MT][4], kpay[MT], kopt[MT];
            bool need[MT];
            mt_decode(t0, r0, r1, r2, r3, rl, key, kpay, kopt, need);
            // the next round (scalar): this batch's next tiles, else the group's next batch with a tile for this wave
            uint32_t nbi = bi, nt0 = t0 + t_step;
            const uint8_t *nh = B.hdr;
            const uint32_t *nl = B.len;
            uint32_t nn = B.n, ns = B.stride;
            bool nlive = true;
            if (nt0 >= ntiles) {
                nt0 = t_first;
                for (;;) {
                    nbi += ngroups;
                    nlive = nbi < a.nbatch;
                    if (!nlive) break;
                    const ppe_bdesc D = bdesc(nbi);
                    if (nt0 < ((D.n + 63u) >> 6)) {
                        nh = D.hdr;
                        nl = D.len;
                        nn = D.n;
                        ns = D.stride;
                        break;
                    }
                }
            }
            if (nlive) load_round(nh, nl, nn, ns, nt0);
            uint4 nd[MT];
            acl_walk_blocks_mt<MODE, L::IMGB, MT>(a.img, geo, key, need, nd);
            int32_t hit[MT];
            bool drop[MT];
#pragma unroll
            for (int t = 0; t < MT; ++t) {
                hit[t] = -1;
                drop[t] = false;
                if (need[t]) {
                    if (geo.off_crec)
                        acl_leaf_compact<L::IMGB>(a.img, geo, nd[t].z, key[t][0], key[t][1], key[t][2] & 0xffffu,
                                                  key[t][2] >> 16, (key[t][3] >> 16) == 6u, hit[t], drop[t]);
                    else
                        mt_leaf(t0 + t, key[t], nd[t], hit[t], drop[t]);
                }
            }
#pragma unroll
            for (int t = 0; t < MT; ++t) {
                if (t0 + t >= ntiles) break;  // wave-uniform
                mt_finish(t0 + t, key[t], kpay[t], kopt[t], need[t], hit[t], drop[t]);
            }
            if (nlive && nbi != bi) B = bdesc(nbi);
            bi = nbi;
            t0 = nt0;
            live = nlive;
        }
    } else if constexpr (MT > 1) {
        // PF_MULTI: wave w takes tiles [MT w, MT w + MT), then + MT W, ...; all MT windows are requested together
        for (uint32_t bi = grp; wave_live && bi < a.nbatch; bi += ngroups) {
            if (bi != grp) B = bdesc(bi);
            const uint32_t ntiles = (B.n + 63u) >> 6;
            for (uint32_t t0 = wtile * MT; t0 < ntiles; t0 += stride_waves * MT) {
                uint4 r0[MT], r1[MT], r2[MT];
                uint32_t r3[MT], rl[MT];
#pragma unroll
                for (int t = 0; t < MT; ++t) {
                    const uint32_t pc = min(((t0 + t) << 6) + lane, B.n - 1u);
                    const uint32_t ro = pc * B.stride;
                    r0[t] = gld<uint4>(B.hdr, ro);
                    r1[t] = gld<uint4>(B.hdr, ro + 16u);
                    r2[t] = gld<uint4>(B.hdr, ro + 32u);
                    r3[t] = gld<uint32_t>(B.hdr, ro + 48u);
                    rl[t] = gld<uint32_t>(B.len, 4u * pc);
                }
                uint32_t key[MT][4], kpay[MT], kopt[MT];
                bool need[MT];
                mt_decode(t0, r0, r1, r2, r3, rl, key, kpay, kopt, need);
                uint4 nd[MT];
                acl_walk_blocks_mt<MODE, L::IMGB, MT>(a.img, geo, key, need, nd);
                // split compact images: tile t + 1's record is requested, by every lane (a lane with no leaf reads
                // slot 0), before tile t's check, so the L2 round trips of the round's records overlap the tiles'
                // finish work instead of one after another (C3 ring step -0.8 %, r4t)
                constexpr bool RPF = MODE == IMG_SPLIT;
                uint4 rnext = make_uint4(0u, 0u, 0u, 0u);
                if (RPF && geo.off_crec) rnext = crec_load<L::IMGB>(a.img, geo, nd[0].z);
#pragma unroll
                for (int t = 0; t < MT; ++t) {
                    const uint32_t tile = t0 + t;
                    if (tile >= ntiles) break;  // wave-uniform
                    uint4 rcur = rnext;
                    if (RPF && geo.off_crec && t + 1 < MT) rnext = crec_load<L::IMGB>(a.img, geo, nd[t + 1].z);
                    int32_t hit = -1;
                    bool drop = false;
                    if (need[t]) {
                        const uint32_t sip = key[t][0], dip = key[t][1], sport = key[t][2] & 0xffffu,
                                       dport = key[t][2] >> 16;
                        const bool tcp = (key[t][3] >> 16) == 6u;
                        if (RPF && geo.off_crec)
                            crec_check<L::IMGB>(a.img, geo, nd[t].z, rcur, sip, dip, sport, dport, tcp, hit, drop);
                        else if (geo.off_crec)
                            acl_leaf_compact<L::IMGB>(a.img, geo, nd[t].z, sip, dip, sport, dport, tcp, hit, drop);
                        else
                            mt_leaf(tile, key[t], nd[t], hit, drop);
                    }
                    mt_finish(tile, key[t], kpay[t], kopt[t], need[t], hit, drop);
                }
            }
        }
    } else
    for (uint32_t bi = grp; wave_live && bi < a.nbatch; bi += ngroups) {
        if (bi != grp) B = bdesc(bi);
        const uint32_t ntiles = (B.n + 63u) >> 6;
        for (uint32_t tile = wtile; tile < ntiles; tile += stride_waves) {
            if (!have) load_tile(tile);
            have = false;
            const uint32_t w[13] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w, q2.x, q2.y, q2.z, q2.w, w12};
            process(tile, w, qlen);
        }
    }

#pragma unroll
    for (int o = 32; o > 0; o >>= 1) rx_bytes += __shfl_xor(rx_bytes, o, 64);
    if (lane == 0 && rx_bytes)
        __hip_atomic_fetch_add(&a.cslots[(size_t)blockIdx.x * PPE_CSLOT_WORDS + PPE_C_RX_BYTES], rx_bytes,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    for (uint32_t b = tid; b < PPE_NBINS; b += BLOCK) {  // expand the bins into counter increments
        const uint32_t c = bins[b];
        if (c) {
            for (uint32_t cb = bin_counters(b, act_table); cb; cb &= cb - 1u) atomicAdd(&lcnt[__builtin_ctz(cb)], c);
        }
    }
    if (FLOW && blockIdx.x < a.flow.upd_wgs) {  // this workgroup's row of bucket counts, for the update kernel
        for (uint32_t o = tid; o < a.flow.upd_owners; o += BLOCK)
            a.flow.ucnt[(size_t)blockIdx.x * a.flow.upd_owners + o] = min(ucur[o], PPE_UPD_CAP);
        if (upd_small(a.flow)) {  // the LDS buckets: 16 lanes write one bucket's 64 B
            uint32_t *ub = (uint32_t *)a.flow.upd;
            for (uint32_t i = tid; i < a.flow.upd_owners * PPE_UPD_CAP; i += BLOCK) {
                const uint32_t o = i / PPE_UPD_CAP, e = i % PPE_UPD_CAP;
                if (e < ucur[o])
                    ub[((size_t)o * a.flow.upd_wgs + blockIdx.x) * PPE_UPD_CAP + e] = ubuf[i];
            }
        }
    }
    __syncthreads();
    // this workgroup's own counter slot: a returnless add (uncontended; the wave does not wait on it)
    if (tid < PPE_C__COUNT && lcnt[tid])
        __hip_atomic_fetch_add(&a.cslots[(size_t)blockIdx.x * PPE_CSLOT_WORDS + tid], (unsigned long long)lcnt[tid],
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // the launch's completion for the host's reader bookkeeping: every wave of this workgroup is past its last image
    // and descriptor read (the barrier above); the workgroup that completes the count publishes the sequence number
    // (a plain system-scope store: the host needs the completion, not any data, so no release fence)
    if (a.done_cnt && tid == 0) {
        const unsigned long long prev = __hip_atomic_fetch_add(a.done_cnt, 1ull, __ATOMIC_RELAXED,
                                                               __HIP_MEMORY_SCOPE_AGENT);
        if (prev + 1ull == a.done_target)
            __hip_atomic_store(a.done_host, a.done_seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// ---------------------------------------------------------------------------------------------------------------
// Flow-table kernels after a FLOW classify launch.  Exact sequential semantics of one core running the batch in
// packet order (flow.c:181-245): among the pending packets of one 5-tuple, the lowest-index packet that passes
// syn_check and the ACL (provisional status ACL_FW) creates the flow; the packets before it keep their own miss
// verdict, the packets after it find the flow.  When the pool runs out, creators beyond the free count (in packet
// order) fail with FLOW_NOMEM, and so do the later would-be creators of their flows.
//   claim     (inside the classify launch, flow_claim) pending would-be creators claim one slot per 5-tuple (CAS
//             EMPTY → PEND | index, or join the claim of an equal key found on the probe path) and lower the slot's
//             creator index (atomicMin); the winning CASes are the batch's creator count;
//   revoke    (finalize's prologue, only when the pool overflows) every workgroup marks its tiles' creators, then
//             workgroup 0 ranks them in packet order and revokes those past the free count, the others waiting on
//             its flag;
//   finalize  per pending packet the flow's claimed slot (the claimer's own, else found, flow_find_claim), final
//             verdicts, flow creation and accounting, the tile's compaction and the pending packets' counters;
//   update    (flow_update_wg, beside finalize in the same launch; owner-computed) the found flows' counters and
//             last-seen times.


struct TileWalk {  // persistent grid: wave gw of W takes the listed tiles gw, gw + W, ... (tiles with pending packets)
    uint32_t lane, gw, W, count;
    template <int BLOCK> __device__ __forceinline__ static TileWalk make(const ppe_flowdev &f, uint32_t nwg) {
        TileWalk t;
        t.lane = threadIdx.x & 63u;
        t.gw = blockIdx.x * (BLOCK / 64) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
        t.W = nwg * (BLOCK / 64);
        t.count = (uint32_t)__hip_atomic_load(&f.ctl[PPE_FCTL_MISS0 + f.parity], __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
        return t;
    }
};

__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// Revoke (finalize's workgroup 0, when the batch's creators overflow the pool): rank the creators in packet order
// (tile masks marked by every finalize workgroup, block scan over the workgroup) and mark the ones past the free
// count revoked.  The creator words go out as sc1 stores and the other workgroups read them with sc1 loads after the
// flag (MI355X_MICROARCH.md hand-off forms; until round 3 this was a one-workgroup launch of its own, until round 4
// a resolve launch marked the creators).
template <int BLOCK>
__device__ __forceinline__ void flow_revoke(const ppe_flow_kargs &a, uint32_t *part, unsigned long long room) {
    const uint32_t tid = threadIdx.x, ntiles = (a.n + 63u) >> 6;
    const uint32_t chunk = (ntiles + BLOCK - 1u) / BLOCK, lo = min(tid * chunk, ntiles), hi = min(lo + chunk, ntiles);
    uint32_t cnt = 0;
    for (uint32_t t = lo; t < hi; ++t)
        if (a.f.tile_miss[t]) cnt += (uint32_t)__popcll(a.f.tile_new[t]);
    part[tid] = cnt;
    __syncthreads();
    for (uint32_t o = 1; o < (uint32_t)BLOCK; o <<= 1) {  // inclusive scan
        const uint32_t v = tid >= o ? part[tid - o] : 0u;
        __syncthreads();
        part[tid] += v;
        __syncthreads();
    }
    unsigned long long rank = part[tid] - cnt;
    for (uint32_t t = lo; t < hi; ++t) {
        uint64_t m = a.f.tile_miss[t] ? a.f.tile_new[t] : 0ull;
        for (; m; m &= m - 1ull, ++rank) {
            if (rank < room) continue;
            const uint32_t p = (t << 6) + (uint32_t)__builtin_ctzll(m);
            __hip_atomic_store(&a.f.creator[a.f.rslot[p]], p | PPE_FLOW_REVOKED, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

// finalize, on the first nwg workgroups of the post-classify launch (ppe_flow_post_kernel)
template <int BLOCK>
__device__ __forceinline__ void flow_finalize_wg(const ppe_flow_kargs &a, uint32_t nwg) {
    __shared__ uint32_t bins[PPE_NBINS];
    __shared__ uint32_t lcnt[32];
    __shared__ uint32_t part[BLOCK];
    __shared__ uint32_t rev_s;
    __shared__ unsigned long long room_s;
    const uint32_t tid = threadIdx.x;
    for (uint32_t i = tid; i < PPE_NBINS; i += BLOCK) bins[i] = 0;
    if (tid < 32u) lcnt[tid] = 0;
    // revoke: when the host's bound says the pool may overflow, every workgroup checks the exact counts; on an
    // overflow every workgroup marks the creators of its miss tiles (tile_new) and arrives on a counter, workgroup 0
    // (dispatched first) waits for all arrivals (the grid, at most two workgroups per CU, is resident), ranks and
    // revokes, then publishes this batch's sequence number, which the others poll for (bounded) before reading any
    // creator word.  The decision and the room come from words no finalize workgroup changes (LIVE_AT_BATCH, written
    // by this batch's classify launch; the creator count, summed by it), so a workgroup dispatched after others have
    // finished and added their creations to LIVE decides exactly as workgroup 0 did.
    if (tid == 0) {
        rev_s = 0u;
        if (a.revoke) {
            const unsigned long long live = __hip_atomic_load(&a.f.ctl[PPE_FCTL_LIVE_AT_BATCH], __ATOMIC_RELAXED,
                                                              __HIP_MEMORY_SCOPE_AGENT),
                                     cr = __hip_atomic_load(&a.f.ctl[fctl_new(a.f.parity)], __ATOMIC_RELAXED,
                                                            __HIP_MEMORY_SCOPE_AGENT);
            rev_s = live + cr > a.f.capacity ? 1u : 0u;
            room_s = a.f.capacity > live ? a.f.capacity - live : 0ull;
        }
        // the next batch's creator counter (last used by the previous batch, whose kernels have all completed)
        if (blockIdx.x == 0) a.f.ctl[fctl_new(a.f.parity ^ 1u)] = 0;
    }
    __syncthreads();
    const bool rev = rev_s != 0u;
    if (rev) {
        {  // mark this workgroup's miss tiles' creators: the claimers (ACL_FW) whose index is their slot's creator
            const TileWalk w = TileWalk::make<BLOCK>(a.f, nwg);
            const uint4 *rec = (const uint4 *)a.f.rec;
            for (uint32_t i = w.gw; i < w.count; i += w.W) {
                const uint32_t t = a.f.miss_tiles[i];
                const uint64_t mask = a.f.tile_miss[t];
                const uint32_t p = (t << 6) + w.lane;
                bool is_new = false;
                if ((mask >> w.lane) & 1ull) {
                    if (((rec[p].w >> 8) & 0xffu) == PPE_ST_ACL_FW) {
                        const uint32_t sl = a.f.rslot[p];
                        is_new = sl != PPE_FLOW_NONE && a.f.creator[sl] == p;
                    }
                }
                const uint64_t bn = __builtin_amdgcn_ballot_w64(is_new);
                if (w.lane == 0) a.f.tile_new[t] = bn;
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (tid == 0) {
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __hip_atomic_fetch_add(&a.f.ctl[PPE_FCTL_ARRIVE], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        if (blockIdx.x == 0) {
            if (tid == 0) {  // every workgroup's marks, then the counter back to 0 for the next overflow batch
                uint32_t k = 0;
                for (; k < (1u << 24) && __hip_atomic_load(&a.f.ctl[PPE_FCTL_ARRIVE], __ATOMIC_RELAXED,
                                                           __HIP_MEMORY_SCOPE_AGENT) < nwg; ++k)
                    __builtin_amdgcn_s_sleep(8);
                if (k == (1u << 24))
                    __hip_atomic_fetch_add(&a.f.ctl[PPE_FCTL_ERR], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __hip_atomic_store(&a.f.ctl[PPE_FCTL_ARRIVE], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            __syncthreads();
            // producer (MI355X_MICROARCH.md, inter-workgroup visibility): every storing wave drains, workgroup
            // barrier, one lane's agent release, then the flag
            flow_revoke<BLOCK>(a, part, room_s);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (tid == 0) {
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __hip_atomic_store(&a.f.ctl[PPE_FCTL_REVOKED_SEQ], a.f.seq + 1ull, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            }
        } else {
            // consumer: one relaxed poll, one agent acquire, its wait, then the workgroup barrier
            if (tid == 0) {
                uint32_t k = 0;
                for (; k < (1u << 24) && __hip_atomic_load(&a.f.ctl[PPE_FCTL_REVOKED_SEQ], __ATOMIC_RELAXED,
                                                           __HIP_MEMORY_SCOPE_AGENT) != a.f.seq + 1ull; ++k)
                    __builtin_amdgcn_s_sleep(8);
                if (k == (1u << 24))  // (never seen; reported by the next synchronising flow call as an error)
                    __hip_atomic_fetch_add(&a.f.ctl[PPE_FCTL_ERR], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            __syncthreads();
        }
    }
    const TileWalk w = TileWalk::make<BLOCK>(a.f, nwg);
    const uint4 *rec = (const uint4 *)a.f.rec;
    const uint64_t act_table = make_act_table(a.unsup_fw);
    uint32_t created = 0, revoked = 0;
    // the next batch's miss-tile counter (last used by the previous batch, whose kernels have all completed)
    if (blockIdx.x == 0 && tid == 0) a.f.ctl[PPE_FCTL_MISS0 + (a.f.parity ^ 1u)] = 0;
    for (uint32_t i = w.gw; i < w.count; i += w.W) {
        const uint32_t t = a.f.miss_tiles[i];
        const uint64_t mask = a.f.tile_miss[t];
        const uint32_t p = (t << 6) + w.lane;
        const bool valid = p < a.n;
        const uint32_t v = valid ? a.verdict[p] : 0u;
        uint32_t act = (v >> 8) & 0xffu;
        bool is_new = false, is_rev = false;
        if ((mask >> w.lane) & 1ull) {
            const uint4 r = rec[p];
            const uint32_t prov = (r.w >> 8) & 0xffu;
            uint32_t st = prov, flags = v >> 16;
            // the flow's claimed slot: the claimer's own (classify launch), else found here (a revoked claim's
            // tombstone reads as "not found", which for a packet that did not claim gives the same verdict)
            const uint32_t s = prov == PPE_ST_ACL_FW ? a.f.rslot[p] : flow_find_claim(a.f, r);
            if (s != PPE_FLOW_NONE) {
                const uint32_t cw = rev ? __hip_atomic_load(&a.f.creator[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                        : a.f.creator[s];
                const bool rev = (cw & PPE_FLOW_REVOKED) != 0u;
                const uint32_t c = cw & ~PPE_FLOW_REVOKED;
                if (p == c) {
                    if (rev) {  // FlowAdd: pool empty (flow.c:124-129); the claimed slot becomes a tombstone
                        st = PPE_ST_FLOW_NOMEM;
                        is_rev = true;
                        a.f.keys[(size_t)PPE_FLOW_SLOT_WORDS * s + 3u] = PPE_FS_TOMB;
                    } else {    // FlowAdd (flow.c:120-158), oriented as this packet, then FlowUpdate
                        st = PPE_ST_ACL_FW;
                        is_new = true;
                        flags |= PPE_F_NEWFLOW | flow_account(a.f, s, r.x, r.z, r.x, r.z, a.len[p], a.now);
                        ((uint4 *)a.f.keys)[(size_t)(PPE_FLOW_SLOT_WORDS / 4u) * s] =
                            make_uint4(r.x, r.y, r.z, PPE_FS_LIVE(r.w & 0xffu));
                    }
                } else if (p > c) {
                    if (rev) {
                        if (prov == PPE_ST_ACL_FW) st = PPE_ST_FLOW_NOMEM;  // FlowAdd fails again, pool still empty
                    } else {  // the flow was created earlier in this batch: found, no ACL lookup (flow.c:197-201)
                        const uint4 rc = rec[c];
                        st = PPE_ST_ACL_FW;
                        flags = (flags & ~PPE_F_ACL) | flow_account(a.f, s, rc.x, rc.z, r.x, r.z, a.len[p], a.now);
                        if (a.hit) a.hit[p] = -1;
                    }
                }
            }
            act = (uint32_t)(act_table >> (2u * st)) & 3u;
            a.verdict[p] = st | (act << 8) | (flags << 16);
            atomicAdd(&bins[st | ((flags & 7u) << 5)], 1u);
        }
        compact_tile(a.fw_idx, a.drop_idx, a.tile_cnt, a.n, 0u, t, w.lane, valid, act, ~0u, a.part8);
        created += (uint32_t)__popcll(__builtin_amdgcn_ballot_w64(is_new));
        revoked += (uint32_t)__popcll(__builtin_amdgcn_ballot_w64(is_rev));
    }
    if (w.lane == 0 && created) {
        __hip_atomic_fetch_add(&a.f.ctl[PPE_FCTL_LIVE], (unsigned long long)created, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_add(&a.f.ctl[PPE_FCTL_NEW_FLOW], (unsigned long long)created, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    }
    if (w.lane == 0 && revoked)
        __hip_atomic_fetch_add(&a.f.ctl[PPE_FCTL_TOMBS], (unsigned long long)revoked, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    for (uint32_t b = tid; b < PPE_NBINS; b += BLOCK) {
        const uint32_t c = bins[b];
        if (c) {
            for (uint32_t cb = bin_counters(b, act_table); cb; cb &= cb - 1u) atomicAdd(&lcnt[__builtin_ctz(cb)], c);
        }
    }
    __syncthreads();
    if (tid < PPE_C__COUNT && lcnt[tid])
        __hip_atomic_fetch_add(&a.cslots[(size_t)blockIdx.x * PPE_CSLOT_WORDS + tid], (unsigned long long)lcnt[tid],
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// FlowUpdate + FLOW_UPDATE_TIMESTAMP of the found packets (flow.c:163-178), owner-computed: workgroup o owns the
// slots [o << upd_osh, (o + 1) << upd_osh), reads its bucket of every classify workgroup's column, sums the entries
// per (slot, direction) in an LDS hash, then updates each touched slot once: plain read-modify-write of the packed
// counters (no other workgroup touches them in this launch; the finalize launch only touches slots claimed in this
// batch, never a found flow's), the fold into the wide counters, the last-seen time.  One update per flow and
// direction instead of one memory-side atomic and one last-seen store per packet.  A slot the full hash cannot take
// is updated by the atomic path directly.
// (owner o's workgroup of the post-classify launch, ppe_flow_post_kernel; usm: its PPE_UPD_HASH * 20 B of LDS)
template <int BLOCK>
__device__ __forceinline__ void flow_update_wg(const ppe_flow_kargs &a, uint32_t o, uint32_t *usm) {
    constexpr uint32_t HC = PPE_UPD_HASH, HB = __builtin_ctz(PPE_UPD_HASH);  // HC = 2^HB
    static_assert(HC == (1u << HB) && HC % BLOCK == 0, "hash geometry");
    // per entry: slot + 1 (0 = empty), then per direction the batch's packets and bytes in the packed counters'
    // format (packets << PPE_PK_SHIFT | bytes): one non-returning LDS add per bucket entry, 20 B per entry.  The
    // fields cannot carry: fewer than 2^24 packets in the batch (else every entry takes the direct path) and wire
    // lengths below 2^16 (longer ones: direct).
    uint32_t *hkey = usm;                                       // [HC]
    unsigned long long *hv = (unsigned long long *)(usm + HC);  // [2][HC]
    const ppe_flowdev &f = a.f;
    const uint32_t tid = threadIdx.x;
    const unsigned long long bmask = (1ull << PPE_PK_SHIFT) - 1u;
    const bool packed_ok = a.n < (1u << (64u - PPE_PK_SHIFT));
    for (uint32_t i = tid; i < HC; i += BLOCK) {
        hkey[i] = 0u;
        hv[i] = hv[HC + i] = 0ull;
    }
    __syncthreads();
    // a slot's update the direct way (the hash is full): flow_account's atomic and fold, the last-seen store
    auto direct = [&](uint32_t s, uint32_t d, uint32_t len) {
        unsigned long long *pk = f.packed + (size_t)PPE_FLOW_REC_WORDS * s + d;
        const unsigned long long inc = (1ull << PPE_PK_SHIFT) | (unsigned long long)len;
        const unsigned long long nv = __hip_atomic_fetch_add(pk, inc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + inc;
        if ((nv >> PPE_PK_SHIFT) >= f.fold_pkts || (nv & bmask) >= f.fold_bytes) {
            const unsigned long long x = __hip_atomic_exchange(pk, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            unsigned long long *wd = f.stats + 4ull * s + 2u * d;
            __hip_atomic_fetch_add(wd, x >> PPE_PK_SHIFT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_fetch_add(wd + 1, x & bmask, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        f.packed[(size_t)PPE_FLOW_REC_WORDS * s + PPE_FLOW_REC_LAST] = a.now;
    };
    const uint32_t ncol = min(f.upd_grid, f.upd_wgs);
    for (uint32_t w = tid; w < ncol; w += BLOCK) {
        const uint32_t n = min(f.ucnt[(size_t)w * f.upd_owners + o], PPE_UPD_CAP);
        // the bucket is one 64-B (4-B entries) or 128-B segment: every entry's load issued before any is used
        const bool sm = upd_small(f);
        const size_t bk = (size_t)o * f.upd_wgs + w;
        const uint4 *e = sm ? (const uint4 *)((const uint32_t *)f.upd + bk * PPE_UPD_CAP)
                            : (const uint4 *)(f.upd + bk * PPE_UPD_CAP);
        // (the segment's loads do not wait for the count: a 4-B-entry bucket is read whole, 64 B, with it)
        uint4 v[PPE_UPD_CAP / 2];
#pragma unroll
        for (uint32_t q = 0; q < PPE_UPD_CAP / 2; ++q)
            v[q] = (sm ? q < PPE_UPD_CAP / 4u : 2u * q < n) ? e[q] : make_uint4(0u, 0u, 0u, 0u);
        // the bucket's entries: slot, direction, wire length (an entry past n: slot ~0, skipped)
        auto entry = [&](uint32_t i, uint32_t &s, uint32_t &d, uint32_t &len) {
            if (sm) {
                const uint4 q = v[i >> 2];
                const uint32_t x = (i & 3u) == 0u ? q.x : (i & 3u) == 1u ? q.y : (i & 3u) == 2u ? q.z : q.w;
                s = (o << f.upd_osh) | (x >> 17);
                d = (x >> 16) & 1u;
                len = x & 0xffffu;
            } else {
                s = (i & 1u) ? v[i >> 1].z : v[i >> 1].x;
                const uint32_t hi = (i & 1u) ? v[i >> 1].w : v[i >> 1].y;
                d = hi >> 31;
                len = hi & 0x7fffffffu;
            }
            if (i >= n) s = ~0u;
        };
        // every entry's claim at its home position issued before any result is used (one LDS round trip for the
        // bucket instead of one per entry: the per-entry probe loop was half the update's time, r5w / r5x); the
        // rare entry whose home holds another slot probes on, one by one.  (Two entries of one slot in one bucket:
        // the lane's CASes execute in order, the second finds the first's key.)
        uint32_t got[PPE_UPD_CAP];
#pragma unroll
        for (uint32_t i = 0; i < PPE_UPD_CAP; ++i) {
            uint32_t s, d, len;
            entry(i, s, d, len);
            got[i] = s != ~0u ? atomicCAS(&hkey[((s * 0x9E3779B1u) >> (32 - HB)) & f.upd_hmask], 0u, s + 1u) : 0u;
        }
#pragma unroll
        for (uint32_t i = 0; i < PPE_UPD_CAP; ++i) {
            uint32_t s, d, len;
            entry(i, s, d, len);
            if (s == ~0u) continue;  // (not break: the loop must unroll, v[] stays in registers)
            uint32_t h = ((s * 0x9E3779B1u) >> (32 - HB)) & f.upd_hmask;
            bool done = got[i] == 0u || got[i] == s + 1u;
            for (uint32_t t = 1; t <= f.upd_hmask && !done; ++t) {
                h = (h + 1u) & f.upd_hmask;
                const uint32_t prev = atomicCAS(&hkey[h], 0u, s + 1u);
                done = prev == 0u || prev == s + 1u;
            }
            if (done && packed_ok && len < 0x10000u)
                atomicAdd(&hv[d * HC + h], (1ull << PPE_PK_SHIFT) | (unsigned long long)len);
            else
                direct(s, d, len);
        }
    }
    __syncthreads();
    // each touched slot once: both directions' packed words in one 16-B read-modify-write, then the last-seen time
    constexpr uint32_t PER = HC / BLOCK;
    uint32_t ks[PER];
    ulonglong2 old[PER];
#pragma unroll
    for (uint32_t j = 0; j < PER; ++j) {
        ks[j] = hkey[tid + j * BLOCK];
        old[j] = ks[j] ? *(const ulonglong2 *)(f.packed + (size_t)PPE_FLOW_REC_WORDS * (ks[j] - 1u))
                       : make_ulonglong2(0ull, 0ull);
    }
#pragma unroll
    for (uint32_t j = 0; j < PER; ++j) {
        if (!ks[j]) continue;
        const uint32_t h = tid + j * BLOCK, s = ks[j] - 1u;
        unsigned long long nw[2] = {old[j].x, old[j].y};
#pragma unroll
        for (uint32_t d = 0; d < 2u; ++d) {
            const unsigned long long v = hv[d * HC + h];
            if (!v) continue;
            const unsigned long long p = (nw[d] >> PPE_PK_SHIFT) + (v >> PPE_PK_SHIFT), b = (nw[d] & bmask) + (v & bmask);
            if (p >= f.fold_pkts || b >= f.fold_bytes) {  // the fold: into the wide counters, the packed word to 0
                unsigned long long *wd = f.stats + 4ull * s + 2u * d;
                wd[0] += p;
                wd[1] += b;
                nw[d] = 0ull;
            } else {
                nw[d] = (p << PPE_PK_SHIFT) | b;
            }
        }
        // the whole 32-B counter record: both directions, the last-seen time
        ulonglong2 *rp = (ulonglong2 *)(f.packed + (size_t)PPE_FLOW_REC_WORDS * s);
        rp[0] = make_ulonglong2(nw[0], nw[1]);
        rp[1] = make_ulonglong2((unsigned long long)a.now, 0ull);
    }
}

// The launch after a flow-mode classify launch: finalize on workgroups [0, fin_wgs) and the owner-computed update on
// the next upd_owners workgroups, side by side (they touch disjoint slots: finalize the ones claimed in this batch,
// the update the found flows'), so the update's memory traffic overlaps finalize's dependent chains.
template <int BLOCK>
__global__ __launch_bounds__(BLOCK) void ppe_flow_post_kernel(ppe_flow_kargs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t usm[];
    if (blockIdx.x < a.fin_wgs) flow_finalize_wg<BLOCK>(a, a.fin_wgs);
    else flow_update_wg<BLOCK>(a, blockIdx.x - a.fin_wgs, usm);
}

// FlowTimeOut + FlowAgeTimeoutCB (flow.c:391-467): live flows idle for more than `timeout` become tombstones.
template <int BLOCK>
__global__ __launch_bounds__(BLOCK) void ppe_flow_age_kernel(ppe_flow_kargs a) {
    uint32_t del = 0;
    for (uint32_t s = blockIdx.x * BLOCK + threadIdx.x; s < a.nslots; s += gridDim.x * BLOCK) {
        uint32_t *rw = a.f.keys + (size_t)PPE_FLOW_SLOT_WORDS * s;
        const uint32_t st = rw[3];
        if ((st & (PPE_FS_PEND | 0xffu)) != PPE_FS_LIVE(0u)) continue;
        const uint64_t l = a.f.packed[(size_t)PPE_FLOW_REC_WORDS * s + PPE_FLOW_REC_LAST];
        if (a.now > l && a.now - l > a.timeout) {
            rw[3] = PPE_FS_TOMB;
            ((uint4 *)a.f.stats)[2ull * s] = make_uint4(0u, 0u, 0u, 0u);
            ((uint4 *)a.f.stats)[2ull * s + 1u] = make_uint4(0u, 0u, 0u, 0u);
            ((uint4 *)a.f.packed)[(size_t)(PPE_FLOW_REC_WORDS / 2u) * s] = make_uint4(0u, 0u, 0u, 0u);
            ((uint4 *)a.f.packed)[(size_t)(PPE_FLOW_REC_WORDS / 2u) * s + 1u] = make_uint4(0u, 0u, 0u, 0u);
            ++del;
        }
    }
    del = wave_sum(del);
    if ((threadIdx.x & 63u) == 0 && del) {
        __hip_atomic_fetch_add(&a.f.ctl[PPE_FCTL_LIVE], 0ull - del, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_add(&a.f.ctl[PPE_FCTL_DEL_FLOW], (unsigned long long)del, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_add(&a.f.ctl[PPE_FCTL_TOMBS], (unsigned long long)del, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    }
}

// Rehash: every live flow of a.f into the empty table a.dst (tombstones dropped).  Inserters only look at slot
// states (keys are distinct), so the state is claimed first and the rest of the slot written after.
template <int BLOCK>
__global__ __launch_bounds__(BLOCK) void ppe_flow_rehash_kernel(ppe_flow_kargs a) {
    for (uint32_t s = blockIdx.x * BLOCK + threadIdx.x; s < a.nslots; s += gridDim.x * BLOCK) {
        const uint4 k = ((const uint4 *)a.f.keys)[(size_t)(PPE_FLOW_SLOT_WORDS / 4u) * s];
        if ((k.w & (PPE_FS_PEND | 0xffu)) != PPE_FS_LIVE(0u)) continue;
        uint32_t g = key_hash(k.x, k.y, k.z, (k.w >> 8) & 0xffu) & a.dst.gmask;
        bool done = false;
#pragma unroll 1
        for (uint32_t it = 0; it <= a.dst.gmask && !done; ++it) {
#pragma unroll 1
            for (uint32_t j = 0; j < PPE_FLOW_GROUP && !done; ++j) {
                const uint32_t d = PPE_FLOW_GROUP * g + j;
                uint32_t *dw = a.dst.keys + (size_t)PPE_FLOW_SLOT_WORDS * d;
                uint32_t expect = PPE_FS_EMPTY;
                if (__hip_atomic_compare_exchange_strong(dw + 3u, &expect, k.w, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                         __HIP_MEMORY_SCOPE_AGENT)) {
                    dw[0] = k.x;
                    dw[1] = k.y;
                    dw[2] = k.z;
                    ((uint4 *)a.dst.stats)[2ull * d] = ((const uint4 *)a.f.stats)[2ull * s];
                    ((uint4 *)a.dst.stats)[2ull * d + 1u] = ((const uint4 *)a.f.stats)[2ull * s + 1u];
                    ((uint4 *)a.dst.packed)[(size_t)(PPE_FLOW_REC_WORDS / 2u) * d] =
                        ((const uint4 *)a.f.packed)[(size_t)(PPE_FLOW_REC_WORDS / 2u) * s];
                    ((uint4 *)a.dst.packed)[(size_t)(PPE_FLOW_REC_WORDS / 2u) * d + 1u] =
                        ((const uint4 *)a.f.packed)[(size_t)(PPE_FLOW_REC_WORDS / 2u) * s + 1u];
                    done = true;
                }
            }
            g = (g + 1u) & a.dst.gmask;
        }
    }
}

// ---------------------------------------------------------------------------------------------------------------
// Flow-hash steering across GPUs (with the flow table, packets go to the GPU owning their flow,
// as Octeon's PIP tag steering sends a flow to one core, dataplane/src/platform/oct-init.c:139-151).
// owner(p) = flow_hash % world for packets that reach the flow table, the local rank for the rest; perm lists the
// packets grouped by owner, ascending within an owner (a stable partition), so each owner sees every source's
// packets in their original order.

__device__ __forceinline__ uint32_t steer_owner(const ppe_steer_kargs &a, uint32_t p) {
    const uint32_t v = a.verdict[p];
    return ((v >> 16) & PPE_F_L4) ? a.flow_hash[p] % a.world : a.rank;
}

// one wave per 64-packet tile: owner counts of the tile (and, SCATTER, each packet's slot in perm)
template <bool SCATTER>
__global__ __launch_bounds__(256) void ppe_steer_tile_kernel(ppe_steer_kargs a) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t gw = blockIdx.x * 4u + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), W = gridDim.x * 4u;
    const uint32_t ntiles = (a.n + 63u) >> 6;
    for (uint32_t t = gw; t < ntiles; t += W) {
        const uint32_t p = (t << 6) + lane;
        const bool valid = p < a.n;
        const uint32_t own = valid ? steer_owner(a, p) : 0xffffffffu;
        uint32_t cnt = 0, rank_in = 0;
        for (uint32_t o = 0; o < a.world; ++o) {
            const uint64_t m = __builtin_amdgcn_ballot_w64(own == o);
            if (lane == o) cnt = (uint32_t)__popcll(m);
            if (own == o)
                rank_in = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
        }
        if (!SCATTER) {
            if (lane < a.world) a.tcount[(size_t)t * a.world + lane] = cnt;
        } else if (valid) {
            a.perm[a.tcount[(size_t)t * a.world + own] + rank_in] = p;
        }
    }
}

// one workgroup: tcount[t][o] ← the offset in perm of tile t's first packet owned by o (owner-major, tile order)
#define STEER_SCAN_T 512u
__global__ __launch_bounds__(STEER_SCAN_T) void ppe_steer_scan_kernel(ppe_steer_kargs a) {
    __shared__ uint32_t part[PPE_STEER_MAX_WORLD][STEER_SCAN_T];
    __shared__ uint32_t base[PPE_STEER_MAX_WORLD];
    const uint32_t tid = threadIdx.x, W = a.world, ntiles = (a.n + 63u) >> 6;
    const uint32_t chunk = (ntiles + STEER_SCAN_T - 1u) / STEER_SCAN_T, lo = min(tid * chunk, ntiles),
                   hi = min(lo + chunk, ntiles);
    for (uint32_t o = 0; o < W; ++o) {
        uint32_t sum = 0;
        for (uint32_t t = lo; t < hi; ++t) sum += a.tcount[(size_t)t * W + o];
        part[o][tid] = sum;
    }
    __syncthreads();
    for (uint32_t off = 1; off < STEER_SCAN_T; off <<= 1) {  // inclusive scans, one per owner
        uint32_t v[PPE_STEER_MAX_WORLD];
        for (uint32_t o = 0; o < W; ++o) v[o] = tid >= off ? part[o][tid - off] : 0u;
        __syncthreads();
        for (uint32_t o = 0; o < W; ++o) part[o][tid] += v[o];
        __syncthreads();
    }
    if (tid == 0) {
        uint32_t b = 0;
        for (uint32_t o = 0; o < W; ++o) {
            base[o] = b;
            a.counts[o] = part[o][STEER_SCAN_T - 1u];
            b += part[o][STEER_SCAN_T - 1u];
        }
    }
    __syncthreads();
    for (uint32_t o = 0; o < W; ++o) {
        uint32_t run = base[o] + (tid ? part[o][tid - 1] : 0u);
        for (uint32_t t = lo; t < hi; ++t) {
            const uint32_t c = a.tcount[(size_t)t * W + o];
            a.tcount[(size_t)t * W + o] = run;
            run += c;
        }
    }
}

// fixed-size rows through a permutation, 4 B per lane-step
__global__ __launch_bounds__(256) void ppe_rows_kernel(ppe_rows_kargs a) {
    const uint32_t words = a.row_bytes >> 2;
    const uint64_t total = (uint64_t)a.n * words;
    for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i < total; i += (uint64_t)gridDim.x * 256u) {
        const uint32_t r = (uint32_t)(i / words), w = (uint32_t)(i % words);
        const uint32_t q = a.perm[r];
        const uint64_t from = a.scatter ? r : q, to = a.scatter ? q : r;
        ((uint32_t *)a.dst)[to * words + w] = ((const uint32_t *)a.src)[from * words + w];
    }
}

// ACL-only lookup over pre-decoded tuples (the DP_Acl_Lookup(mbuf) entry, dataplane/src/flow/flow.c:232):
// tuple = {sip, dip, sport | dport << 16, proto}, macs = {dmac lo, dmac hi, smac lo, smac hi} (optional).
template <int MODE>
__global__ __launch_bounds__(PPE_BLOCK) void ppe_acl_tuple_kernel(ppe_tuple_kargs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    using L = Lds<PPE_BLOCK>;
    const uint32_t tid = threadIdx.x;
    const uint32_t lanebase = (tid >> 6) * KEY_WAVE_BYTES + 4u * (tid & 63u);
    lds_st32(lanebase + 256u * PPE_NODE_LEAF, 0u);
    if (MODE == IMG_LDS) stage_image<PPE_BLOCK>(a.img, smem + L::IMGB / 4u, a.img_words, tid);
    __syncthreads();
    const uint32_t depth = a.img[PPE_IMG_W_MAXDEPTH];
    const AclGeo geo = {0u, depth, a.img[PPE_IMG_W_MAXLEAF], a.img[PPE_IMG_W_ROOTKS], a.img[PPE_IMG_W_OFFLEAF],
                        a.img[PPE_IMG_W_OFFRULES], a.img[PPE_IMG_W_OFFRESID], MODE == IMG_LDS ? a.img_words : 0u,
                        a.default_action, a.img[PPE_IMG_W_JUMP], a.img[PPE_IMG_W_OFFNODES], 0u, 0u, 0u, 0u, 0u,
                        0u, 0u, 0u, ~0u, ~0u};
    for (uint32_t i = blockIdx.x * PPE_BLOCK + tid; i < a.n; i += gridDim.x * PPE_BLOCK) {
        const uint4 t = ((const uint4 *)a.tuple)[i];
        uint4 m = make_uint4(0, 0, 0, 0);
        if (a.macs) m = ((const uint4 *)a.macs)[i];
        int32_t hit;
        uint32_t act;
        const MacValues mac = {m.x, m.y, m.z, m.w};
        const uint32_t sport = t.z & 0xffffu, dport = t.z >> 16, proto = t.w & 0xffu;
        lds_st32(lanebase + 256u * PPE_DIM_SIP, t.x);
        lds_st32(lanebase + 256u * PPE_DIM_DIP, t.y);
        lds_st32(lanebase + 256u * PPE_DIM_SPORT, sport);
        lds_st32(lanebase + 256u * PPE_DIM_DPORT, dport);
        lds_st32(lanebase + 256u * PPE_DIM_PROTO, proto);
        acl_lookup<MODE, L::IMGB>(a.img, geo, lanebase, t.x, t.y, sport, dport, proto, mac, a.ts, i, a.now, hit, act);
        if (a.hit) a.hit[i] = hit;
        if (a.action) a.action[i] = act;
    }
}

}  // namespace

#ifdef PPE_TU_HOIST
// csrc/ppe_kernels_hoist.hip: this file again, built with LLVM's iterative-ILP machine scheduler, exporting only the
// stateless hoisted-fetch kernels over an LDS-resident image (C1's variant: kernel −2 %, r6s; the cut-list and split
// variants are slower under it and stay in the default build, profiles/r6_ab_runs.md r6j / r6s)
template <int B>
static int launch_hoist_b(const ppe_kargs *a, uint32_t grid, size_t shmem, hipStream_t s, hipEvent_t e0,
                          hipEvent_t e1) {
    if (a->part_layout)
        hipExtLaunchKernelGGL((ppe_classify_kernel<IMG_LDS, PF_HOIST, B, false, true>), dim3(grid), dim3(B), shmem, s,
                              e0, e1, 0, *a);
    else
        hipExtLaunchKernelGGL((ppe_classify_kernel<IMG_LDS, PF_HOIST, B, false>), dim3(grid), dim3(B), shmem, s, e0,
                              e1, 0, *a);
    return (int)hipGetLastError();
}
extern "C" int ppe_launch_classify_hoist_lds(const ppe_kargs *a, uint32_t grid, size_t shmem, int block, void *stream,
                                             void *ev_start, void *ev_stop) {
    const hipStream_t s = (hipStream_t)stream;
    const hipEvent_t e0 = (hipEvent_t)ev_start, e1 = (hipEvent_t)ev_stop;
    if (block == 1024) return launch_hoist_b<1024>(a, grid, shmem, s, e0, e1);
    if (block == 512) return launch_hoist_b<512>(a, grid, shmem, s, e0, e1);
    return launch_hoist_b<256>(a, grid, shmem, s, e0, e1);
}
template <int B>
static int occ_hoist_b(size_t shmem) {
    int nb = 0;
    const hipError_t e =
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, ppe_classify_kernel<IMG_LDS, PF_HOIST, B, false>, B, shmem);
    return e == hipSuccess ? nb : -1;
}
extern "C" int ppe_occupancy_hoist_lds(size_t shmem, int block) {
    if (block == 1024) return occ_hoist_b<1024>(shmem);
    if (block == 512) return occ_hoist_b<512>(shmem);
    return occ_hoist_b<256>(shmem);
}
#else
extern "C" int ppe_launch_classify_hoist_lds(const ppe_kargs *a, uint32_t grid, size_t shmem, int block, void *stream,
                                             void *ev_start, void *ev_stop);
extern "C" int ppe_occupancy_hoist_lds(size_t shmem, int block);

template <int M, int P, int B>
static int launch_t(const ppe_kargs *a, uint32_t grid, size_t shmem, hipStream_t s, hipEvent_t e0, hipEvent_t e1,
                    int flow) {
    // hipExtLaunchKernelGGL's events are the dispatch packet's own start/end timestamps (what rocprofv3 reports),
    // unlike hipEventRecord markers around the launch
    if (flow) {  // the flow-table variant is built for the default tile fetch only
        hipExtLaunchKernelGGL((ppe_classify_kernel<M, PF_HOIST, B, true>), dim3(grid), dim3(B), shmem, s, e0, e1, 0,
                              *a);
    } else if constexpr (M == IMG_LDS && P == PF_HOIST) {  // (the iterative-ILP build, ppe_kernels_hoist.hip)
        return ppe_launch_classify_hoist_lds(a, grid, shmem, B, (void *)s, (void *)e0, (void *)e1);
    } else if constexpr (P != PF_NONE) {
        if (a->part_layout)
            hipExtLaunchKernelGGL((ppe_classify_kernel<M, P, B, false, true>), dim3(grid), dim3(B), shmem, s, e0, e1, 0,
                                  *a);
        else
            hipExtLaunchKernelGGL((ppe_classify_kernel<M, P, B, false>), dim3(grid), dim3(B), shmem, s, e0, e1, 0, *a);
    } else {
        hipExtLaunchKernelGGL((ppe_classify_kernel<M, P, B, false>), dim3(grid), dim3(B), shmem, s, e0, e1, 0, *a);
    }
    return (int)hipGetLastError();
}

template <int M, int P, int B>
static int occ_t(size_t shmem, bool flow = false) {
    int nb = 0;
    hipError_t e;
    if (flow) {
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, ppe_classify_kernel<M, PF_HOIST, B, true>, B, shmem);
    } else if constexpr (M == IMG_LDS && P == PF_HOIST) {  // (the iterative-ILP build, ppe_kernels_hoist.hip)
        return ppe_occupancy_hoist_lds(shmem, B);
    } else {
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, ppe_classify_kernel<M, P, B, false>, B, shmem);
    }
    return e == hipSuccess ? nb : -1;
}

static size_t classify_shmem(uint32_t lds_words, int mode, int pipe, int block, bool flow = false) {
    // key slots (node walks) + counter bins (+ flow-table launches: the owner-update bucket cursors)
    const size_t base = ppe_classify_fixed_lds(block, pipe, mode) + (flow ? ppe_flow_lds_extra() : 0u);
    if (mode == IMG_GLOBAL) return base;
    return base + (((size_t)lds_words * 4u + 1023u) & ~(size_t)1023u);
}

#define PPE_DISPATCH_B(FN, M, P, ...)                                \
    do {                                                             \
        if (block == 1024) return FN<M, P, 1024>(__VA_ARGS__);       \
        if (block == 512) return FN<M, P, 512>(__VA_ARGS__);         \
        return FN<M, P, 256>(__VA_ARGS__);                           \
    } while (0)
#define PPE_DISPATCH_P(FN, M, ...)                                   \
    do {                                                             \
        if (pipe == PF_NONE) PPE_DISPATCH_B(FN, M, PF_NONE, __VA_ARGS__); \
        if (pipe == PF_MULTI) PPE_DISPATCH_B(FN, M, PF_MULTI, __VA_ARGS__); \
        if (pipe == PF_CUT) PPE_DISPATCH_B(FN, M, PF_CUT, __VA_ARGS__); \
        PPE_DISPATCH_B(FN, M, PF_HOIST, __VA_ARGS__);                \
    } while (0)
#define PPE_DISPATCH(FN, ...)                                        \
    do {                                                             \
        if (mode == IMG_LDS) PPE_DISPATCH_P(FN, IMG_LDS, __VA_ARGS__);     \
        if (mode == IMG_SPLIT) PPE_DISPATCH_P(FN, IMG_SPLIT, __VA_ARGS__); \
        PPE_DISPATCH_P(FN, IMG_GLOBAL, __VA_ARGS__);                 \
    } while (0)

extern "C" int ppe_launch_classify(const ppe_kargs *a, uint32_t grid, int mode, int pipe, int block, int flow,
                                   void *stream, void *ev_start, void *ev_stop) {
    const size_t shmem = classify_shmem(a->stage_words, mode, pipe, block, flow != 0);
    hipStream_t s = (hipStream_t)stream;
    hipEvent_t e0 = (hipEvent_t)ev_start, e1 = (hipEvent_t)ev_stop;
    PPE_DISPATCH(launch_t, a, grid, shmem, s, e0, e1, flow);
}

extern "C" int ppe_launch_flow(int kind, const ppe_flow_kargs *a, uint32_t grid, void *stream) {
    const hipStream_t s = (hipStream_t)stream;
    const dim3 g(grid), b(PPE_FLOW_BLOCK);
    switch (kind) {
        case PPE_FLOW_K_POST:
            hipLaunchKernelGGL(ppe_flow_post_kernel<PPE_FLOW_POST_BLOCK>, g, dim3(PPE_FLOW_POST_BLOCK),
                               a->f.upd_wgs ? PPE_UPD_HASH * 20u : 0u, s, *a);
            break;
        case PPE_FLOW_K_AGE: hipLaunchKernelGGL(ppe_flow_age_kernel<PPE_FLOW_BLOCK>, g, b, 0, s, *a); break;
        case PPE_FLOW_K_REHASH: hipLaunchKernelGGL(ppe_flow_rehash_kernel<PPE_FLOW_BLOCK>, g, b, 0, s, *a); break;
        default: return (int)hipErrorInvalidValue;
    }
    return (int)hipGetLastError();
}

// resident workgroups per CU for the kernel variant (the persistent grid is sized to exactly fill the chip)
extern "C" int ppe_classify_occupancy(uint32_t lds_words, int mode, int pipe, int block) {
    const size_t shmem = classify_shmem(lds_words, mode, pipe, block);
    PPE_DISPATCH(occ_t, shmem);
}
// the same for the flow-table variant (its own waves per SIMD and LDS)
extern "C" int ppe_classify_occupancy_flow(uint32_t lds_words, int mode, int block) {
    const int pipe = PF_HOIST;
    const size_t shmem = classify_shmem(lds_words, mode, pipe, block, true);
    PPE_DISPATCH(occ_t, shmem, true);
}

// classify LDS of a flow-table launch beyond the stateless kernel's: the owner-update bucket cursors (and buckets)
extern "C" uint32_t ppe_flow_lds_extra() {
    return 4u * PPE_UPD_OWNERS + (PPE_UPD_LDS ? 4u * PPE_UPD_OWNERS * PPE_UPD_CAP : 0u);
}
// waves per SIMD the flow-table classify kernel is compiled for (its LDS share per workgroup)
extern "C" uint32_t ppe_flow_waves() { return PPE_FLOW_WAVES; }

// LDS of a workgroup besides the staged image: the per-wave key slots of node walks and the counter bins.  Block
// and cut-list walks keep the keys in registers.
extern "C" uint32_t ppe_classify_fixed_lds(int block, int pipe, int mode) {
    const bool regkeys = pipe == PF_MULTI || pipe == PF_CUT;
    return (regkeys ? 0u : (uint32_t)(block / 64) * KEY_WAVE_BYTES) + PPE_LDS_FIXED;
}

extern "C" int ppe_launch_steer(int phase, const ppe_steer_kargs *a, uint32_t grid, void *stream) {
    const hipStream_t s = (hipStream_t)stream;
    if (phase == 0) hipLaunchKernelGGL(ppe_steer_tile_kernel<false>, dim3(grid), dim3(256), 0, s, *a);
    else if (phase == 1) hipLaunchKernelGGL(ppe_steer_scan_kernel, dim3(1), dim3(STEER_SCAN_T), 0, s, *a);
    else hipLaunchKernelGGL(ppe_steer_tile_kernel<true>, dim3(grid), dim3(256), 0, s, *a);
    return (int)hipGetLastError();
}

extern "C" int ppe_launch_rows(const ppe_rows_kargs *a, uint32_t grid, void *stream) {
    hipLaunchKernelGGL(ppe_rows_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, *a);
    return (int)hipGetLastError();
}

extern "C" int ppe_launch_acl_tuples(const ppe_tuple_kargs *a, uint32_t grid, int lds_img, void *stream) {
    const size_t keys = (size_t)ppe_classify_fixed_lds(PPE_BLOCK, PF_NONE, IMG_GLOBAL);  // node walk: key slots
    if (lds_img) {
        const size_t shmem = keys + (((size_t)a->img_words * 4u + 1023u) & ~(size_t)1023u);
        hipLaunchKernelGGL(ppe_acl_tuple_kernel<IMG_LDS>, dim3(grid), dim3(PPE_BLOCK), shmem, (hipStream_t)stream, *a);
    } else {
        hipLaunchKernelGGL(ppe_acl_tuple_kernel<IMG_GLOBAL>, dim3(grid), dim3(PPE_BLOCK), keys, (hipStream_t)stream, *a);
    }
    return (int)hipGetLastError();
}
#endif  // PPE_TU_HOIST
