/*
 * ppe_defrag.hip — IPv4 reassembly on the GPU (ppe_defrag_* in include/ppe_hip.h).
 *
 * The reference's Defrag (dataplane/src/decode/decode-defrag.c:449-487) is sequential per fragment: find or create
 * the FCB of (sip, dip, ip_id), then run Frag_defrag_begin / Frag_defrag_process on it.  Different FCBs never
 * interact except through the FCB cap (fcb_create, :71-97), so one batch runs as:
 *
 *   parse      one lane per fragment: re-derive the fields DecodeIPV4 stored in the mbuf (decode-ipv4.c:216-222) and
 *              look the key up in the device FCB hash table (open addressing, linear probing);
 *   claim      (the parse launch) fragments whose FCB does not exist claim a slot (CAS, key = the claiming fragment's
 *              parsed key) and record the lowest claiming index: that fragment is the one whose fcb_create runs;
 *   admit      creators in index order (ballot counts, a look-back over the workgroups in one launch) get FCB
 *              records while running + rank < fcb_max (fcb_create's fetch-and-add cap); the others fail, and with
 *              them every later fragment of their key in this batch, because the running count cannot fall inside
 *              a batch;
 *   group      one launch: each fragment's group key is its FCB's first fragment index in the batch; every other
 *              fragment of the FCB takes one of the group's 15 slots by an atomic ticket (past them, an overflow
 *              list).  (Until round 4: a stable 2-pass LSD radix sort of the fragments by that key, 4 launches.)
 *   process    one lane per FCB (the group's first fragment) sorts its group's slots into arrival order in registers
 *              and runs the reference state machine over the fragments in that order (chain ≤ cache_max entries,
 *              kept as a nibble list of store slots);
 *   place      completing fragments in index order get datagram indices (ballot counts, summed per workgroup)
 *              and write their datagram's assembly plan;
 *   stash      one wave per held fragment copies its frame into the FCB's store slot (PACKET_HW2SW, mbuf.c:117-156);
 *   assemble   (the stash's launch) one wave per datagram concatenates the chain (Frag_defrag_reasm,
 *              decode-defrag.c:222-289) from the plan the place kernel wrote for it, patches ip_len / ip_off / the
 *              header checksum, and writes a classify-ready window + length.
 *
 * Aging (Frag_defrag_timeout, decode-defrag.c:490-551) is one workgroup: free completed / idle FCBs, then rebuild
 * the hash table from the live records (which also clears the tombstones left by failed claims).
 *
 * Integer / byte work only: the rare path of the classifier (fragments are PUNTed), sized by the fragment count.
 */
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>

#include "ppe_hip.h"

namespace {

constexpr uint32_t kEmpty = 0u, kTomb = 1u, kLive = 2u, kPend = 0x80000000u;
constexpr uint32_t kNone = 0xffffffffu;
constexpr uint32_t kBlock = 256;        // workgroup size of the per-fragment kernels
#ifndef DF_SLOT_WAVES
#define DF_SLOT_WAVES 4
#endif
constexpr uint32_t kSlotBlock = 64 * DF_SLOT_WAVES;   // workgroup size of the wave-per-item kernels (stash, assemble)
constexpr uint32_t kScanT = 1024;       // one-workgroup scans

// FCB record header word 0
constexpr uint32_t kRecLive = 1u << 0;
constexpr uint32_t kRecDelete = 1u << 1;    // DEFRAG_DELETE (decode-defrag.h:21)
constexpr uint32_t kRecComplete = 1u << 2;  // DEFRAG_COMPLETE: the chain moved to the datagram
constexpr uint32_t kFirstIn = 1u, kLastIn = 2u;  // DEFRAG_FIRST_IN / DEFRAG_LAST_IN (decode-defrag.h:18-19)
// header words: 0 flags | last_in << 8 | cache_num << 16 | nlist << 24; 1 total_fraglen; 2 meat; 3 pad;
//               4,5 chain order (4-bit store slots, position 0 in the low nibble); 6,7 pad
constexpr uint32_t kRecWords = 8;

// control words (u64)
enum { C_RUNNING = 0, C_NEW, C_DEL, C_FREE_TOP, C_DGRAMS, C_TEARDROP, C_TIMEOUT_DROP, C_NDGRAM, C_ST0 = 8,
       C_CREATORS = C_ST0 + PPE_DF__COUNT + 2, C_AGE_DROPPED, C_AGE_FREED, C_SCRATCH, C_LOOK_ERR,
       C_FAILN, C_FAIL0, C_WORDS = C_FAIL0 + 4 + 3 };
// C_FAILN / C_FAIL0..: this call's admission workgroups whose look-back failed (count, then the first kMaxFail ids):
// the group kernel returns the free-stack records their creators' ranks skipped
constexpr uint32_t kMaxFail = 4;
static_assert(C_FAIL0 + kMaxFail <= C_WORDS, "control words");

// parsed fragment record words (frec): sip, dip, id | proto << 16 | mf << 24, off | flen << 16, totlen,
// l2 | ihl4 << 8, hash, valid
constexpr uint32_t kFrecWords = 8;

struct DfArgs {
    // batch
    const uint8_t *pkt;
    const uint64_t *off;
    const uint32_t *len;
    const uint64_t *id;
    uint32_t n;
    uint32_t hdr_stride;
    uint64_t now;
    uint64_t timeout;
    // outputs
    uint32_t *status;
    uint32_t *dgram_of;
    uint8_t *dgram_hdr;
    uint32_t *dgram_len;
    uint8_t *dgram_pkt;
    uint64_t *dgram_frags;
    uint32_t *n_dgram;
    // table
    uint32_t *tstate, *tkey, *creator;
    uint32_t smask;
    // records
    uint32_t *rhdr, *rdesc;
    unsigned long long *rts, *rid;
    uint8_t *store;
    uint32_t *freestk;
    unsigned long long *ctl;
    uint32_t fcb_max, cache_max, frag_buf, reasm_buf, sstride;
    // batch scratch
    uint32_t *frec, *fslot, *inserted, *dgrec, *tcnt;
    uint32_t *plan;                      // assembly plan: min(max_batch, fcb_max) × cache_max entries of 8 words
    // grouping (df_group_kernel): each fragment's group key; per group key, its members besides the key fragment
    // (count, kGroupSlots slots in claim order; a group with more members is enumerated from gkey); the per-tile
    // counts of completing fragments (process → place)
    uint32_t *gkey, *gcnt, *gslot, *dcnt;
    unsigned long long *look;            // admission: per-workgroup look-back words (epoch << 32 | flags | count)
    uint32_t epoch, nlook;               // this call's tag (never 0) and the look-back array's length
    uint32_t look_spins;                 // admission: polls of an unpublished predecessor before giving up
    uint32_t look_fail_wg;               // test hook (PPE_DF_LOOK_FAIL): this workgroup's look-back fails at once, in
                                         // the handle's first ppe_defrag call
    unsigned long long *err_host;        // pinned, device-mapped: set by a failed look-back (ppe_defrag reports it)
    uint64_t *dropped;                   // age: ids of dropped fragments
    uint32_t max_dropped;
    uint32_t max_batch;
};

__device__ __forceinline__ uint32_t ld_be16(const uint8_t *p) { return ((uint32_t)p[0] << 8) | p[1]; }

__device__ __forceinline__ uint32_t key_hash(uint32_t sip, uint32_t dip, uint32_t id) {
    // bucket choice only (the reference's jhash_3words bucket, decode-defrag.c:108-112, orders nothing observable)
    uint32_t h = sip * 0x9e3779b1u ^ (dip + 0x7f4a7c15u) * 0x85ebca77u ^ (id + 0x165667b1u) * 0xc2b2ae3du;
    h ^= h >> 15;
    h *= 0x2c1b3c6du;
    h ^= h >> 12;
    return h;
}

__device__ __forceinline__ uint64_t lanemask_lt() {
    const uint32_t lane = __lane_id();
    return lane ? (~0ull >> (64u - lane)) : 0ull;
}


// ---- parse + find ------------------------------------------------------------------------------------------------
// The fields DecodeIPV4 hands to Defrag (decode-ipv4.c:216-222): sip/dip (BE32 @12/16), defrag_id (BE16 @4),
// frag_offset = (ip_off & 0x1fff) << 3, frag_len = L3 length − ihl*4 where the L3 length is what is left of
// (uint16_t)pkt_totallen after the L2 header (Decode, decode.c:25; DecodeEthernet / DecodeVLAN len − 14 / − 4).
// A frame that would not reach Defrag (any earlier drop, not a fragment, OSPF, frag_len 0) is PPE_DF_NOT_FRAG.
__global__ void __launch_bounds__(kBlock) df_parse_kernel(DfArgs a) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= a.n) return;
    const uint8_t *p = a.pkt + a.off[i];
    const uint32_t tot = a.len[i];
    const uint32_t L = tot & 0xffffu;
    uint32_t valid = 0, l2 = 14, ihl4 = 0, sip = 0, dip = 0, idp = 0, offf = 0, dummy = 0;
    // the frame's first 40 bytes (Ethernet, a VLAN tag, the IPv4 header's first 20 bytes) as 10 frame-aligned dwords:
    // 11 aligned loads, all in flight together (not one byte load per field, which the lane's branches would spread
    // over several round trips), each clamped to the frame's last dword (no read past the frame); issued before the
    // length test, so the frame offset and length loads go out together too (an empty frame reads its length word)
    const uintptr_t pa = (uintptr_t)p;
    const uint32_t sh = (uint32_t)(pa & 3u) * 8u;
    const uint32_t *ap = L ? (const uint32_t *)(pa & ~(uintptr_t)3) : a.len + i;
    const uint32_t lastw = L ? ((uint32_t)(pa & 3u) + L - 1u) >> 2 : 0u;
    uint32_t raw[11];
#pragma unroll
    for (uint32_t k = 0; k < 11; ++k) raw[k] = ap[k < lastw ? k : lastw];
    // (kept ahead of the branch: the compiler would otherwise sink the loads, and the offset load with them, into it)
#pragma unroll
    for (uint32_t k = 0; k < 11; ++k) asm volatile("" ::"v"(raw[k]));
    if (L >= 14) {
        uint32_t fw[10];
#pragma unroll
        for (uint32_t k = 0; k < 10; ++k) fw[k] = sh ? (raw[k] >> sh) | (raw[k + 1] << (32u - sh)) : raw[k];
        auto byte = [&](uint32_t b) -> uint32_t { return (fw[b >> 2] >> (8u * (b & 3u))) & 0xffu; };
        auto be16 = [&](uint32_t b) -> uint32_t { return (byte(b) << 8) | byte(b + 1); };
        auto be32 = [&](uint32_t b) -> uint32_t { return (be16(b) << 16) | be16(b + 2); };
        const bool mac0 = fw[0] == 0 && (fw[1] & 0xffffu) == 0;   // bytes 0-5
        const bool mac1 = (fw[1] >> 16) == 0 && fw[2] == 0;       // bytes 6-11
        const uint32_t et = be16(12);
        bool ok = !mac0 && !mac1;
        const bool tag = et == 0x8100u || et == 0x9100u;
        if (ok && tag) {
            ok = L >= 18 && be16(16) == 0x0800u;   // a second tag or another inner type never reaches IPv4
            l2 = 18;
        } else {
            ok = ok && et == 0x0800u;
        }
        if (ok && L >= l2 + 20) {
            // the IPv4 header's fields at l2 = 14 or 18, both read at compile-time byte positions, then selected
            const uint32_t b0 = tag ? byte(18) : byte(14);
            const uint32_t l3 = L - l2;
            ihl4 = (b0 & 0x0fu) * 4u;
            const uint32_t iplen = tag ? be16(20) : be16(16);
            const uint32_t offw = tag ? be16(24) : be16(20);
            const uint32_t proto = tag ? byte(27) : byte(23);
            const bool is_frag = (offw & 0x1fffu) != 0 || (offw & 0x2000u) != 0;
            if ((b0 >> 4) == 4u && ihl4 >= 20 && iplen >= ihl4 && l3 >= iplen && is_frag && proto != 89u &&
                l3 - ihl4 != 0) {
                valid = 1;
                sip = tag ? be32(30) : be32(26);
                dip = tag ? be32(34) : be32(30);
                idp = (tag ? be16(22) : be16(18)) | (proto << 16) | (((offw >> 13) & 1u) << 24);
                offf = ((offw & 0x1fffu) << 3) | (((l3 - ihl4) & 0xffffu) << 16);
            }
        }
    }
    (void)dummy;
    uint32_t *fr = a.frec + (size_t)i * kFrecWords;
    const uint32_t h = key_hash(sip, dip, idp & 0xffffu);
    uint32_t slot = kNone;
    if (valid) {
        // FragFind (decode-defrag.c:124-146): ip4_frag_match compares id, sip, dip (not the protocol).  Claims of this
        // launch make slots PEND only (never LIVE), so a plain probe of the table as it stood before the batch finds
        // exactly what the reference's FragFind finds; a stale EMPTY only sends the fragment to the claim, which
        // re-reads every slot by CAS.
        uint32_t s = h & a.smask;
        for (uint32_t probe = 0; probe <= a.smask; ++probe, s = (s + 1) & a.smask) {
            // the slot's state and key read together (one round trip per probe, not two)
            const uint32_t st = a.tstate[s];
            const uint4 k = *(const uint4 *)(a.tkey + (size_t)s * 4);
            asm volatile("" ::"v"(k.x), "v"(k.y), "v"(k.z));   // (not sunk into the LIVE branch)
            if (st == kEmpty) break;
            if (st == kLive) {
                if (k.x == sip && k.y == dip && k.z == (idp & 0xffffu)) {
                    slot = s;
                    break;
                }
            }
        }
    }
    const bool claim = valid && slot == kNone;
    if (claim) {
        // the key words other lanes of this launch compare when they meet this fragment's PEND claim: written through
        // to memory (agent scope) and waited for before the CAS that publishes the index
        unsigned long long *q = (unsigned long long *)fr;
        __hip_atomic_store(q, (unsigned long long)sip | ((unsigned long long)dip << 32), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(q + 1, (unsigned long long)idp | ((unsigned long long)offf << 32), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    } else {
        *(uint4 *)fr = make_uint4(sip, dip, idp, offf);
    }
    *(uint4 *)(fr + 4) = make_uint4(tot, l2 | (ihl4 << 8), h, valid);
    if (!claim) {
        // found in the table: the FCB's first fragment in this batch is its group key
        if (valid) atomicMin(a.creator + slot, i);
        a.fslot[i] = valid ? slot : (kNone - 1);   // kNone − 1: not a fragment
        return;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // claim: a slot per new key, lowest claiming index recorded.  Terminates: slots >= 2 (fcb_max + max_batch) >
    // live + pending, and EMPTY / TOMB slots are claimable.  The first CAS of each slot expects EMPTY (the common
    // case) and doubles as its load: a failed CAS returns the slot's state.
    const uint32_t id = idp & 0xffffu;
    uint32_t s = h & a.smask;
    for (;;) {
        uint32_t st = kEmpty;
        for (;;) {
            if (st == kEmpty || st == kTomb) {
                const uint32_t old = atomicCAS(a.tstate + s, st, kPend | i);
                if (old == st) {
                    atomicMin(a.creator + s, i);
                    a.fslot[i] = s;
                    return;
                }
                st = old;   // re-examine this slot
                continue;
            }
            if (st & kPend) {
                // join an equal key's claim: its key words, read past this XCD's L2
                const unsigned long long *q = (const unsigned long long *)(a.frec + (size_t)(st & ~kPend) * kFrecWords);
                const unsigned long long k01 = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                                         k23 = __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if ((uint32_t)k01 == sip && (uint32_t)(k01 >> 32) == dip && ((uint32_t)k23 & 0xffffu) == id) {
                    atomicMin(a.creator + s, i);
                    a.fslot[i] = s;
                    return;
                }
            }
            break;
        }
        s = (s + 1) & a.smask;
    }
}

// ---- per-tile ballot counts of a flag, one-workgroup scan, ranked placement ------------------------------------------
// a creator: the fragment whose claim (or join) recorded the lowest index on its still-pending slot
__device__ __forceinline__ bool df_creator(const DfArgs &a, uint32_t i) {
    if (i >= a.n) return false;
    const uint32_t s = a.fslot[i];
    if (s >= kNone - 1) return false;
    return (a.tstate[s] & kPend) && a.creator[s] == i;
}

// This workgroup's exclusive prefix of the tile counts: the sum of cnt[0, t0), and (total != nullptr) the sum of
// cnt[0, tiles).  Every workgroup reads the whole (small: n / 64 words) count array from L2 itself, so the ranked
// kernels need no separate scan launch.
template <int T>
__device__ uint32_t wg_tile_prefix(const uint32_t *cnt, uint32_t t0, uint32_t tiles, uint32_t *total) {
    __shared__ uint32_t wsum[2][T / 64];
    uint32_t before = 0, all = 0;
    for (uint32_t k = threadIdx.x; k < tiles; k += T) {
        const uint32_t v = cnt[k];
        all += v;
        before += k < t0 ? v : 0u;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        before += __shfl_xor(before, o, 64);
        all += __shfl_xor(all, o, 64);
    }
    if (__lane_id() == 0) {
        wsum[0][threadIdx.x >> 6] = before;
        wsum[1][threadIdx.x >> 6] = all;
    }
    __syncthreads();
    uint32_t b = 0, t = 0;
#pragma unroll
    for (uint32_t w = 0; w < T / 64; ++w) {
        b += wsum[0][w];
        t += wsum[1][w];
    }
    if (total) *total = t;
    return b;
}

// The creators' ranks come from a look-back over the workgroups in index order (one launch: the workgroups are
// dispatched in index order and all resident, so every wait is on an earlier, running one).  Workgroup b publishes
// its count as an aggregate, adds its predecessors' words back to the first inclusive one, then publishes its
// inclusive prefix.  Words carry the call's epoch, so the array needs no clearing between calls.  The per-tile counts
// are kept for the sort's first pass (the running-count update).  The running count and free-stack top are read as
// they stood before this batch: that histogram pass, which runs next, moves them past this batch's admissions.
__global__ void __launch_bounds__(kBlock) df_admit_kernel(DfArgs a) {
    __shared__ uint32_t wc[kBlock / 64], wbase;
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    const uint32_t w = threadIdx.x >> 6;
    const bool f = df_creator(a, i);
    const uint64_t b = __builtin_amdgcn_ballot_w64(f);
    if (__lane_id() == 0) {
        wc[w] = (uint32_t)__popcll(b);
        if (i < a.n) a.tcnt[i >> 6] = (uint32_t)__popcll(b);
    }
    __syncthreads();
    if (w == 0) {
        // wave 0 looks back 64 predecessors per round (one load each, all in flight together): the nearest inclusive
        // word ends the walk; a window with an unpublished word before it is read again
        constexpr unsigned long long kAgg = 1ull << 30, kIncl = 1ull << 31, kCount = kAgg - 1;
        const unsigned long long tag = (unsigned long long)a.epoch << 32;
        const uint32_t lane = __lane_id();
        uint32_t agg = 0;
        for (uint32_t k = 0; k < kBlock / 64; ++k) agg += wc[k];
        if (lane == 0)
            __hip_atomic_store(a.look + blockIdx.x, tag | kAgg | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        uint32_t excl = 0, spins = 0;
        bool failed = false;
        for (int end = (int)blockIdx.x; end > 0;) {
            if (blockIdx.x == a.look_fail_wg) {
                failed = true;
                break;
            }
            const int p = end - 1 - (int)lane;   // lane 0: the nearest predecessor
            const unsigned long long v =
                p >= 0 ? __hip_atomic_load(a.look + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : tag | kIncl;
            const bool ready = (v >> 32) == a.epoch;
            const uint64_t incl = __builtin_amdgcn_ballot_w64(ready && (v & kIncl));
            const uint64_t wait = __builtin_amdgcn_ballot_w64(!ready);
            const uint32_t fi = incl ? (uint32_t)__builtin_ctzll(incl) : 64u;   // the nearest inclusive lane
            const uint64_t upto = fi < 63 ? (2ull << fi) - 1ull : ~0ull;          // lanes [0, fi]
            if (wait & upto) {   // a predecessor before it has not published yet
                // bounded: a word that never arrives (a broken dispatch-order assumption) is reported, not waited
                // for forever
                if (++spins > a.look_spins) {
                    failed = true;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
                continue;
            }
            uint32_t c = lane <= fi ? (uint32_t)(v & kCount) : 0u;
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
            excl += c;
            if (incl) break;
            end -= 64;
        }
        if (lane == 0) {
            // a failed look-back publishes no inclusive prefix (its aggregate stands, so the workgroups after it
            // still sum the right prefix through it) and admits none of its creators (their FCBs are not created:
            // no two creators can take one record); the failure reaches the caller: the next ppe_defrag call and
            // ppe_defrag_info return PPE_EIO
            if (failed) {
                atomicAdd(a.ctl + C_LOOK_ERR, 1ull);
                const unsigned long long q = atomicAdd(a.ctl + C_FAILN, 1ull);
                if (q < kMaxFail) a.ctl[C_FAIL0 + q] = blockIdx.x;
                __hip_atomic_store(a.err_host, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            } else {
                __hip_atomic_store(a.look + blockIdx.x, tag | kIncl | (excl + agg), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            }
            wbase = failed ? ~0u : excl;
        }
    }
    __syncthreads();
    uint32_t base = wbase;
    const bool failed = base == ~0u;
    for (uint32_t k = 0; k < w; ++k) base += wc[k];   // the workgroup's earlier waves
    if (!f) return;
    const uint32_t rank = base + (uint32_t)__popcll(b & lanemask_lt());
    const uint32_t s = a.fslot[i];
    // fcb_create (decode-defrag.c:74-81): fetch-and-add, fail when the previous count reached DEFRAG_FCB_MAX
    if (!failed && a.ctl[C_RUNNING] + rank < a.fcb_max) {
        const uint32_t r = a.freestk[a.ctl[C_FREE_TOP] - 1 - rank];
        const uint32_t *fr = a.frec + (size_t)i * kFrecWords;
        uint32_t *k = a.tkey + (size_t)s * 4;
        k[0] = fr[0];
        k[1] = fr[1];
        k[2] = fr[2] & 0xffffu;
        k[3] = r;
        uint32_t *h = a.rhdr + (size_t)r * kRecWords;
        h[0] = kRecLive;   // memset(fcb, 0) + key (decode-defrag.c:91-95)
        h[1] = h[2] = h[4] = h[5] = 0;
        h[3] = fr[2] & 0xffffu;   // key copy for the table rebuild: id, sip, dip
        h[6] = fr[0];
        h[7] = fr[1];
        a.rts[r] = a.now;
        a.tstate[s] = kLive;
    } else {
        a.tkey[(size_t)s * 4 + 3] = kNone;
        a.tstate[s] = kTomb;
    }
}

// ---- grouping: each FCB's fragments of this batch, under the key of its first one ------------------------------------
__device__ __forceinline__ uint32_t df_group_key(const DfArgs &a, uint32_t i) {
    const uint32_t s = a.fslot[i];
    // fragments without a record (not a fragment, or its FCB could not be created) form singleton groups keyed by
    // their own index, which no FCB group uses (a group's key is the index of one of its own fragments)
    if (s >= kNone - 1 || a.tstate[s] != kLive) return i;
    return a.creator[s];   // the FCB's first fragment in this batch
}
#ifndef DF_PROC_WIN
#define DF_PROC_WIN 16   // the process kernel's register window: the group's head + its slots
#endif
constexpr uint32_t kGroupSlots = DF_PROC_WIN - 1;  // members besides the key fragment held in a group's slots
constexpr uint32_t kGroupStride = DF_PROC_WIN;     // words per group in gslot (64 B at 16)

// One lane per fragment: its group key; a member (key != its index) takes a slot of its group by an atomic ticket
// (claim order, sorted back into batch order by the group's head in df_process_kernel) while slots remain; past
// kGroupSlots it is only counted (the head then finds every member from gkey).  Also: the parsed record's words 6-7 for the process kernel, the completion tile counts cleared,
// and (workgroup 0) the running count and free-stack top moved past this batch's admissions.
__global__ void __launch_bounds__(kBlock) df_group_kernel(DfArgs a) {
    const uint32_t j = blockIdx.x * kBlock + threadIdx.x;
    if (blockIdx.x == 0) {
        // after the admission kernel: the creators of this batch (the tile counts it ranked) move the running count
        // and the free-stack top (fcb_create's fetch-and-add, decode-defrag.c:74-81)
        const uint32_t tiles = (a.n + 63) / 64;
        uint32_t creators = 0;
        wg_tile_prefix<kBlock>(a.tcnt, 0u, tiles, &creators);
        const unsigned long long run = a.ctl[C_RUNNING], top = a.ctl[C_FREE_TOP];
        const unsigned long long room = run < a.fcb_max ? a.fcb_max - run : 0ull;
        const uint32_t adm = (uint32_t)(creators < room ? creators : room);
        // A workgroup whose look-back failed created none of its creators' FCBs, but its count stands in every later
        // rank: the records at its ranks (below adm) were skipped.  They go back onto the stack, under the new top, so
        // the running count and the free stack stay exact.  (Rare: no failure, nothing to do.)
        const uint32_t nfail = (uint32_t)(a.ctl[C_FAILN] < kMaxFail ? a.ctl[C_FAILN] : kMaxFail);
        uint32_t skipped = 0, held[kMaxFail], hn[kMaxFail], ho[kMaxFail];
        for (uint32_t f = 0; f < nfail; ++f) {
            const uint32_t t0 = min((uint32_t)a.ctl[C_FAIL0 + f] * (kBlock / 64), tiles);
            __syncthreads();   // (wg_tile_prefix's partial sums are reused)
            const uint32_t lo = min(wg_tile_prefix<kBlock>(a.tcnt, t0, tiles, nullptr), adm);
            __syncthreads();
            const uint32_t hi = min(wg_tile_prefix<kBlock>(a.tcnt, min(t0 + kBlock / 64, tiles), tiles, nullptr), adm);
            hn[f] = hi - lo;
            ho[f] = skipped;
            skipped += hi - lo;
            if (threadIdx.x < hi - lo) held[f] = a.freestk[top - 1 - (lo + threadIdx.x)];
        }
        __syncthreads();   // every skipped record read before any is written
        for (uint32_t f = 0; f < nfail; ++f)
            if (threadIdx.x < hn[f]) a.freestk[top - adm + ho[f] + threadIdx.x] = held[f];
        if (threadIdx.x == 0) {
            a.ctl[C_CREATORS] = creators;
            a.ctl[C_RUNNING] = run + adm - skipped;
            a.ctl[C_FREE_TOP] = top - adm + skipped;
            a.ctl[C_NEW] += adm - skipped;
            a.ctl[C_FAILN] = 0;
        }
    }
    if (j >= a.n) return;
    if (__lane_id() == 0) a.dcnt[j >> 6] = 0u;
    const uint32_t key = df_group_key(a, j);
    a.gkey[j] = key;
    // the process kernel's view of the fragment, in its parsed record's last two words (the hash and the valid flag
    // are dead after the claim): word 6 = its FCB record (kNone: none), word 7 = its table slot (kNone: not a
    // fragment).  The group head then reaches its FCB header in one load instead of three dependent ones.
    const uint32_t s = a.fslot[j];
    const bool rec = s < kNone - 1 && a.tstate[s] == kLive;
    uint2 w67;
    w67.x = rec ? a.tkey[(size_t)s * 4 + 3] : kNone;
    w67.y = s < kNone - 1 ? s : kNone;
    *(uint2 *)(a.frec + (size_t)j * kFrecWords + 6) = w67;
    if (key != j) {
        const uint32_t pos = atomicAdd(a.gcnt + key, 1u);
        if (pos < kGroupSlots) a.gslot[(size_t)key * kGroupStride + pos] = j;
    }
}

// ---- the reference state machine, one lane per FCB --------------------------------------------------------------------
__device__ __forceinline__ uint32_t chain_at(uint64_t order, uint32_t pos) { return (uint32_t)(order >> (4 * pos)) & 15u; }

// cdesc: word 0 (offset | frag_len << 16) of the lane's FCB's chain descriptors, which the chain scan reads serially:
// LDS round trips instead of global ones.  Private per lane ([slot][lane]: no bank conflicts), no barrier.
// cidx: batch index + 1 of the fragment each chain slot received in this batch (0: an earlier batch).  When the FCB
// completes, these go to descriptor word 3 and the fragments are not stashed: the assembly reads them from the input.
// The head lane's loads come in three dependent rounds, not one per chain step: (1) its group's member count and
// slots (one 64-B row; a bitonic network puts them in batch order); (2) the head's parsed record, which carries its
// FCB record and table slot (df_group_kernel), and the members' parsed records; (3) the FCB header (and, for an FCB
// from an earlier batch, its chain descriptors).  A group with more members than slots steps them one by one.
constexpr uint32_t kWin = DF_PROC_WIN;
__device__ __forceinline__ void df_process_one(const DfArgs &a, uint32_t j, uint32_t (*cdesc)[kBlock],
                                               uint32_t (*cidx)[kBlock], uint32_t *st, uint32_t &teardrop) {
    const uint32_t tl = threadIdx.x;
    if (a.gkey[j] != j) return;   // not the head of its group: the group's key is its first fragment's index
    const uint32_t g = j;
    const uint32_t cnt = a.gcnt[g];    // members besides the head (in slots, past kGroupSlots in the overflow list)
    uint32_t iq[kWin];
    iq[0] = g;
#pragma unroll
    for (uint32_t u = 1; u < kWin; ++u) iq[u] = u <= cnt ? a.gslot[(size_t)g * kGroupStride + u - 1] : kNone;
    if (cnt) a.gcnt[g] = 0;            // (for the next call)
    const bool more = cnt > kGroupSlots;   // (rare) the members are stepped one by one, by index, below
    // the slots hold the members in ticket order: a bitonic network puts the window in batch order (the head, the
    // group's smallest index, stays first; the unused entries, kNone, last)
    static_assert(kWin == kGroupSlots + 1 && (kWin & (kWin - 1)) == 0, "window = head + slots, a power of two");
#pragma unroll
    for (uint32_t k = 2; k <= kWin; k <<= 1)
#pragma unroll
        for (uint32_t jj = k >> 1; jj > 0; jj >>= 1)
#pragma unroll
            for (uint32_t i = 0; i < kWin; ++i) {
                const uint32_t l = i ^ jj;
                if (l > i) {
                    const uint32_t x = iq[i], y = iq[l], lo = min(x, y), hi = max(x, y);
                    iq[i] = (i & k) == 0 ? lo : hi;
                    iq[l] = (i & k) == 0 ? hi : lo;
                }
            }
    const uint32_t m = more ? 1u : 1u + cnt;   // window entries stepped from registers
    // the window's parsed-record words 2-5 (id | proto | mf, offset | frag_len, frame length, l2 | ihl*4): the state
    // machine reads nothing else of a fragment (its id goes to the FCB's id list in the stash / place kernels)
    uint4 fw[kWin];
    const uint2 h67 = *(const uint2 *)(a.frec + (size_t)g * kFrecWords + 6);
    fw[0] = *(const uint4 *)(a.frec + (size_t)g * kFrecWords + 2);
#pragma unroll
    for (uint32_t u = 1; u < kWin; ++u)
        if (u < m) fw[u] = *(const uint4 *)(a.frec + (size_t)iq[u] * kFrecWords + 2);
    const uint32_t r = h67.x, s0 = h67.y;
    if (s0 != kNone) a.creator[s0] = kNone;   // the group key has been used: reset for the next batch
    if (r == kNone) {   // a fragment without a record (no FCB, or not a fragment): a singleton group
        const uint32_t s = s0 != kNone ? PPE_DF_FCB_FULL : PPE_DF_NOT_FRAG;
        a.status[g] = s;
        a.inserted[g] = kNone;
        a.dgrec[g] = kNone;
        atomicAdd(st + s, 1u);   // (LDS: the workgroup's status counts)
        return;
    }
    uint32_t *h = a.rhdr + (size_t)r * kRecWords;
    const uint4 h03 = *(const uint4 *)h;
    const uint2 h45 = *(const uint2 *)(h + 4);
    uint32_t flags = h03.x & 0xffu, last_in = (h03.x >> 8) & 0xffu, cache_num = (h03.x >> 16) & 0xffu,
             nlist = h03.x >> 24;
    int total = (int)h03.y, meat = (int)h03.z;
    uint64_t order = (uint64_t)h45.x | ((uint64_t)h45.y << 32);
    uint32_t *descw = a.rdesc + (size_t)r * a.cache_max * 4;
    // descriptor word 2 of chain position 0 (l2 | ihl*4 << 8 | proto << 16): the completion's buffer check
    uint32_t hd0 = 0;
    if (cache_num) {   // an FCB from an earlier batch: its chain descriptors, one round of loads
        uint32_t cw[16];
#pragma unroll
        for (uint32_t k = 0; k < 16; ++k) cw[k] = k < cache_num ? descw[k * 4] : 0u;
        if (nlist) hd0 = descw[chain_at(order, 0) * 4 + 2];
#pragma unroll
        for (uint32_t k = 0; k < 16; ++k) {
            cdesc[k][tl] = cw[k];
            cidx[k][tl] = 0;
        }
    }
    // the segment's fragments in order: the window's entries by static index (the step is inlined once per window
    // position, so no register array is shifted or indexed per lane), then a longer segment's rest one by one
    auto step = [&](const uint32_t i, const uint4 w) {
        const uint32_t fr[6] = {0u, 0u, w.x, w.y, w.z, w.w};   // (words 0-1 unused here)
        uint32_t out = PPE_DF_CACHED, ins = kNone, done = kNone;
        bool tear = false;
        // FragFind / fcb_create refresh the FCB's timestamp (decode-defrag.c:139, 472); a.rts[r] = now below
        if (fr[4] > a.frag_buf) {
            out = PPE_DF_HW2SW_ERR;                    // PACKET_HW2SW (decode-defrag.c:415-420)
        } else if (flags & kRecDelete) {
            out = PPE_DF_DELETED;                      // decode-defrag.c:422-427 (no counter)
        } else if (cache_num >= a.cache_max) {
            out = PPE_DF_CACHE_FULL;                   // decode-defrag.c:429-437
        } else {
            // Frag_defrag_process (decode-defrag.c:292-406)
            const int offset = (int)(fr[3] & 0xffffu);
            const int flen = (int)(fr[3] >> 16);
            const int end = offset + flen;
            const bool mf = (fr[2] >> 24) & 1u;
            bool err = false;
            if (!mf) {
                if (end < total || (last_in & kLastIn)) err = true;
                else {
                    last_in |= kLastIn;
                    total = end;
                }
            } else if (end > total) {
                if (last_in & kLastIn) err = true;
                else total = end;
            }
            uint32_t pos = nlist;       // insert before chain position pos
            if (!err) {
                int prev = -1, next = -1;
                if (nlist == 0 || (int)(cdesc[chain_at(order, nlist - 1)][tl] & 0xffffu) < offset) {
                    prev = nlist ? (int)chain_at(order, nlist - 1) : -1;
                } else {
                    // the reference's scan compares the chained fragment's frag_len with the new offset
                    // (decode-defrag.c:344-349)
                    for (pos = 0; pos < nlist; ++pos) {
                        const uint32_t k = chain_at(order, pos);
                        if ((int)(cdesc[k][tl] >> 16) >= offset) {
                            next = (int)k;
                            break;
                        }
                        prev = (int)k;
                    }
                }
                if (prev >= 0) {
                    const uint32_t pd = cdesc[prev][tl];
                    if ((int)(pd & 0xffffu) + (int)(pd >> 16) - offset > 0) err = tear = true;
                }
                if (!err && next >= 0 && (int)(cdesc[next][tl] & 0xffffu) - end < 0) err = tear = true;
            }
            if (err) {
                out = PPE_DF_DEFRAG_ERR;
                teardrop += tear ? 1u : 0u;
            } else {
                const uint32_t k = cache_num;      // store slot: the fragment's arrival rank in this FCB
                const uint32_t w2 = fr[5] | ((fr[2] >> 16) & 0xffu) << 16;
                *(uint4 *)(descw + k * 4) = make_uint4(fr[3], fr[4], w2, 0u);
                cdesc[k][tl] = fr[3];
                cidx[k][tl] = i + 1;
                if (pos == 0) hd0 = w2;
                const uint64_t lo = order & ((1ull << (4 * pos)) - 1ull);
                const uint64_t hi = pos + 1 < 16 ? (order >> (4 * pos)) << (4 * (pos + 1)) : 0ull;
                order = lo | ((uint64_t)k << (4 * pos)) | hi;
                nlist++;
                cache_num++;
                meat += flen;
                if (offset == 0) last_in |= kFirstIn;
                ins = (r << 8) | k;
                if (last_in == (kFirstIn | kLastIn) && meat == total) {
                    // Frag_defrag_reasm / Frag_defrag_setup: the buffer is total + L2 + ihl*4 bytes of an 8 KB
                    // slice (ICMP: 1000 bytes, always available)
                    const uint32_t need = (uint32_t)total + (hd0 & 0xffu) + ((hd0 >> 8) & 0xffu);
                    if (((hd0 >> 16) & 0xffu) != 1u && need > a.reasm_buf) {
                        out = PPE_DF_SETUP_ERR;
                    } else {
                        out = PPE_DF_REASM;
                        flags |= kRecComplete | kRecDelete;
                        done = r;
                        // this batch's fragments of the datagram are read from the input, not stashed
                        for (uint32_t kk = 0; kk < cache_num; ++kk) {
                            const uint32_t x = cidx[kk][tl];
                            descw[kk * 4 + 3] = x;
                            if (x && x - 1 != i) a.inserted[x - 1] = kNone;
                        }
                        ins = kNone;
                    }
                }
            }
        }
        a.status[i] = out | (tear ? PPE_DF_TEARDROP : 0u);
        a.inserted[i] = ins;
        a.dgrec[i] = done;
        // the place kernel's per-tile count of completing fragments (zeroed by the group kernel)
        if (done != kNone) atomicAdd(a.dcnt + (i >> 6), 1u);
        atomicAdd(st + out, 1u);
    };
#pragma unroll
    for (uint32_t u = 0; u < kWin; ++u)
        if (u < m) step(iq[u], fw[u]);
    if (more) {
        // more members than slots (rare): the members are the indices above the head whose group key is the head's,
        // found in batch order by one pass over gkey from g + 1 that stops at the last member.  Cost: the span from
        // the head to its last member in 16-index rounds (independent key loads, then the matches' records loaded
        // together), plus one step per member: linear in the batch, whatever the number of members or of groups
        // past their slots (a scan of a shared overflow list per member was O(cnt x overflow)).
        constexpr uint32_t R = 16;
        uint32_t left = cnt;
        for (uint32_t base = g + 1; left && base < a.n; base += R) {
            uint32_t mask = 0;
#pragma unroll
            for (uint32_t u = 0; u < R; ++u) {
                const uint32_t x = base + u;
                mask |= (x < a.n && a.gkey[x] == g) ? 1u << u : 0u;
            }
            uint4 fr[R];
#pragma unroll
            for (uint32_t u = 0; u < R; ++u)
                if ((mask >> u) & 1u) fr[u] = *(const uint4 *)(a.frec + (size_t)(base + u) * kFrecWords + 2);
            while (mask) {
                const uint32_t u = (uint32_t)__builtin_ctz(mask);
                mask &= mask - 1u;
                uint4 w = fr[0];
#pragma unroll
                for (uint32_t v = 1; v < R; ++v) w = v == u ? fr[v] : w;   // (a select chain: no indexed registers)
                step(base + u, w);
                --left;
            }
        }
    }
    *(uint4 *)h = make_uint4(flags | (last_in << 8) | (cache_num << 16) | (nlist << 24), (uint32_t)total,
                             (uint32_t)meat, h03.w);
    *(uint2 *)(h + 4) = make_uint2((uint32_t)order, (uint32_t)(order >> 32));
    a.rts[r] = a.now;
}

__global__ void __launch_bounds__(kBlock) df_process_kernel(DfArgs a) {
    __shared__ uint32_t cdesc[16][kBlock];
    __shared__ uint32_t cidx[16][kBlock];
    __shared__ uint32_t wg[PPE_DF__COUNT + 1];   // per-status counts + teardrops of this workgroup
    if (threadIdx.x <= PPE_DF__COUNT) wg[threadIdx.x] = 0;
    __syncthreads();
    uint32_t teardrop = 0;
    const uint32_t j = blockIdx.x * kBlock + threadIdx.x;
    // per-fragment LDS atomics into the workgroup's status counts (one instruction each, nothing waits on them), then
    // one global atomic per counter per workgroup: per-lane global atomics on the same few words serialise in one L2
    // channel (they were most of this kernel's time)
    if (j < a.n) df_process_one(a, j, cdesc, cidx, wg, teardrop);
    if (teardrop) atomicAdd(&wg[PPE_DF__COUNT], teardrop);
    __syncthreads();
    if (threadIdx.x <= PPE_DF__COUNT && wg[threadIdx.x])
        atomicAdd(a.ctl + (threadIdx.x < PPE_DF__COUNT ? C_ST0 + threadIdx.x : C_TEARDROP),
                  (unsigned long long)wg[threadIdx.x]);
}

// DF_AB (diagnostic builds only, wrong outputs): 2 = no window bytes, 4 = no header checksum, 8 = datagram bytes not
// copied, 16 = held frames not stashed
#ifndef DF_AB
#define DF_AB 0
#endif

// a raw buffer descriptor over [p, p + bytes) from wave-uniform values (readfirstlane: the compiler cannot prove a
// wave's frame pointer uniform, and a descriptor in VGPRs would be waterfalled)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t df_rsrc(uint64_t p, uint32_t bytes) {
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)p), hi = __builtin_amdgcn_readfirstlane((uint32_t)(p >> 32));
    return __builtin_amdgcn_make_buffer_rsrc((void *)(uintptr_t)(((uint64_t)hi << 32) | lo), 0,
                                             (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}

// ---- stash: copy held frames into their FCB's store slot (PACKET_HW2SW; run in the assembly launch) ------------------
__device__ __forceinline__ void df_stash_one(const DfArgs &a, uint32_t i) {
    if (DF_AB & 16) return;
    // the fragment's slot, frame and id read together (one round trip, not two)
    const uint32_t ins = a.inserted[i];
    const uint64_t off = a.off[i];
    const uint32_t tot = a.len[i];
    const uint64_t fid = a.id ? a.id[i] : (uint64_t)i;
    if (ins == kNone) return;
    const uint32_t r = ins >> 8, k = ins & 0xffu;
    const uint8_t *src = a.pkt + off;
    uint8_t *dst = a.store + ((size_t)r * a.cache_max + k) * a.sstride;
    const uint32_t lane = __lane_id();
    // the held fragment's id, kept with its store slot (the FCB's id list: later datagram plans and aging read it)
    if (lane == 0) a.rid[(size_t)r * a.cache_max + k] = fid;
    // every load of a pass is issued before its stores (2 KB per pass: one pass for a frag_buf frame), through buffer
    // descriptors whose range check drops the lanes past the frame: no lane-dependent branch, so the stores do not
    // each wait for the one before (global stores count in vmcnt on gfx950, and a store under a branch after
    // predicated loads gets a full wait)
    const uint64_t sp = (uint64_t)(uintptr_t)src, dp = (uint64_t)(uintptr_t)dst;
    const __amdgpu_buffer_rsrc_t rsb = df_rsrc(sp, tot), rdb = df_rsrc(dp, tot);
    if ((sp & 3u) == 0) {
        const uint32_t words = tot / 4;
        const __amdgpu_buffer_rsrc_t rs = df_rsrc(sp, words * 4u), rd = df_rsrc(dp, words * 4u);
        const uint8_t t = __builtin_amdgcn_raw_buffer_load_b8(rsb, words * 4u + lane, 0, 0);   // the last 0-3 bytes
        constexpr uint32_t U = 8;
        for (uint32_t base = 0; base < words; base += 64 * U) {
            uint32_t v[U];
#pragma unroll
            for (uint32_t u = 0; u < U; ++u)
                v[u] = __builtin_amdgcn_raw_buffer_load_b32(rs, 4u * (base + u * 64 + lane), 0, 0);
#pragma unroll
            for (uint32_t u = 0; u < U; ++u)
                __builtin_amdgcn_raw_buffer_store_b32(v[u], rd, 4u * (base + u * 64 + lane), 0, 0);
        }
        if (lane < 4) __builtin_amdgcn_raw_buffer_store_b8(t, rdb, words * 4u + lane, 0, 0);
    } else {   // an unaligned frame: bytes, 16 per lane per pass
        constexpr uint32_t U = 16;
        for (uint32_t base = 0; base < tot; base += 64 * U) {
            uint8_t v[U];
#pragma unroll
            for (uint32_t u = 0; u < U; ++u) v[u] = __builtin_amdgcn_raw_buffer_load_b8(rsb, base + u * 64 + lane, 0, 0);
#pragma unroll
            for (uint32_t u = 0; u < U; ++u) __builtin_amdgcn_raw_buffer_store_b8(v[u], rdb, base + u * 64 + lane, 0, 0);
        }
    }
}

// ---- place: datagram index of each completing fragment, in index order ------------------------------------------------
__global__ void __launch_bounds__(kBlock) df_place_kernel(DfArgs a) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    const uint32_t t0 = blockIdx.x * (kBlock / 64), w = threadIdx.x >> 6;
    uint32_t nd = 0;
    uint32_t base = wg_tile_prefix<kBlock>(a.dcnt, t0, (a.n + 63) / 64, &nd);
    for (uint32_t k = 0; k < w; ++k) base += a.dcnt[t0 + k];   // the workgroup's earlier waves
    if (blockIdx.x == 0 && threadIdx.x == 0) {   // the datagram count (read by the assembly kernel, next)
        a.ctl[C_NDGRAM] = nd;
        a.ctl[C_DGRAMS] += nd;
        if (a.n_dgram) *a.n_dgram = nd;
    }
    // the slots of this workgroup's range past the datagram count: length 0 (a classify over all n slots sees runt
    // frames there, whatever their window bytes; the window and id rows past the count are not written)
    if (a.dgram_len && i < a.n && i >= nd) a.dgram_len[i] = 0;
    const uint32_t r = i < a.n ? a.dgrec[i] : kNone;
    const bool f = r != kNone;
    const uint64_t b = __builtin_amdgcn_ballot_w64(f);
    if (i >= a.n) return;
    uint32_t j = kNone;
    if (f) {
        j = base + (uint32_t)__popcll(b & lanemask_lt());
        // datagram j's assembly plan: its chain in chain order, entry p = {descriptor words 0-2, total | nlist << 24,
        // frame base address, fragment id}.  The FCB header → descriptors → frame offsets chain is walked here, one
        // lane per datagram, so each assembly wave starts from one read (j < min(n, fcb_max): one record each).
        const uint32_t *h = a.rhdr + (size_t)r * kRecWords;
        const uint4 h03 = *(const uint4 *)h;
        const uint2 h45 = *(const uint2 *)(h + 4);
        const uint32_t nlist = h03.x >> 24, hw = h03.y | (nlist << 24);
        const uint64_t order = (uint64_t)h45.x | ((uint64_t)h45.y << 32);
        const uint32_t *desc = a.rdesc + (size_t)r * a.cache_max * 4;
        uint4 dd[16];
        uint64_t id[16], fb[16];
#pragma unroll
        for (uint32_t p = 0; p < 16; ++p) {
            if (p < nlist) {
                const uint32_t kk = chain_at(order, p);
                dd[p] = *(const uint4 *)(desc + kk * 4);
            }
        }
#pragma unroll
        for (uint32_t p = 0; p < 16; ++p) {
            if (p < nlist) {
                const uint32_t kk = chain_at(order, p);
                // this batch's fragments (word 3 = index + 1): the input frame and id; earlier ones: the store slot
                // and the id the stash kept
                const uint32_t x = dd[p].w;
                fb[p] = x ? (uint64_t)(uintptr_t)(a.pkt + a.off[x - 1])
                          : (uint64_t)(uintptr_t)(a.store + ((size_t)r * a.cache_max + kk) * a.sstride);
                id[p] = x ? (a.id ? a.id[x - 1] : (uint64_t)(x - 1)) : a.rid[(size_t)r * a.cache_max + kk];
            }
        }
        uint32_t *pe = a.plan + (size_t)j * a.cache_max * 8;
#pragma unroll
        for (uint32_t p = 0; p < 16; ++p) {
            if (p < nlist) {
                *(uint4 *)(pe + p * 8) = make_uint4(dd[p].x, dd[p].y, dd[p].z, hw);
                *(uint4 *)(pe + p * 8 + 4) =
                    make_uint4((uint32_t)fb[p], (uint32_t)(fb[p] >> 32), (uint32_t)id[p], (uint32_t)(id[p] >> 32));
            }
        }
    }
    if (a.dgram_of) a.dgram_of[i] = j;
}

// ---- assemble: one wave per datagram slot ----------------------------------------------------------------------
#ifndef DF_COPY_U
#define DF_COPY_U 8
#endif
__device__ __forceinline__ void df_assemble_slot(const DfArgs &a, uint32_t j, uint32_t nd) {
    const uint32_t tid = __lane_id();
    uint8_t *win = (a.dgram_hdr && !(DF_AB & 2)) ? a.dgram_hdr + (size_t)j * a.hdr_stride : nullptr;
    if (j >= nd) return;   // an empty slot: the place kernel wrote its length
    // lane p holds chain entry p of the plan (df_place_kernel): descriptor words 0 (offset | frag_len << 16), 1 (frame
    // length), 2 (l2 | ihl*4 << 8 | proto << 16), the frame's base (the input frame when the fragment arrived in
    // this batch, else its store slot) and its id: one read for the whole chain, used below by lane broadcasts
    uint4 e0 = make_uint4(0u, 0u, 0u, 0u), e1 = e0;
    if (tid < a.cache_max) {
        const uint32_t *pe = a.plan + ((size_t)j * a.cache_max + tid) * 8;
        e0 = *(const uint4 *)pe;
        e1 = *(const uint4 *)(pe + 4);
    }
    const uint32_t hw = __shfl(e0.w, 0, 64);
    const uint32_t nlist = hw >> 24, total = hw & 0xffffffu;
    const bool live = tid < nlist;
    const uint32_t cd0 = live ? e0.x : 0u, cd1 = live ? e0.y : 0u, cd2 = live ? e0.z : 0u;
    const uintptr_t cbase = live ? (uintptr_t)(((uint64_t)e1.y << 32) | e1.x) : 0;
    auto seg_base = [&](uint32_t p) -> const uint8_t * {
        const uint32_t lo = __shfl((uint32_t)cbase, p, 64), hi = __shfl((uint32_t)((uint64_t)cbase >> 32), p, 64);
        return (const uint8_t *)(((uint64_t)hi << 32) | lo);
    };
    const uint32_t hd = __shfl(cd2, 0, 64);
    const uint32_t l2 = hd & 0xffu, ihl4 = (hd >> 8) & 0xffu, proto = (hd >> 16) & 0xffu;
    const uint32_t head_tot = __shfl(cd1, 0, 64);
    const bool icmp = proto == 1u;
    const uint8_t *hsrc = seg_base(0);
    // out_len = head frame + the later fragments' payloads (reasm_mb->pkt_totallen, decode-defrag.c:240-266)
    uint32_t out_len = head_tot;
    for (uint32_t p = 1; p < nlist; ++p) out_len += __shfl(cd0, p, 64) >> 16;
    // the IPv4 header's ten 16-bit words, all loaded in one round and the patch computed without a branch (under an
    // ICMP branch the compiler issued them in two dependent rounds)
    uint32_t hw16[10];
#pragma unroll
    for (uint32_t q = 0; q < 10; ++q) hw16[q] = ld_be16(hsrc + l2 + 2u * q);
    // header patch (non-ICMP: ip_len = ihl*4 + total, ip_off = 0, checksum; ICMP: ip_off = 0)
    const uint32_t iplen_new = (ihl4 + total) & 0xffffu;
    // IPV4CalculateChecksum (decode-ipv4.h:117-163) over the patched header: words 0-4, 6-9, then the options
    uint32_t cs = hw16[0] + iplen_new + hw16[2] + 0u /* ip_off */ + hw16[4] + hw16[6] + hw16[7] + hw16[8] + hw16[9];
    if (!icmp && ihl4 <= 60)
        for (uint32_t o = 20; o < ihl4; o += 2) cs += ld_be16(hsrc + l2 + o);
    cs = (cs >> 16) + (cs & 0xffffu);
    cs += cs >> 16;
    const bool fix = !icmp && !(DF_AB & 4);
    const uint32_t w_iplen = fix ? iplen_new : hw16[1], w_csum = fix ? (~cs) & 0xffffu : hw16[5];
    auto patched = [&](uint32_t b, uint32_t v) -> uint32_t {
        const uint32_t o = b - l2;
        if (b < l2 || o >= 12) return v;
        if (o == 2) return w_iplen >> 8;
        if (o == 3) return w_iplen & 0xffu;
        if (o == 6 || o == 7) return 0u;
        if (o == 10) return w_csum >> 8;
        if (o == 11) return w_csum & 0xffu;
        return v;
    };
    // the reassembled frame: segment 0 = the head frame, segment p = the last flen bytes of chain entry p
    // (ICMP: the head frame only; the reference sizes the buffer but copies nothing else)
    uint8_t *full = (a.dgram_pkt && !(DF_AB & 8)) ? a.dgram_pkt + (size_t)j * a.reasm_buf : nullptr;
    const uint32_t stride = a.hdr_stride;
    uint32_t dst0 = 0;
    // whole output dwords are assembled from two aligned source dwords (a funnel shift) and stored as dwords; the
    // partial dwords at a segment's ends are stored bytewise (the neighbouring segment owns their other bytes)
    const bool wide = full && ((uintptr_t)full & 3u) == 0 && (a.reasm_buf & 3u) == 0;
    // when the head frame covers the whole window, the window is the first `stride` bytes of the frame: its dwords
    // are stored from the wide pass's registers (no byte pass of its own: one dependent round trip fewer)
    const bool wfast = wide && win && ((uintptr_t)win & 3u) == 0 && head_tot >= stride && a.reasm_buf >= stride;
    for (uint32_t p = 0; p < (icmp ? 1u : nlist); ++p) {
        const uint32_t tot = __shfl(cd1, p, 64), flen = __shfl(cd0, p, 64) >> 16;
        const uint8_t *src = seg_base(p) + (p == 0 ? 0u : tot - flen);
        const uint32_t cnt = p == 0 ? tot : flen;
        if (win && dst0 < stride && !wfast) {
            const uint32_t wl = cnt < stride - dst0 ? cnt : stride - dst0;
            for (uint32_t b = tid; b < wl; b += 64) win[dst0 + b] = (uint8_t)patched(dst0 + b, src[b]);
        }
        if (full) {
            const uint32_t end = dst0 + cnt < a.reasm_buf ? dst0 + cnt : a.reasm_buf;   // output bytes [dst0, end)
            if (wide && end > dst0) {
                const uint32_t wa = (dst0 + 3u) >> 2, we = end >> 2;   // whole dwords [wa, we)
                // the segment's source shift is the same for every dword: aligned loads, funnel-shifted pairs
                const uintptr_t s0 = (uintptr_t)(src + (4u * wa - dst0));
                const uint32_t sh = (uint32_t)(s0 & 3u) * 8u;
                const uint32_t *ap = (const uint32_t *)(s0 & ~(uintptr_t)3);   // source dword of output dword wa
                // DF_COPY_U dwords per lane per pass, every load issued before the stores; each source dword is
                // loaded once: the funnel partner of dword w is dword w + 1, the next lane's (lane 63: the next
                // row's lane 0, or for the last row one more dword)
                constexpr uint32_t U = DF_COPY_U;
                for (uint32_t base = wa; base < we; base += 64 * U) {
                    uint32_t lo[U];
#pragma unroll
                    for (uint32_t u = 0; u < U; ++u) {
                        const uint32_t w = base + u * 64 + tid;
                        lo[u] = (w < we || (w == we && sh)) ? ap[w - wa] : 0u;
                    }
                    const uint32_t wn = base + 64 * U;   // the dword after the pass (lane 63's last partner)
                    const uint32_t nx = (sh && wn <= we) ? ap[wn - wa] : 0u;
#pragma unroll
                    for (uint32_t u = 0; u < U; ++u) {
                        const uint32_t w = base + u * 64 + tid;
                        uint32_t hi = __shfl_down(lo[u], 1, 64);
                        const uint32_t hn = u + 1 < U ? __shfl(lo[u + 1 < U ? u + 1 : u], 0, 64) : nx;
                        if (tid == 63) hi = hn;
                        if (w >= we) continue;
                        uint32_t v = sh ? (lo[u] >> sh) | (hi << (32u - sh)) : lo[u];
                        if (4u * w + 3u >= l2 && 4u * w < l2 + 12u) {
                            uint32_t pv = 0;
                            for (uint32_t q = 0; q < 4; ++q)
                                pv |= patched(4u * w + q, (v >> (8u * q)) & 0xffu) << (8u * q);
                            v = pv;
                        }
                        ((uint32_t *)full)[w] = v;
                        if (wfast && p == 0 && w < stride / 4u) ((uint32_t *)win)[w] = v;
                    }
                }
                // head bytes [dst0, 4*wa) and tail bytes [4*we, end) (when the segment lies inside one dword, all)
                const uint32_t hb = 4u * wa < end ? 4u * wa : end;
                const uint32_t tb = 4u * we > hb ? 4u * we : hb;
                const uint32_t t = tid;
                if (t < hb - dst0) full[dst0 + t] = (uint8_t)patched(dst0 + t, src[t]);
                if (t < end - tb) full[tb + t] = (uint8_t)patched(tb + t, src[tb - dst0 + t]);
            } else {
                for (uint32_t ob = dst0 + tid; ob < end; ob += 64)
                    full[ob] = (uint8_t)patched(ob, src[ob - dst0]);
            }
        }
        dst0 += cnt;
    }
    if (icmp && full) {   // bytes the reference never wrote: zero
        const uint32_t lim = out_len < a.reasm_buf ? out_len : a.reasm_buf;
        for (uint32_t b = dst0 + tid; b < lim; b += 64) full[b] = 0;
    }
    if (win)
        for (uint32_t b = dst0 + tid; b < stride; b += 64) win[b] = 0;
    if (tid == 0 && a.dgram_len) a.dgram_len[j] = out_len;
    if (a.dgram_frags && tid < a.cache_max)
        a.dgram_frags[(size_t)j * a.cache_max + tid] = live ? (((uint64_t)e1.w << 32) | e1.z) : ~0ull;
}

// one wave per batch position w: datagram slot w, or (positions past the datagram count) the stashes of a share of
// the fragments (a fixed grid striding over the slots measured slower: 50 vs 40 µs for D1).  The two are independent
// (the stash writes the store slots of fragments held past this batch; the assembly reads this batch's fragments
// from the input and earlier batches' from their store slots), so they share one launch.
#ifndef DF_ASM_WAVES
#define DF_ASM_WAVES 0   // > 0: the compiler is held to this many waves per SIMD (A/B builds)
#endif
#if DF_ASM_WAVES > 0
__global__ void __launch_bounds__(kSlotBlock) __attribute__((amdgpu_waves_per_eu(DF_ASM_WAVES, DF_ASM_WAVES)))
#else
__global__ void __launch_bounds__(kSlotBlock)
#endif
df_assemble_kernel(DfArgs a) {
    const uint32_t w = blockIdx.x * (kSlotBlock / 64) + (threadIdx.x >> 6);
    if (w >= a.n) return;
    const uint32_t nd = (uint32_t)a.ctl[C_NDGRAM];
    if (w < nd) {
        df_assemble_slot(a, w, nd);
        if (nd == a.n) df_stash_one(a, w);   // (every position a datagram: nothing is held, checked anyway)
    } else {
        // the stashes go to the waves without a datagram, so no wave copies both: wave w takes fragments
        // w - nd, w - nd + (n - nd), ...
        for (uint32_t i = w - nd; i < a.n; i += a.n - nd) df_stash_one(a, i);
    }
}

// ---- aging + table rebuild (one workgroup) ----------------------------------------------------------------------------
__global__ void __launch_bounds__(kScanT) df_age_kernel(DfArgs a) {
    __shared__ uint32_t nfreed, ndropped;
    if (threadIdx.x == 0) nfreed = ndropped = 0;
    __syncthreads();
    const uint32_t top = (uint32_t)a.ctl[C_FREE_TOP];
    for (uint32_t r = threadIdx.x; r < a.fcb_max; r += kScanT) {
        uint32_t *h = a.rhdr + (size_t)r * kRecWords;
        const uint32_t f = h[0];
        if (!(f & kRecLive)) continue;
        const unsigned long long t = a.rts[r];
        // Frag_defrag_timeout (decode-defrag.c:515-520): idle past the timeout, or marked DEFRAG_DELETE
        if (!((a.now > t && a.now - t > a.timeout) || (f & kRecDelete))) continue;
        if (!(f & kRecComplete)) {
            const uint32_t nlist = f >> 24;
            const uint64_t order = (uint64_t)h[4] | ((uint64_t)h[5] << 32);
            for (uint32_t p = 0; p < nlist; ++p) {
                const uint32_t slot = atomicAdd(&ndropped, 1u);
                if (slot < a.max_dropped) a.dropped[slot] = a.rid[(size_t)r * a.cache_max + chain_at(order, p)];
            }
        }
        h[0] = 0;
        a.freestk[top + atomicAdd(&nfreed, 1u)] = r;
    }
    // rebuild the table from the live records (deleted keys and tombstones vanish)
    for (uint32_t s = threadIdx.x; s <= a.smask; s += kScanT) {
        a.tstate[s] = kEmpty;
        a.creator[s] = kNone;
    }
    __threadfence();
    __syncthreads();
    for (uint32_t r = threadIdx.x; r < a.fcb_max; r += kScanT) {
        const uint32_t *h = a.rhdr + (size_t)r * kRecWords;
        if (!(h[0] & kRecLive)) continue;
        // the key of record r: the table keys are rebuilt from the record's copy
        const uint32_t sip = h[6], dip = h[7], id = h[3];
        uint32_t s = key_hash(sip, dip, id) & a.smask;
        while (atomicCAS(a.tstate + s, kEmpty, kLive) != kEmpty) s = (s + 1) & a.smask;
        uint32_t *k = a.tkey + (size_t)s * 4;
        k[0] = sip;
        k[1] = dip;
        k[2] = id;
        k[3] = r;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        a.ctl[C_RUNNING] -= nfreed;
        a.ctl[C_DEL] += nfreed;
        a.ctl[C_FREE_TOP] = top + nfreed;
        a.ctl[C_TIMEOUT_DROP] += ndropped;
        a.ctl[C_AGE_DROPPED] = ndropped;
        a.ctl[C_AGE_FREED] = nfreed;
    }
}

__global__ void df_init_kernel(DfArgs a) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t <= a.smask) {
        a.tstate[t] = kEmpty;
        a.creator[t] = kNone;
    }
    if (t < a.fcb_max) {
        a.freestk[t] = a.fcb_max - 1 - t;
        a.rhdr[(size_t)t * kRecWords] = 0;
    }
    if (t < C_WORDS) a.ctl[t] = t == C_FREE_TOP ? a.fcb_max : 0ull;
    if (t < a.nlook) a.look[t] = 0ull;
    if (t < a.max_batch) a.gcnt[t] = 0u;   // (then each group's head clears its count after use)
}

}  // namespace

struct ppe_defrag_table {
    int device = 0;
    ppe_defrag_cfg_t cfg{};
    uint32_t nslots = 0, sstride = 0;
    DfArgs base{};   // persistent device pointers + sizes
    void *allocs[24] = {};
    int nalloc = 0;
    unsigned long long *h_ctl = nullptr;   // pinned
    unsigned long long *h_err = nullptr;   // pinned, device-mapped: a batch's admission look-back failed
    uint32_t epoch = 0;                    // admission look-back tag of the last call
    char err[256] = {0};
};

namespace {

int dfail(ppe_defrag_t *d, int code, const char *fmt, ...) {
    if (d) {
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(d->err, sizeof(d->err), fmt, ap);
        va_end(ap);
    }
    return code;
}

template <typename T>
bool dalloc(ppe_defrag_t *d, T **p, size_t count) {
    void *q = nullptr;
    if (hipMalloc(&q, std::max<size_t>(count * sizeof(T), 64)) != hipSuccess) return false;
    d->allocs[d->nalloc++] = q;
    *p = (T *)q;
    return true;
}

uint32_t blocks(uint64_t items, uint32_t per) { return (uint32_t)std::max<uint64_t>(1, (items + per - 1) / per); }

int launched(ppe_defrag_t *d, const char *what) {
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? PPE_OK : dfail(d, PPE_EIO, "%s: %s", what, hipGetErrorString(e));
}

}  // namespace

extern "C" {

int ppe_defrag_create(ppe_ctx_t *ctx, const ppe_defrag_cfg_t *cfg, ppe_defrag_t **out) {
    if (!ctx || !out) return PPE_EINVAL;
    *out = nullptr;
    ppe_defrag_cfg_t c = cfg ? *cfg : ppe_defrag_cfg_t{};
    if (!c.fcb_max) c.fcb_max = 1024;
    if (!c.cache_max) c.cache_max = 8;
    if (!c.frag_buf_bytes) c.frag_buf_bytes = 2024;
    if (!c.reasm_buf_bytes) c.reasm_buf_bytes = 8168;
    if (!c.max_batch) c.max_batch = 65536;
    if (c.cache_max > 16 || c.fcb_max > (1u << 20) || c.frag_buf_bytes > 4096 || c.reasm_buf_bytes > (1u << 20) ||
        c.max_batch > (1u << 24))
        return PPE_EINVAL;
    const int dev = ppe_ctx_device(ctx);
    if (dev < 0 || hipSetDevice(dev) != hipSuccess) return PPE_ENODEV;
    ppe_defrag_t *d = new (std::nothrow) ppe_defrag_t();
    if (!d) return PPE_ENOMEM;
    d->device = dev;
    d->cfg = c;
    uint32_t ns = 1024;
    while (ns < 2ull * ((uint64_t)c.fcb_max + c.max_batch)) ns <<= 1;
    d->nslots = ns;
    d->sstride = (c.frag_buf_bytes + 63u) & ~63u;
    DfArgs &a = d->base;
    a.smask = ns - 1;
    a.fcb_max = c.fcb_max;
    a.cache_max = c.cache_max;
    a.frag_buf = c.frag_buf_bytes;
    a.reasm_buf = c.reasm_buf_bytes;
    a.sstride = d->sstride;
    const uint32_t mb = c.max_batch;
    // the store carries 64 spare bytes: df_assemble_kernel reads whole aligned dwords past a frame's last byte
    bool ok = dalloc(d, &a.tstate, ns) && dalloc(d, &a.tkey, (size_t)ns * 4) && dalloc(d, &a.creator, ns) &&
              dalloc(d, &a.rhdr, (size_t)c.fcb_max * kRecWords) &&
              dalloc(d, &a.rdesc, (size_t)c.fcb_max * c.cache_max * 4) && dalloc(d, &a.rts, c.fcb_max) &&
              dalloc(d, &a.rid, (size_t)c.fcb_max * c.cache_max) &&
              dalloc(d, &a.store, (size_t)c.fcb_max * c.cache_max * d->sstride + 64) && dalloc(d, &a.freestk, c.fcb_max) &&
              dalloc(d, &a.ctl, C_WORDS) && dalloc(d, &a.frec, (size_t)mb * kFrecWords) && dalloc(d, &a.fslot, mb) &&
              dalloc(d, &a.inserted, mb) && dalloc(d, &a.dgrec, mb) &&
              dalloc(d, &a.plan, (size_t)std::min(mb, c.fcb_max) * c.cache_max * 8) &&
              dalloc(d, &a.tcnt, blocks(mb, 64)) && dalloc(d, &a.dcnt, blocks(mb, 64)) && dalloc(d, &a.gkey, mb) &&
              dalloc(d, &a.gcnt, mb) && dalloc(d, &a.gslot, (size_t)mb * kGroupStride) &&
              dalloc(d, &a.dropped, (size_t)c.fcb_max * c.cache_max) &&
              dalloc(d, &a.look, blocks(mb, kBlock));
    if (ok && hipHostMalloc((void **)&d->h_ctl, C_WORDS * sizeof(unsigned long long), hipHostMallocDefault) != hipSuccess)
        ok = false;
    if (ok && (hipHostMalloc((void **)&d->h_err, sizeof(unsigned long long), hipHostMallocMapped) != hipSuccess ||
               hipHostGetDevicePointer((void **)&a.err_host, d->h_err, 0) != hipSuccess))
        ok = false;
    if (!ok) {
        ppe_defrag_destroy(d);
        return PPE_ENOMEM;
    }
    a.max_dropped = c.fcb_max * c.cache_max;
    a.max_batch = mb;
    a.nlook = blocks(mb, kBlock);
    *d->h_err = 0;
    a.look_spins = 1u << 22;
    a.look_fail_wg = ~0u;
    if (const char *e = getenv("PPE_DF_LOOK_FAIL"))  // test hook: this workgroup index fails its look-back
        a.look_fail_wg = (uint32_t)atoi(e);
    const uint32_t span = std::max(std::max(std::max(ns, a.nlook), std::max(c.fcb_max, (uint32_t)C_WORDS)), mb);
    hipLaunchKernelGGL(df_init_kernel, dim3(blocks(span, 256)), dim3(256), 0, 0, a);
    if (hipDeviceSynchronize() != hipSuccess) {
        ppe_defrag_destroy(d);
        return PPE_EIO;
    }
    *out = d;
    return PPE_OK;
}

int ppe_defrag_destroy(ppe_defrag_t *d) {
    if (!d) return PPE_EINVAL;
    (void)hipSetDevice(d->device);
    (void)hipDeviceSynchronize();
    for (int k = 0; k < d->nalloc; ++k) (void)hipFree(d->allocs[k]);
    if (d->h_ctl) (void)hipHostFree(d->h_ctl);
    if (d->h_err) (void)hipHostFree(d->h_err);
    delete d;
    return PPE_OK;
}

const char *ppe_defrag_last_error(ppe_defrag_t *d) { return d ? d->err : "null defrag table"; }

int ppe_defrag(ppe_defrag_t *d, const ppe_frag_batch_t *in, const ppe_defrag_out_t *out, void *stream) {
    if (!d || !in || !out) return PPE_EINVAL;
    if (in->n == 0) return PPE_OK;
    if (in->n > d->cfg.max_batch) return dfail(d, PPE_EINVAL, "batch of %u fragments > max_batch %u", in->n,
                                               d->cfg.max_batch);
    if (!in->pkt || !in->off || !in->len || !out->status || !out->dgram_hdr || !out->dgram_len)
        return dfail(d, PPE_EINVAL, "pkt/off/len and status/dgram_hdr/dgram_len are required");
    if (out->hdr_stride != 64 && out->hdr_stride != 128) return dfail(d, PPE_EINVAL, "hdr_stride must be 64 or 128");
    if (hipSetDevice(d->device) != hipSuccess) return PPE_ENODEV;
    // an earlier batch's admission look-back failed (its creators were not admitted; reported once, then cleared):
    // read from pinned memory the admit kernel writes, no synchronisation
    if (__atomic_load_n(d->h_err, __ATOMIC_ACQUIRE)) {
        __atomic_store_n(d->h_err, 0ull, __ATOMIC_RELAXED);
        return dfail(d, PPE_EIO, "ppe_defrag: an earlier batch's admission look-back timed out: the FCBs of that "
                                 "batch's workgroup were not created (its fragments' results are wrong)");
    }
    const hipStream_t s = (hipStream_t)stream;
    DfArgs a = d->base;
    a.pkt = in->pkt;
    a.off = in->off;
    a.len = in->len;
    a.id = in->id;
    a.n = in->n;
    a.now = in->now_seconds;
    a.status = out->status;
    a.dgram_of = out->dgram_of;
    a.dgram_hdr = out->dgram_hdr;
    a.dgram_len = out->dgram_len;
    a.dgram_pkt = out->dgram_pkt;
    a.dgram_frags = out->dgram_frags;
    a.n_dgram = out->n_dgram;
    a.hdr_stride = out->hdr_stride;
    const uint32_t g = blocks(a.n, kBlock);
    hipLaunchKernelGGL(df_parse_kernel, dim3(g), dim3(kBlock), 0, s, a);
    if (++d->epoch == 0) d->epoch = 1;   // (0 is the cleared array's tag)
    a.epoch = d->epoch;
    hipLaunchKernelGGL(df_admit_kernel, dim3(g), dim3(kBlock), 0, s, a);
    d->base.look_fail_wg = ~0u;   // (the test hook fails one call's look-back, the first)
    hipLaunchKernelGGL(df_group_kernel, dim3(g), dim3(kBlock), 0, s, a);
    hipLaunchKernelGGL(df_process_kernel, dim3(g), dim3(kBlock), 0, s, a);
    hipLaunchKernelGGL(df_place_kernel, dim3(g), dim3(kBlock), 0, s, a);
    hipLaunchKernelGGL(df_assemble_kernel, dim3(blocks(a.n, kSlotBlock / 64)), dim3(kSlotBlock), 0, s, a);
    return launched(d, "ppe_defrag");
}

int ppe_defrag_age(ppe_defrag_t *d, uint64_t now_seconds, uint64_t timeout_seconds, uint64_t *dropped, uint32_t max,
                   uint32_t *n_dropped, uint32_t *n_freed) {
    if (!d) return PPE_EINVAL;
    if (hipSetDevice(d->device) != hipSuccess) return PPE_ENODEV;
    DfArgs a = d->base;
    a.now = now_seconds;
    a.timeout = timeout_seconds;
    hipLaunchKernelGGL(df_age_kernel, dim3(1), dim3(kScanT), 0, 0, a);
    if (hipDeviceSynchronize() != hipSuccess) return dfail(d, PPE_EIO, "ppe_defrag_age: kernel failed");
    if (hipMemcpy(d->h_ctl, a.ctl, C_WORDS * sizeof(unsigned long long), hipMemcpyDeviceToHost) != hipSuccess)
        return PPE_EIO;
    const uint32_t nd = (uint32_t)d->h_ctl[C_AGE_DROPPED];
    if (n_dropped) *n_dropped = nd;
    if (n_freed) *n_freed = (uint32_t)d->h_ctl[C_AGE_FREED];
    const uint32_t copy = std::min(std::min(nd, max), a.max_dropped);
    if (dropped && copy &&
        hipMemcpy(dropped, a.dropped, copy * sizeof(uint64_t), hipMemcpyDeviceToHost) != hipSuccess)
        return PPE_EIO;
    return PPE_OK;
}

int ppe_defrag_info(ppe_defrag_t *d, ppe_defrag_info_t *info) {
    if (!d || !info) return PPE_EINVAL;
    if (hipSetDevice(d->device) != hipSuccess) return PPE_ENODEV;
    if (hipDeviceSynchronize() != hipSuccess ||
        hipMemcpy(d->h_ctl, d->base.ctl, C_WORDS * sizeof(unsigned long long), hipMemcpyDeviceToHost) != hipSuccess)
        return dfail(d, PPE_EIO, "ppe_defrag_info: device error");
    const unsigned long long *c = d->h_ctl;
    if (c[C_LOOK_ERR]) {   // reported once: cleared, so only this call fails
        const unsigned long long zero = 0;
        (void)hipMemcpy(d->base.ctl + C_LOOK_ERR, &zero, sizeof(zero), hipMemcpyHostToDevice);
        __atomic_store_n(d->h_err, 0ull, __ATOMIC_RELAXED);
        return dfail(d, PPE_EIO, "ppe_defrag_info: %llu admission look-back timeouts (results of those batches wrong)",
                     c[C_LOOK_ERR]);
    }
    memset(info, 0, sizeof(*info));
    info->running = c[C_RUNNING];
    info->new_fcb = c[C_NEW];
    info->del_fcb = c[C_DEL];
    for (int k = 0; k < PPE_DF__COUNT; ++k) info->st[k] = c[C_ST0 + k];
    info->teardrop = c[C_TEARDROP];
    info->timeout_drop = c[C_TIMEOUT_DROP];
    info->datagrams = c[C_DGRAMS];
    info->fcb_max = d->cfg.fcb_max;
    info->cache_max = d->cfg.cache_max;
    info->frag_buf_bytes = d->cfg.frag_buf_bytes;
    info->reasm_buf_bytes = d->cfg.reasm_buf_bytes;
    info->max_batch = d->cfg.max_batch;
    info->slots = d->nslots;
    return PPE_OK;
}

}  // extern "C"
