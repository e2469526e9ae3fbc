/*
 * ppe_engine.hip — host runtime behind the C ABI in include/ppe_hip.h.
 *
 * Owns, per context (one per GPU, like one per-core dataplane instance):
 *   - the double-buffered classifier image (g_acltree_1/2 + running pointer + rwlock-protected swap of
 *     dataplane/src/common/dp_cmd.c:1963-1985): commit writes the back image only after the last launch that
 *     read it has completed (HIP event), then flips `running` — the swap happens at a batch boundary;
 *   - per-workgroup counter slots (the per-core pktstat[] of dataplane/src/decode/decode-statistic.c:4-22);
 *   - HIP-event kernel timing, and the pipelined host-buffer path (H2D → classify → D2H on 3 streams).
 */
#include <hip/hip_runtime.h>
#include <sched.h>

#include <algorithm>
#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "ppe_hip.h"
#include "ppe_image.h"
#include "ppe_internal.h"

namespace {

constexpr int kSlotSets = 4;      // set 0: ppe_classify; 1..3: host pipeline streams
constexpr int kHostStreams = 3;
// ppe_classify_batches: two streams, so a batch's launch ramp-up overlaps the previous batch's tail (C1: 20.6 ->
// 16.5 us per batch; three streams measured 17.0)
constexpr int kPipeStreams = 2;
// tile fetch / walk of the classify kernel (PF_* in ppe_kernels.hip): 0 one tile per wave, its window at the loop
// top; 1 the first tile's loads issued before the image staging (C1 21.7 us vs 22.2); 3 the multi-tile block walk;
// 5 the cut lists (image v8).  Register double-buffering (next tile's window, or only its first 16 B, requested
// before the current tile is processed) and an LDS-DMA next-tile pipeline were measured slower.
constexpr int kPfNone = 0, kPfHoist = 1, kPfMulti = 3, kPfCut = 5;
constexpr uint32_t kMaxBlocksPerCU = 32;  // > resident: the grid then runs in rounds (non-persistent)
// ppe_classify_batches: batches per launch.  0 = every batch of the call in one persistent launch (descriptor ring in
// device memory): the launch ramp and tail are paid once per call instead of once per batch
constexpr uint32_t kBatchesPerLaunch = 0;

struct HostStage {
    hipStream_t s = nullptr;
    uint8_t *hdr = nullptr;
    uint32_t *len = nullptr;
    uint64_t *ts = nullptr;
    uint32_t *verdict = nullptr, *fhash = nullptr, *fw = nullptr, *drop = nullptr, *tcnt = nullptr,
             *tuple = nullptr;
    int32_t *hit = nullptr;
    uint32_t cap = 0, stride = 0;
};

// Per-context staging of the host-pointer ACL lookup (DP_Acl_Lookup, one call per flow miss on the reference's hot
// path, flow.c:232): pinned, device-mapped host memory the lookup kernel reads its tuples from and writes its results
// to across PCIe (no hipMalloc, no copies, no device-wide synchronisation per call), its own stream and a spin wait
// on that stream only.
struct LookupStage {
    hipStream_t s = nullptr;
    uint8_t *h = nullptr;   // host view: tuples (16 B) | macs (16 B) | ts (8 B) | hit (4 B) | action (4 B), per entry
    uint8_t *d = nullptr;   // the same memory as the device sees it
    uint32_t cap = 0;       // entries
};

// Device flow table (ppe_classify_flow) and what the host knows about it without synchronising.
struct FlowArrays {
    uint32_t *keys = nullptr, *creator = nullptr;
    unsigned long long *stats = nullptr, *recs = nullptr;
};
struct FlowTable {
    uint32_t capacity = 0, max_batch = 0, nslots = 0;
    FlowArrays arr[2];  // arr[cur] in use; the other is the rehash target (allocated on first rehash)
    int cur = 0;
    unsigned long long *ctl = nullptr;
    uint32_t *rec = nullptr, *rslot = nullptr, *miss_tiles = nullptr;
    unsigned long long *tile_miss = nullptr, *tile_new = nullptr;
    // owner-computed FlowUpdate (flow_update_wg in ppe_flow_post_kernel): bucket columns for upd_wgs classify workgroups
    unsigned long long *upd = nullptr;
    uint32_t *ucnt = nullptr;
    uint32_t upd_wgs = 0, upd_osh = 0, upd_owners = 0, upd_hmask = PPE_UPD_HASH - 1u;
    uint64_t batches = 0;   // ppe_classify_flow calls (the parity selects the miss-tile counter)
    unsigned long long fold_pkts = PPE_PK_FOLD_PKTS, fold_bytes = PPE_PK_FOLD_BYTES;
    uint64_t live_ub = 0;   // upper bound of live flows: a snapshot's count + n per batch since
    uint64_t tomb_ub = 0;   // upper bound of tombstones: a snapshot's count + n per batch that could revoke
    uint32_t rehashes = 0;
    // zero-copy snapshot of ctl in pinned host memory, written by every flow-mode classify launch (block 0) as it
    // starts: {batches completed, live, tombstones}.  The host tightens its bounds from it without synchronising.
    // refreshes them without synchronising
    unsigned long long *snap_h = nullptr, *snap_d = nullptr;  // host / device views
    uint64_t snap_used = 0;            // highest snapshot sequence applied
    // recorded on the stream right before each batch's classify launch: once it completes, that launch is the next
    // thing the stream runs, and its snapshot follows within microseconds (blocking-sync: the host sleeps on it)
    hipEvent_t pre_launch = nullptr;
    bool use_event = true;
    uint32_t fin_cap = 0;  // finalize workgroups at most (0: one per CU; PPE_FLOW_FIN_WGS, default half the CUs)
    // ring over the last kSnapRing batches: packets submitted before batch b (of batches that may revoke: _rev)
    static constexpr uint32_t kSnapRing = 4096;
    std::vector<uint64_t> cum_n, cum_rev;
    uint64_t tot_n = 0, tot_rev = 0;
    // set when a batch's post-classify launch failed after its classify launch ran: that batch's claims were never
    // finalized (miss-tile counter, snapshot, creators), so every later call on the table fails until
    // ppe_flow_destroy / ppe_flow_create
    bool broken = false;
};

}  // namespace

// A launch that reads an image slot or a descriptor-ring slot, the last one per stream (streams run their launches in
// order): a classify launch is tracked by its sequence number, which its last workgroup publishes to pinned memory
// (ppe_kargs.done_*; no event marker behind the launch: a marker cost the F1 stream 4.5 µs per batch, r6o); other
// launches (ppe_acl_lookup) by an event recorded behind them.
struct Reader {
    hipStream_t s;
    hipEvent_t ev;  // nullptr: tracked by seq
    uint64_t seq;
};
constexpr uint32_t kDoneSlots = 4096;  // launch-completion slots (sequence numbers modulo this)

struct ppe_ctx {
    int device = 0;
    uint32_t n_cu = 256;
    // classifier images
    uint32_t *d_img[2] = {nullptr, nullptr};
    size_t img_cap[2] = {0, 0};
    std::vector<uint32_t> h_img[2];
    std::vector<uint32_t> level_end[2];  // per image: number of tree nodes at depth <= d (BFS order)
    ppe_acl_stats_t stats[2];
    hipEvent_t img_done[2] = {nullptr, nullptr};
    std::vector<Reader> img_readers[2];  // per slot: launch streams, their last launch with it
    hipStream_t aux = nullptr;                 // image uploads
    int running = 0;
    int staged = -1;              // ppe_rules_stage: the slot holding an unpublished image (-1: none)
    uint32_t rule_slots[2] = {0, 0};  // per image: the rule array length it was built from (acl_hit < this)
    uint64_t stage_token = 0, tokens = 0;
    // counters
    unsigned long long *d_cslots = nullptr;
    uint32_t max_grid = 0;
    // timing
    bool timing = false;
    std::vector<hipEvent_t> ev;  // pairs
    size_t ev_used = 0;
    // host pipeline
    HostStage hs[kHostStreams];
    // device-batch pipeline (ppe_classify_batches): consecutive batches alternate over these streams
    hipStream_t pipe[kPipeStreams] = {};
    hipEvent_t pipe_ev[kPipeStreams + 1] = {};
    int pipe_mode = 1;  // PPE_PIPE_MODE at context creation (see ppe_classify_batches)
    // descriptor rings of launches over more than PPE_MAX_BATCH batches: two slots used alternately; a slot is
    // rewritten only after every launch that read it has completed (one event per slot and reading stream, like the
    // image slots); a launch on another stream that reuses a slot's content waits only for its upload (ring_up)
    ppe_bdesc *d_ring[2] = {nullptr, nullptr};
    ppe_bdesc *h_ring[2] = {nullptr, nullptr};  // pinned staging of the H2D descriptor copy
    std::vector<Reader> ring_readers[2];
    // launch completions (struct Reader): pinned words the launches' last workgroups write, device running counts
    volatile unsigned long long *done_h = nullptr;
    unsigned long long *done_hd = nullptr, *done_cnt = nullptr;
    uint64_t done_cum[kDoneSlots] = {};  // per slot: the running workgroup count its next launch completes
    uint64_t launch_seq = 0;
    hipEvent_t ring_up[2] = {nullptr, nullptr};  // behind the slot's last upload, on ring_up_stream
    hipStream_t ring_up_stream[2] = {nullptr, nullptr};
    uint32_t ring_n[2] = {0, 0};       // descriptors the slot holds (its content = h_ring[slot][0, ring_n))
    int ring_next = 0;
    std::vector<ppe_bdesc> ring_tmp;   // descriptors of the launch being built
    ppe_tuning_t tune;
    std::vector<std::pair<uint64_t, uint32_t>> occ_cache;  // resident workgroups per CU by kernel variant
    // batch groups of waves a launch may split into (PPE_GROUPS): more groups = more tiles per wave between batch
    // setups, but more batches streamed at once (DRAM locality); C1, 20-32 batches per launch, per batch: 1 / 2 / 4
    // / 8 / 32 groups 20.2 / 18.7 / 18.3 / 18.3 / 19.1 us (one run, tools/ab_bench.py)
    uint32_t max_groups = 8;
    FlowTable *flow = nullptr;  // ppe_flow_create
    LookupStage lk;             // ppe_acl_lookup_host
    uint32_t *d_steer = nullptr;  // ppe_steer_partition: per-tile owner counts / offsets
    size_t steer_cap = 0;
    char err[256] = {0};
};

namespace {

int fail(ppe_ctx *c, int code, const char *fmt, ...) {
    if (c) {
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(c->err, sizeof c->err, fmt, ap);
        va_end(ap);
    }
    return code;
}

#define HIPCHK(c, expr)                                                                           \
    do {                                                                                          \
        hipError_t e_ = (expr);                                                                   \
        if (e_ != hipSuccess) return fail((c), PPE_EIO, "%s: %s", #expr, hipGetErrorString(e_)); \
    } while (0)

int env_int(const char *name, int dflt) {
    const char *e = getenv(name);
    return e && *e ? atoi(e) : dflt;
}

// Kernel variant knobs live per context (ppe_set_tuning); the defaults are the fastest measured on MI355X
//  and can be overridden by PPE_BLOCK / PPE_BLOCKS_PER_CU / PPE_LDS_IMG.
ppe_tuning_t default_tuning() {
    ppe_tuning_t t;
    const int b = env_int("PPE_BLOCK", 0);
    t.block = (uint32_t)(b == 256 || b == 512 || b == 1024 ? b : 0);  // 0 = chosen per image
    const int bpc = env_int("PPE_BLOCKS_PER_CU", 0);
    t.blocks_per_cu = bpc > 0 && bpc <= (int)kMaxBlocksPerCU ? (uint32_t)bpc : 0u;
    const int pl = env_int("PPE_PIPELINE", 0);
    t.pipeline = pl == 1 || pl == 3 || pl == 4 || pl == 5 ? (uint32_t)pl : 0u;
    t.lds_image = env_int("PPE_LDS_IMG", 1) != 0 ? 1u : 0u;
    t.batches_per_launch = (uint32_t)std::max(0, std::min(env_int("PPE_BATCHES_PER_LAUNCH", (int)kBatchesPerLaunch),
                                                          PPE_MAX_RING));
    return t;
}

// How the classify kernel holds the classifier image (see IMG_* in ppe_kernels.hip) and how it fetches tiles.
struct StagePlan {
    int mode;            // 0 global, 1 whole image in LDS, 2 prefix in LDS
    int pipe;            // tile fetch (kPf*)
    uint32_t block;
    uint32_t lds_words, lds_nodes;  // image words staged from word 0 (single-tile walks: binary nodes)
    uint32_t stage_src, stage_words;  // what the kernel copies into LDS: image words [stage_src, + stage_words)
    uint32_t lds_blocks;              // multi-tile walks: blocks [0, lds_blocks) in LDS
    uint32_t bsec_lds, blk_lds;       // LDS byte offsets (from the image base in LDS) of the block section / block 0
    uint32_t crec_lds = ~0u, idtab_lds = ~0u;  // compact records / index table in LDS (byte offsets), ~0u = global
    uint32_t cut_gbase_lds = 0, cut_fp_lds = 0;    // cut lists: LDS byte offsets of the group bases / fingerprints
    uint32_t cut_ent_lds = ~0u;                    // cut lists: entry lines in LDS (byte offset), ~0u = global
};

// LDS left for the image per workgroup when the CU holds 2048 / block workgroups (32 waves; a flow-table launch:
// the waves per CU its kernel is compiled for): 160 KiB shared, minus the per-wave walk keys and counter bins
// (flow-table launches: and the owner-update buckets), and the 1-KB rounding of the staged image
uint32_t image_budget(uint32_t block, int mode, bool flow = false) {
    const uint32_t waves_cu = flow ? std::min(32u, std::max(block / 64u, 4u * ppe_flow_waves())) : 32u;
    const uint32_t per_wg = (160u * 1024u) / std::max(1u, waves_cu / (block / 64u));
    const uint32_t fixed = ppe_classify_fixed_lds((int)block, kPfHoist, mode) + 1024u + (flow ? ppe_flow_lds_extra() : 0u);
    return per_wg > fixed ? per_wg - fixed : 0u;
}

// single: the plan for the single-tile node-walk kernel only (the flow-table classify kernel is built for it: its
// key slots and node prefix), never the multi-tile or cut-list plans
StagePlan stage_plan(const ppe_ctx *c, const std::vector<uint32_t> &img, bool single = false) {
    const int pf = c->tune.pipeline == 1 ? kPfNone : kPfHoist;
    // the single-tile walk reads the binary nodes only: what it stages "whole" is the image before the block section
    const uint32_t all_words = img[PPE_IMG_W_OFFCUT] ? img[PPE_IMG_W_OFFCUT] : (uint32_t)img.size();  // tree part
    const uint32_t off_bsec = img[PPE_IMG_W_OFFBSEC], off_blocks = img[PPE_IMG_W_OFFBLOCKS];
    const uint32_t n_blocks = img[PPE_IMG_W_NBLOCKS];
    const uint32_t words = off_bsec, bytes = words * 4u;
    StagePlan p = {0, pf, c->tune.block ? c->tune.block : 1024u, 0, 0, 0, 0, 0, 0, 0};
    // the multi-tile walk reads the 2-level blocks: whole image in LDS, else the block jump table and the first
    // block levels (breadth-first), else global
    const uint32_t off_crec = img[PPE_IMG_W_OFFCREC], off_idtab = img[PPE_IMG_W_OFFIDTAB];
    constexpr uint32_t bbytes = 32u;
    auto mt_plan = [&](uint32_t budget) {
        const uint32_t bjt = 4u * (off_blocks - off_bsec);
        if (off_crec && (all_words - off_bsec) * 4u <= budget) {
            // compact image (v6): the block walk needs only the block section and the compact records after it, so
            // the whole walk is LDS-resident when they fit (C2 / C4: 4,096 rules, ~140 KB)
            p.mode = 1;
            p.stage_src = off_bsec;
            p.lds_words = p.stage_words = all_words - off_bsec;
            p.lds_blocks = n_blocks;
            p.bsec_lds = 0;
            p.blk_lds = 4u * (off_blocks - off_bsec);
            p.crec_lds = 4u * (off_crec - off_bsec);
            if (off_idtab) p.idtab_lds = 4u * (off_idtab - off_bsec);
        } else if (!off_crec && all_words * 4u <= budget) {
            p.mode = 1;
            p.lds_words = p.stage_words = all_words;
            p.lds_blocks = n_blocks;
            p.bsec_lds = 4u * off_bsec;
            p.blk_lds = 4u * off_blocks;
        } else if (budget >= bjt + bbytes * 64u) {
            p.mode = 2;
            p.lds_blocks = std::min(n_blocks, (budget - bjt) / bbytes);
            p.stage_src = off_bsec;
            p.stage_words = (off_blocks - off_bsec) + (bbytes / 4u) * p.lds_blocks;
            p.bsec_lds = 0;
            p.blk_lds = bjt;
        }
    };
    // the cut lists (image v8): the bucket groups in LDS (the smallest workgroup whose share at 32 waves per CU holds
    // them; the entries too when they fit beside them), the entries read from L2 otherwise; one tile per wave at 8
    // waves per SIMD.  lds_image = 0: both from global memory.
    const uint32_t off_cut = img[PPE_IMG_W_OFFCUT];
    auto cut_plan = [&]() {
        const uint32_t *h = img.data() + off_cut;
        const uint32_t grp_bytes = 4u * (h[5] - h[4]);  // slices, bases and fingerprints (the L2-entry plan's LDS)
        const uint32_t all_words = h[5] - h[4] + 32u * h[11] +  // ... to the end of the entry lines (and the ids)
                                   (h[0] & PPE_CUT_LINES ? 0u : h[0] & PPE_CUT_IDS16 ? (h[2] + 1u) / 2u : h[2]);
        p.pipe = kPfCut;
        p.mode = 0;
        p.block = c->tune.block ? c->tune.block : 1024u;
        if (!c->tune.lds_image) return;
        auto budget = [&](uint32_t b) {  // (no key slots: the keys stay in registers)
            const uint32_t per_wg = (160u * 1024u) / std::max(1u, 32u / (b / 64u));
            const uint32_t fixed = ppe_classify_fixed_lds((int)b, kPfCut, 1) + 1024u;
            return per_wg > fixed ? per_wg - fixed : 0u;
        };
        if (!c->tune.block)
            for (uint32_t b : {256u, 512u, 1024u})
                if (4u * all_words <= budget(b) || (b == 1024u && grp_bytes <= budget(b))) {
                    p.block = b;
                    break;
                }
        const uint32_t bud = budget(p.block);
        if (grp_bytes > bud) return;  // (groups larger than the share: global)
        p.stage_src = h[4];
        p.cut_gbase_lds = 4u * (h[8] - h[4]);
        p.cut_fp_lds = 4u * (h[9] - h[4]);
        // everything in LDS (IMG_LDS: the dense layout only, the kernel's entry addressing assumes it)
        if (4u * all_words <= bud && !(h[0] & PPE_CUT_LINES) && env_int("PPE_CUT_ENT_LDS", 1)) {
            p.mode = 1;
            p.stage_words = all_words;
            p.cut_ent_lds = 4u * (h[5] - h[4]);
        } else {  // slices, bases and fingerprints in LDS, the entry lines from L2 (IMG_SPLIT)
            p.mode = 2;
            p.stage_words = h[5] - h[4];
        }
        p.lds_words = p.stage_words;
    };
    if (!single && off_cut && c->tune.pipeline == 5) {
        cut_plan();
        return p;
    }
    if (!c->tune.lds_image) {
        if (!c->tune.block) p.block = 256;
        if (!single && (c->tune.pipeline == 3 || (c->tune.pipeline == 0 && !c->tune.block))) {  // PF_MULTI, global image
            p.pipe = kPfMulti;
            p.block = 1024u;
        }
        return p;
    }
    // the whole image in LDS: the smallest workgroup (most copies per CU) whose share holds it (a node walk reads
    // the part before the block section)
    const uint32_t lds_bytes = bytes;
    if (!c->tune.block) {
        for (uint32_t b : {256u, 512u, 1024u}) {
            if (lds_bytes <= image_budget(b, 1, single)) {
                p.block = b;
                break;
            }
        }
    }
    uint32_t budget = image_budget(p.block, 1, single);
    const bool fits = lds_bytes <= budget;
    // images that do not fit whole: the cut lists when the image has them (C2 / C3 / C4), else PF_MULTI
    // (1024-thread workgroups, one per CU, with the CU's whole LDS for the image prefix: C2 / C3 / C4 step 27.2 /
    // 52.1 / 27.3 -> 23.6 / 42.8 / 22.7 us against the single-tile node walk)
    if (!single && off_cut && c->tune.pipeline == 0 && !fits && !c->tune.block && env_int("PPE_CUT_PLAN", 1)) {
        cut_plan();
        return p;
    }
    if (!single && (c->tune.pipeline == 3 || (c->tune.pipeline == 0 && !fits && !c->tune.block))) {
        p.pipe = kPfMulti;
        // tuning knobs (A/B only): workgroup size and the LDS bytes each workgroup may take (default: all of it, one
        // workgroup per CU); less LDS lets more workgroups share a CU
        const int mb = env_int("PPE_MT_BLOCK", 1024);
        p.block = (mb == 256 || mb == 512) ? (uint32_t)mb : 1024u;
        const uint32_t fixed = ppe_classify_fixed_lds((int)p.block, kPfMulti, 2) + 1024u;  // no key slots
        const uint32_t cap = (uint32_t)std::min(160 * 1024, std::max(8 * 1024, env_int("PPE_MT_LDS", 160 * 1024)));
        budget = cap > fixed ? cap - fixed : 0u;
        mt_plan(budget);
        return p;
    }
    const uint32_t off_resid = img[PPE_IMG_W_OFFRESID], off_rules = img[PPE_IMG_W_OFFRULES];
    const uint32_t n_nodes = img[PPE_IMG_W_NNODES], off_nodes = img[PPE_IMG_W_OFFNODES];
    if (fits) {
        p.mode = 1;
        p.lds_words = p.stage_words = words;
        return p;
    }
    budget = image_budget(p.block, 2, single);  // node walks of a partly staged image keep their key slots
    if (off_resid * 4u <= budget) {  // nodes, leaf lists and rule records; residual records from global
        p.mode = 2;
        p.lds_words = off_resid;
        p.lds_nodes = n_nodes;
    } else if (off_rules * 4u <= budget) {  // every node and leaf list; rule records from global (L2)
        p.mode = 2;
        p.lds_words = off_rules;
        p.lds_nodes = n_nodes;
    } else if (budget >= 4u * (off_nodes + PPE_NODE_WORDS * 64u)) {  // header, jump table, top of the BFS forest
        p.mode = 2;
        p.lds_nodes = std::min(n_nodes, (budget / 4u - off_nodes) / PPE_NODE_WORDS);
        p.lds_words = off_nodes + PPE_NODE_WORDS * p.lds_nodes;
    }
    p.stage_words = p.lds_words;  // single-tile walks stage a prefix from word 0
    return p;
}

// Resident workgroups per CU: the occupancy API's answer (register and LDS limits) unless the tuning fixes it.
// The persistent grid is CUs × this, so no workgroup waits for a second round.
uint32_t blocks_per_cu(ppe_ctx *c, const StagePlan &p, bool flow = false) {
    const uint32_t cap = kMaxBlocksPerCU * 256u / p.block;
    if (c->tune.blocks_per_cu) return std::max(1u, std::min(c->tune.blocks_per_cu, cap));  // may exceed residency
    // the occupancy query costs microseconds of host time per call: cached per kernel variant and LDS size (a
    // flow-table launch: the flow variant's own occupancy, so its grid is resident in one round and each workgroup's
    // owner-update buckets hold as many entries as it can)
    const uint64_t key = (uint64_t)p.stage_words | ((uint64_t)p.mode << 32) | ((uint64_t)p.pipe << 40) |
                         ((uint64_t)p.block << 48) | ((uint64_t)(flow ? 1u : 0u) << 63);
    for (const auto &e : c->occ_cache)
        if (e.first == key) return e.second;
    const int occ = flow ? ppe_classify_occupancy_flow(p.stage_words, p.mode, (int)p.block)
                         : ppe_classify_occupancy(p.stage_words, p.mode, p.pipe, (int)p.block);
    const uint32_t r = occ > 0 ? std::min<uint32_t>((uint32_t)occ, cap) : 1u;
    c->occ_cache.emplace_back(key, r);
    return r;
}

// A launch on stream s reads slot r of an image or descriptor ring: an event (one per slot and stream) is recorded
// behind it, so a rewrite of the slot waits for exactly the launches that read it (the event outlives the stream if
// the caller frees it).  Events of other streams whose launches have completed are dropped once the list grows, so a
// caller that uses a new stream per call does not make the list (and every later rewrite's wait) grow without bound.
// ---- readers of image / descriptor-ring slots (struct Reader) --------------------------------------------------------
static bool launch_done(const ppe_ctx *c, uint64_t seq) { return c->done_h[seq % kDoneSlots] >= seq; }

// a tracked launch's completion: the pinned word its last workgroup writes, polled (the core yielded between polls,
// as for the flow snapshot), bounded; past the bound the device is synchronised and the word read once more
static int wait_launch(ppe_ctx *c, uint64_t seq) {
    const auto until = std::chrono::steady_clock::now() + std::chrono::seconds(30);
    while (!launch_done(c, seq)) {
        if (std::chrono::steady_clock::now() > until) {
            HIPCHK(c, hipDeviceSynchronize());
            if (!launch_done(c, seq)) return fail(c, PPE_EIO, "launch %llu never reported its completion", (unsigned long long)seq);
            break;
        }
        sched_yield();
    }
    return PPE_OK;
}
static bool reader_done(const ppe_ctx *c, const Reader &x) {
    return x.ev ? hipEventQuery(x.ev) == hipSuccess : launch_done(c, x.seq);
}
static int wait_reader(ppe_ctx *c, Reader &x) {
    if (!x.ev) return wait_launch(c, x.seq);   // (an entry with an event: its event is behind any seq it had)
    HIPCHK(c, hipEventSynchronize(x.ev));
    return PPE_OK;
}
static void drop_readers(std::vector<Reader> &v) {
    for (auto &x : v)
        if (x.ev) (void)hipEventDestroy(x.ev);
    v.clear();
}
// stream s's entry (created empty), after pruning other streams' completed ones
static Reader &reader_of(const ppe_ctx *c, std::vector<Reader> &readers, hipStream_t s) {
    constexpr size_t kPruneAt = 8;
    if (readers.size() >= kPruneAt) {
        size_t k = 0;
        for (size_t i = 0; i < readers.size(); ++i) {
            Reader &x = readers[i];
            if (x.s != s && reader_done(c, x)) {
                if (x.ev) (void)hipEventDestroy(x.ev);
                continue;
            }
            readers[k++] = x;
        }
        readers.resize(k);
    }
    for (auto &x : readers)
        if (x.s == s) return x;
    readers.push_back(Reader{s, nullptr, 0});
    return readers.back();
}
// a tracked classify launch (sequence number seq) read the slot on stream s: it completes after every earlier launch
// on s, so it replaces their entry
static void note_launch_reader(ppe_ctx *c, std::vector<Reader> &readers, hipStream_t s, uint64_t seq) {
    Reader &x = reader_of(c, readers, s);
    if (x.ev) (void)hipEventDestroy(x.ev);
    x.ev = nullptr;
    x.seq = seq;
}
// an untracked launch read the slot on stream s: an event behind it
int note_reader(ppe_ctx *c, std::vector<Reader> &readers, hipStream_t s) {
    Reader &x = reader_of(c, readers, s);
    if (!x.ev) HIPCHK(c, hipEventCreateWithFlags(&x.ev, hipEventDisableTiming));
    HIPCHK(c, hipEventRecord(x.ev, s));
    return PPE_OK;
}
int note_image_reader(ppe_ctx *c, int r, hipStream_t s) { return note_reader(c, c->img_readers[r], s); }

// the next tracked launch's sequence number and completion slot, in its kernel arguments (the slot's previous launch,
// kDoneSlots launches ago, has completed: at most one launch per slot in flight)
static int track_launch(ppe_ctx *c, uint32_t grid, ppe_kargs &a) {
    const uint64_t seq = c->launch_seq + 1u;
    const uint32_t q = (uint32_t)(seq % kDoneSlots);
    if (seq > kDoneSlots) {
        const int rc = wait_launch(c, seq - kDoneSlots);
        if (rc != PPE_OK) return rc;
    }
    c->launch_seq = seq;
    c->done_cum[q] += grid;
    a.done_cnt = c->done_cnt + q;
    a.done_host = c->done_hd + q;
    a.done_target = c->done_cum[q];
    a.done_seq = seq;
    return PPE_OK;
}
// the launch did not start: its slot is completed by hand (its workgroups will never count)
static void untrack_launch(ppe_ctx *c, uint32_t grid, const ppe_kargs &a) {
    const uint32_t q = (uint32_t)(a.done_seq % kDoneSlots);
    c->done_cum[q] -= grid;
    c->done_h[q] = a.done_seq;
}

int upload_image(ppe_ctx *c, int slot, uint32_t *words, uint32_t n_words, const ppe_acl_stats_t *st) {
    // The back image may still be read by launches queued before the previous swap.  Wait for exactly those (the
    // events recorded behind them, note_image_reader): unrelated work on any stream is never waited on.
    for (auto &x : c->img_readers[slot]) {
        const int rc = wait_reader(c, x);
        if (rc != PPE_OK) return rc;
    }
    drop_readers(c->img_readers[slot]);
    if (!c->aux) HIPCHK(c, hipStreamCreateWithFlags(&c->aux, hipStreamNonBlocking));
    const size_t bytes = (size_t)n_words * 4u;
    if (bytes > c->img_cap[slot]) {
        // (grown with headroom: a growing rule set reallocates rarely; the free of an unused slot is then safe)
        const size_t cap = std::max(bytes + bytes / 2, (size_t)64 * 1024);
        if (c->d_img[slot]) HIPCHK(c, hipFree(c->d_img[slot]));
        c->d_img[slot] = nullptr;
        HIPCHK(c, hipMalloc(&c->d_img[slot], cap + 64));
        c->img_cap[slot] = cap;
    }
    // the copy runs on the engine's own non-blocking stream: no implicit synchronisation with other streams
    HIPCHK(c, hipMemcpyAsync(c->d_img[slot], words, bytes, hipMemcpyHostToDevice, c->aux));
    HIPCHK(c, hipStreamSynchronize(c->aux));
    c->h_img[slot].assign(words, words + n_words);
    // BFS node order: the nodes of depth <= d are exactly [0, level_end[d])
    {
        std::vector<uint32_t> &le = c->level_end[slot];
        le.clear();
        const uint32_t nn = words[PPE_IMG_W_NNODES], on = words[PPE_IMG_W_OFFNODES];
        std::vector<uint8_t> depth(nn, 0);  // every root of the forest (jump root: several) has depth 0
        for (uint32_t k = 0; k < nn; ++k) {
            const uint32_t *nd = words + on + PPE_NODE_WORDS * k;
            if (nd[0] != PPE_LEAF_THR) {  // children: byte offsets from the image start
                depth[(nd[1] / 4u - on) / PPE_NODE_WORDS] = (uint8_t)(depth[k] + 1u);
                depth[(nd[2] / 4u - on) / PPE_NODE_WORDS] = (uint8_t)(depth[k] + 1u);
            }
            if (le.size() <= depth[k]) le.resize(depth[k] + 1u, 0u);
            le[depth[k]] = k + 1u;
        }
    }
    c->stats[slot] = *st;
    c->stats[slot].lds_resident = (uint32_t)stage_plan(c, c->h_img[slot]).mode;
    return PPE_OK;
}

// One launch over batches in[0..nb) (nb <= PPE_MAX_BATCH, each n > 0): every wave takes its tiles of batch 0, then
// of batch 1, ... (no barrier between batches, one image staging for all of them).
int launch(ppe_ctx *c, const ppe_batch_t *in, const ppe_result_t *out, uint32_t nb, const ppe_cfg_t *cfg,
           hipStream_t s, int slot_set, uint32_t idx_base = 0, const ppe_flowdev *fl = nullptr,
           uint32_t *grid_out = nullptr) {
    const int r = c->running;
    const uint32_t words = (uint32_t)c->h_img[r].size();
    const StagePlan plan = stage_plan(c, c->h_img[r], fl != nullptr);
    const uint32_t wpb = plan.block / 64u;
    ppe_kargs a;
    std::memset(&a, 0, sizeof a);
    uint32_t tiles = 0;
    uint64_t tiles_total = 0;
    bool part = true;  // the throughput layout in every batch (ppe_kargs.part_layout)
    const bool use_ring = nb > PPE_MAX_BATCH;
    int rslot = 0;
    std::vector<ppe_bdesc> &rd = c->ring_tmp;
    if (use_ring) {
        if (nb > PPE_MAX_RING) return fail(c, PPE_EINVAL, "more than %d batches in one launch", PPE_MAX_RING);
        rd.resize(nb);
    }
    for (uint32_t i = 0; i < nb; ++i) {
        ppe_bdesc &d = use_ring ? rd[i] : a.batch[i];
        d.hdr = in[i].hdr;
        d.len = in[i].len;
        d.ts = in[i].ts;
        d.n = in[i].n;
        d.stride = in[i].stride;
        d.verdict = out[i].verdict;
        d.fhash = out[i].flow_hash;
        d.hit = out[i].acl_hit;
        d.fw_idx = out[i].fw_idx;
        d.drop_idx = out[i].drop_idx;
        d.tile_cnt = out[i].tile_cnt;
        d.tuple = out[i].tuple;
        d.idx_base = idx_base;
        d.flags = 0;
        if (out[i].part8) {
            if (d.fw_idx || d.drop_idx || d.tile_cnt)
                return fail(c, PPE_EINVAL, "part8 replaces fw_idx / drop_idx / tile_cnt (pass them NULL)");
            d.tile_cnt = (uint32_t *)out[i].part8;  // (the kernel reads the compact list from the tile_cnt field)
            d.flags = PPE_BD_PART8;
        }
        if (out[i].packed) {
            if (d.verdict || d.fhash || d.hit)
                return fail(c, PPE_EINVAL, "packed replaces verdict / flow_hash / acl_hit (pass them NULL)");
            if (fl) return fail(c, PPE_EINVAL, "the packed result layout is for ppe_classify / ppe_classify_batches");
            if (c->rule_slots[r] > PPE_PACKED_MAX_RULES)
                return fail(c, PPE_EINVAL, "packed results hold rule indices below %u (classifier of %u rule slots)",
                            PPE_PACKED_MAX_RULES, c->rule_slots[r]);
            d.verdict = (uint32_t *)out[i].packed;  // (the kernel writes the 8-B words through the verdict field)
            d.flags |= PPE_BD_PACKED;
        }
        part = part && ((d.verdict && d.fhash && d.hit) || (d.flags & PPE_BD_PACKED)) && !d.tuple &&
               ((d.fw_idx && d.fw_idx == d.drop_idx && !d.tile_cnt) || (d.flags & PPE_BD_PART8));
        tiles = std::max(tiles, (in[i].n + 63u) / 64u);
        tiles_total += (uint64_t)((in[i].n + 63u) / 64u);
    }
    bool ring_copy = false;
    if (use_ring) {
        // a slot already holding exactly these descriptors is reused as is (a dataplane cycling over a fixed set of
        // batch buffers uploads its descriptor table once); otherwise the next slot is rewritten once the launch
        // that last read it (two ring launches ago) has completed
        const size_t bytes = sizeof(ppe_bdesc) * nb;
        rslot = -1;
        for (int k = 0; k < 2; ++k)
            if (c->ring_n[k] == nb && c->h_ring[k] && std::memcmp(c->h_ring[k], rd.data(), bytes) == 0) rslot = k;
        if (rslot < 0) {
            rslot = c->ring_next;
            c->ring_next ^= 1;
            for (auto &x : c->ring_readers[rslot]) {  // its last readers
                const int rc = wait_reader(c, x);
                if (rc != PPE_OK) return rc;
            }
            drop_readers(c->ring_readers[rslot]);
            std::memcpy(c->h_ring[rslot], rd.data(), bytes);
            c->ring_n[rslot] = nb;
            HIPCHK(c, hipMemcpyAsync(c->d_ring[rslot], c->h_ring[rslot], bytes, hipMemcpyHostToDevice, s));
            HIPCHK(c, hipEventRecord(c->ring_up[rslot], s));
            c->ring_up_stream[rslot] = s;
            ring_copy = true;
        }
        if (!ring_copy && c->ring_up_stream[rslot] != s && hipEventQuery(c->ring_up[rslot]) != hipSuccess)
            HIPCHK(c, hipStreamWaitEvent(s, c->ring_up[rslot], 0));  // reused on another stream: after the upload only
        a.batch[0] = rd[0];
        a.ring = c->d_ring[rslot];
    }
    a.nbatch = nb;
    a.part_layout = (part && !fl && !env_int("PPE_NO_PART", 0)) ? 1u : 0u;
    a.max_tiles = tiles;
    // enough workgroups for every tile of every batch (the kernel splits its waves into batch groups), at most
    // the resident grid
    const uint32_t want = (uint32_t)std::min<uint64_t>((tiles_total + wpb - 1) / wpb, 1u << 30);
    const uint32_t maxg = c->n_cu * blocks_per_cu(c, plan, fl != nullptr);
    const uint32_t grid = std::max(1u, std::min(want, std::min(maxg, c->max_grid)));
    a.img = c->d_img[r];
    a.img_words = words;
    a.unsup_fw = cfg ? cfg->unsupport_proto_action : 0u;
    a.syn_check = cfg ? cfg->syn_check : 1u;
    a.now = cfg ? cfg->now_seconds : 0u;
    a.default_action = c->h_img[r][PPE_IMG_W_DEFACT];
    a.lds_words = plan.lds_words;
    a.stage_src = plan.stage_src;
    a.stage_words = plan.stage_words;
    a.lds_blocks = plan.lds_blocks;
    a.bsec_lds = plan.bsec_lds;
    a.blk_lds = plan.blk_lds;
    a.off_bsec = c->h_img[r][PPE_IMG_W_OFFBSEC];
    a.off_blocks = c->h_img[r][PPE_IMG_W_OFFBLOCKS];
    a.max_bdepth = c->h_img[r][PPE_IMG_W_MAXBDEPTH];
    a.off_crec = c->h_img[r][PPE_IMG_W_OFFCREC];
    a.off_idtab = c->h_img[r][PPE_IMG_W_OFFIDTAB];
    a.crec_lds = plan.crec_lds;
    a.idtab_lds = plan.idtab_lds;
    if (plan.pipe == kPfCut) {  // (image v8 cut lists: header at PPE_IMG_W_OFFCUT)
        const uint32_t *h = c->h_img[r].data() + c->h_img[r][PPE_IMG_W_OFFCUT];
        a.cut = h[0];
        a.cut_slc = h[4];
        a.cut_ent = h[5];
        a.cut_epl = h[7];
        a.cut_div = h[10];
        a.cut_idrel = (h[0] & PPE_CUT_LINES) ? 0u : 4u * (h[12] - h[5]);
        a.cut_gbase = h[8];
        a.cut_fp = h[9];
        a.cut_gbase_lds = plan.cut_gbase_lds;
        a.cut_fp_lds = plan.cut_fp_lds;
        a.cut_ent_lds = plan.cut_ent_lds;
    }
    // batch groups: the kernel splits its waves into min(batches, max_groups) groups, group g taking batches g, g + G,
    // ...; when G does not divide the batch count the last round leaves groups idle (20 batches at G = 8: the last
    // 4 run on half the grid; C3 / C4 ring step +12 %, profiles/r3_ab_runs.md r4l).  Take the power-of-two G up to the
    // cap (or the batch count itself when smaller) with the least work-slot time, ceil(batches / G) x G batch slots
    // weighted by the per-batch cost of G groups (1 group 1.10, 2 groups 1.02, more 1.00: C1 per-batch 20.2 / 18.7 /
    // 18.3 us at 1 / 2 / >= 4 groups); ties go to the larger G.  20 batches -> 4 groups, 32 -> 8, 33 -> 2.
    {
        const uint32_t gmax = std::max(1u, std::min(c->max_groups, nb));
        auto cost = [&](uint32_t g) {
            return (double)((nb + g - 1u) / g * g) * (g == 1u ? 1.10 : g == 2u ? 1.02 : 1.0);
        };
        uint32_t best = gmax;
        double cbest = cost(gmax);
        for (uint32_t g = 1u << (31 - __builtin_clz(gmax)); g >= 1u; g >>= 1) {
            if (g == gmax) continue;
            if (cost(g) < cbest - 1e-9) {
                best = g;
                cbest = cost(g);
            }
        }
        a.max_groups = best;
    }
    a.max_depth = c->h_img[r][PPE_IMG_W_MAXDEPTH];
    a.max_leaf = c->h_img[r][PPE_IMG_W_MAXLEAF];
    a.root_ks = c->h_img[r][PPE_IMG_W_ROOTKS];
    a.jump = c->h_img[r][PPE_IMG_W_JUMP];
    a.off_nodes = c->h_img[r][PPE_IMG_W_OFFNODES];
    if (plan.mode == 1) {
        a.lds_iters = a.max_depth + 1u;
    } else if (plan.mode == 2) {  // node reads 0..L-1 only visit depths < L: all inside the staged prefix
        const std::vector<uint32_t> &le = c->level_end[r];
        uint32_t L = 0;
        while (L < le.size() && le[L] <= plan.lds_nodes) ++L;
        a.lds_iters = std::min(L, a.max_depth + 1u);
    }
    a.off_leaf = c->h_img[r][PPE_IMG_W_OFFLEAF];
    a.off_rules = c->h_img[r][PPE_IMG_W_OFFRULES];
    a.off_resid = c->h_img[r][PPE_IMG_W_OFFRESID];
    a.cslots = c->d_cslots + (size_t)slot_set * c->max_grid * PPE_CSLOT_WORDS;
    if (fl) a.flow = *fl;
    if (grid_out) *grid_out = grid;

    hipEvent_t e0 = nullptr, e1 = nullptr;
    {
        const int rc0 = track_launch(c, grid, a);
        if (rc0 != PPE_OK) return rc0;
    }
    if (c->timing) {
        if (c->ev_used + 2 > c->ev.size()) {
            for (int i = 0; i < 256; ++i) {
                hipEvent_t e;
                HIPCHK(c, hipEventCreate(&e));
                c->ev.push_back(e);
            }
        }
        e0 = c->ev[c->ev_used];
        e1 = c->ev[c->ev_used + 1];
        c->ev_used += 2;
    }
    const int rc =
        ppe_launch_classify(&a, grid, plan.mode, plan.pipe, (int)plan.block, fl != nullptr, (void *)s, (void *)e0,
                            (void *)e1);
    if (rc != 0) {
        untrack_launch(c, grid, a);
        return fail(c, PPE_EIO, "kernel launch failed: %s", hipGetErrorString((hipError_t)rc));
    }
    // the launch reads its image slot (and ring slot): a later rewrite waits for its completion
    if (use_ring) note_launch_reader(c, c->ring_readers[rslot], s, a.done_seq);
    note_launch_reader(c, c->img_readers[r], s, a.done_seq);
    return PPE_OK;
}

hipError_t use_device(ppe_ctx *c) {
    int cur = -1;
    if (hipGetDevice(&cur) == hipSuccess && cur == c->device) return hipSuccess;
    return hipSetDevice(c->device);
}

int check_batch(ppe_ctx *c, const ppe_batch_t *in, const ppe_cfg_t *cfg) {
    if (!in) return fail(c, PPE_EINVAL, "null batch");
    if (in->n == 0) return PPE_OK;
    if (!in->hdr || !in->len) return fail(c, PPE_EINVAL, "hdr/len required");
    if (in->stride < 64 || in->stride > 256 || in->stride % 16u)
        return fail(c, PPE_EINVAL, "stride must be a multiple of 16 from 64 to 256");
    // byte offsets inside the kernel are 32-bit, and partition-list entries keep the action in bits 31:30
    if ((uint64_t)in->n * in->stride >= (1ull << 31)) return fail(c, PPE_EINVAL, "batch too large (n * stride >= 2^31)");
    if (((uintptr_t)in->hdr & 15u) != 0) return fail(c, PPE_EINVAL, "hdr must be 16-byte aligned");
    if (cfg && cfg->unsupport_proto_action > 1) return fail(c, PPE_EINVAL, "unsupport_proto_action must be 0/1");
    if (cfg && cfg->syn_check > 1) return fail(c, PPE_EINVAL, "syn_check must be 0/1");
    return PPE_OK;
}

}  // namespace

extern "C" {

int ppe_abi_version(void) { return PPE_ABI_VERSION; }

const char *ppe_last_error(ppe_ctx_t *ctx) { return ctx ? ctx->err : "null context"; }

int ppe_ctx_create(int device, ppe_ctx_t **out) {
    if (!out) return PPE_EINVAL;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return PPE_ENODEV;
    if (device < 0 || device >= ndev) return PPE_ENODEV;
    ppe_ctx *c = new (std::nothrow) ppe_ctx();
    if (!c) return PPE_ENOMEM;
    c->device = device;
    if (hipSetDevice(device) != hipSuccess) {
        delete c;
        return PPE_ENODEV;
    }
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0)
        c->n_cu = (uint32_t)prop.multiProcessorCount;
    c->max_grid = c->n_cu * kMaxBlocksPerCU;
    c->tune = default_tuning();
    c->max_groups = (uint32_t)std::max(1, env_int("PPE_GROUPS", 8));
    c->pipe_mode = env_int("PPE_PIPE_MODE", 1);
    const size_t cs_bytes = (size_t)kSlotSets * c->max_grid * PPE_CSLOT_WORDS * sizeof(unsigned long long);
    int rc = PPE_OK;
    if (hipMalloc(&c->d_cslots, cs_bytes) != hipSuccess || hipMemset(c->d_cslots, 0, cs_bytes) != hipSuccess)
        rc = PPE_ENOMEM;
    for (int i = 0; i < 2 && rc == PPE_OK; ++i)
        if (hipEventCreateWithFlags(&c->img_done[i], hipEventDisableTiming) != hipSuccess) rc = PPE_EIO;
    // launch completions (struct Reader): pinned, device-mapped words and the device running counts
    if (rc == PPE_OK) {
        void *h = nullptr;
        if (hipHostMalloc(&h, kDoneSlots * 8u, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
            hipHostGetDevicePointer((void **)&c->done_hd, h, 0) != hipSuccess ||
            hipMalloc(&c->done_cnt, kDoneSlots * 8u) != hipSuccess || hipMemset(c->done_cnt, 0, kDoneSlots * 8u) != hipSuccess)
            rc = PPE_ENOMEM;
        c->done_h = (volatile unsigned long long *)h;
        if (h) std::memset(h, 0, kDoneSlots * 8u);
    }
    // descriptor ring slots (launches over more than PPE_MAX_BATCH batches): allocated here, not on first use, so
    // no batch call pays an allocation
    for (int i = 0; i < 2 && rc == PPE_OK; ++i)
        if (hipMalloc(&c->d_ring[i], sizeof(ppe_bdesc) * PPE_MAX_RING) != hipSuccess ||
            hipHostMalloc(&c->h_ring[i], sizeof(ppe_bdesc) * PPE_MAX_RING, hipHostMallocDefault) != hipSuccess ||
            hipEventCreateWithFlags(&c->ring_up[i], hipEventDisableTiming) != hipSuccess)
            rc = PPE_ENOMEM;
    if (rc == PPE_OK) {
        // empty rule set, management default action DROP (mgrplane/src/srv/srvnet/srv_rule.c:84)
        rc = ppe_rules_commit(c, nullptr, nullptr, 0, ACL_RULE_ACTION_DROP, nullptr);
    }
    if (rc != PPE_OK) {
        ppe_ctx_destroy(c);
        return rc;
    }
    *out = c;
    return PPE_OK;
}

int ppe_ctx_destroy(ppe_ctx_t *c) {
    if (!c) return PPE_EINVAL;
    (void)hipSetDevice(c->device);
    (void)hipDeviceSynchronize();
    for (int i = 0; i < 2; ++i) {
        if (c->d_img[i]) (void)hipFree(c->d_img[i]);
        if (c->img_done[i]) (void)hipEventDestroy(c->img_done[i]);
    }
    if (c->d_cslots) (void)hipFree(c->d_cslots);
    for (hipEvent_t e : c->ev) (void)hipEventDestroy(e);
    for (int i = 0; i < 2; ++i) {
        if (c->d_ring[i]) (void)hipFree(c->d_ring[i]);
        if (c->h_ring[i]) (void)hipHostFree(c->h_ring[i]);
        if (c->ring_up[i]) (void)hipEventDestroy(c->ring_up[i]);
        drop_readers(c->ring_readers[i]);
    }
    for (hipStream_t s : c->pipe)
        if (s) (void)hipStreamDestroy(s);
    if (c->aux) (void)hipStreamDestroy(c->aux);
    for (auto &v : c->img_readers) drop_readers(v);
    if (c->done_h) (void)hipHostFree((void *)c->done_h);
    if (c->done_cnt) (void)hipFree(c->done_cnt);
    for (hipEvent_t e : c->pipe_ev)
        if (e) (void)hipEventDestroy(e);
    if (c->flow) ppe_flow_destroy(c);
    if (c->lk.s) (void)hipStreamDestroy(c->lk.s);
    if (c->lk.h) (void)hipHostFree(c->lk.h);
    if (c->d_steer) (void)hipFree(c->d_steer);
    for (auto &h : c->hs) {
        if (h.s) (void)hipStreamDestroy(h.s);
        (void)hipFree(h.hdr);
        (void)hipFree(h.len);
        (void)hipFree(h.ts);
        (void)hipFree(h.verdict);
        (void)hipFree(h.fhash);
        (void)hipFree(h.hit);
        (void)hipFree(h.fw);
        (void)hipFree(h.drop);
        (void)hipFree(h.tcnt);
        (void)hipFree(h.tuple);
    }
    delete c;
    return PPE_OK;
}

int ppe_ctx_device(ppe_ctx_t *c) { return c ? c->device : PPE_EINVAL; }

int ppe_rules_stage(ppe_ctx_t *c, const RCP_BLOCK_ACL_RULE_TUPLE *rules, const uint8_t *used, uint32_t n,
                    uint32_t default_action, ppe_acl_stats_t *stats, uint64_t *token) {
    if (!c) return PPE_EINVAL;
    if (default_action > 0xffffu) return fail(c, PPE_EINVAL, "default action out of range");
    HIPCHK(c, hipSetDevice(c->device));
    uint32_t *words = nullptr, n_words = 0;
    ppe_acl_stats_t st;
    const char *bt = getenv("PPE_BINTH");
    const uint32_t binth = bt ? (uint32_t)atoi(bt) : 0u;
    int rc = ppe_acl_build_image(rules, used, n, default_action, binth, &words, &n_words, &st);
    if (rc != PPE_OK) return fail(c, rc, "classifier build failed (%d)", rc);
    // the back slot (the context's creation commits an image, so the running slot is never empty after it)
    const int back = c->h_img[c->running].empty() ? c->running : 1 - c->running;
    c->staged = -1;  // (an unpublished image there is replaced: its token no longer publishes)
    rc = upload_image(c, back, words, n_words, &st);
    ppe_acl_free_image(words);
    if (rc != PPE_OK) return rc;
    c->staged = back;
    c->rule_slots[back] = n;
    c->stage_token = ++c->tokens;
    if (token) *token = c->stage_token;
    if (stats) *stats = c->stats[back];
    return PPE_OK;
}

int ppe_rules_publish(ppe_ctx_t *c, uint64_t token) {
    if (!c) return PPE_EINVAL;
    if (token == 0 || c->staged < 0 || token != c->stage_token)
        return fail(c, PPE_EINVAL, "no staged classifier with token %llu", (unsigned long long)token);
    c->running = c->staged;  // later launches read the new image (set_running_acltree, dp_cmd.c:1980-1985)
    c->staged = -1;
    return PPE_OK;
}

int ppe_rules_commit(ppe_ctx_t *c, const RCP_BLOCK_ACL_RULE_TUPLE *rules, const uint8_t *used, uint32_t n,
                     uint32_t default_action, ppe_acl_stats_t *stats) {
    uint64_t token = 0;
    const int rc = ppe_rules_stage(c, rules, used, n, default_action, stats, &token);
    return rc != PPE_OK ? rc : ppe_rules_publish(c, token);
}

int ppe_classify(ppe_ctx_t *c, const ppe_batch_t *in, const ppe_result_t *out, const ppe_cfg_t *cfg,
                 void *stream) {
    if (!c || !out) return PPE_EINVAL;
    int rc = check_batch(c, in, cfg);
    if (rc != PPE_OK || in->n == 0) return rc;
    HIPCHK(c, use_device(c));
    return launch(c, in, out, 1, cfg, (hipStream_t)stream, 0);
}

int ppe_classify_batches(ppe_ctx_t *c, const ppe_batch_t *in, const ppe_result_t *out, uint32_t nbatch,
                         const ppe_cfg_t *cfg, void *stream) {
    if (!c || (nbatch && (!in || !out))) return PPE_EINVAL;
    for (uint32_t i = 0; i < nbatch; ++i) {
        const int rc = check_batch(c, &in[i], cfg);
        if (rc != PPE_OK) return rc;
    }
    if (nbatch == 0) return PPE_OK;
    HIPCHK(c, use_device(c));
    const hipStream_t s = (hipStream_t)stream;
    const int mode = c->pipe_mode;
    const uint32_t per = c->tune.batches_per_launch ? std::min<uint32_t>(c->tune.batches_per_launch, PPE_MAX_RING)
                                                    : (uint32_t)PPE_MAX_RING;
    uint32_t nonempty = 0;
    for (uint32_t i = 0; i < nbatch; ++i) nonempty += in[i].n != 0;
    if (nonempty == 0) return PPE_OK;
    if (nonempty <= per) {  // one launch: straight onto the caller's stream, no fork / join
        std::vector<ppe_batch_t> gin;
        std::vector<ppe_result_t> gout;
        gin.reserve(nonempty);
        gout.reserve(nonempty);
        for (uint32_t i = 0; i < nbatch; ++i)
            if (in[i].n) {
                gin.push_back(in[i]);
                gout.push_back(out[i]);
            }
        return launch(c, gin.data(), gout.data(), nonempty, cfg, s, 0);
    }
    if (!c->pipe[0]) {
        for (int k = 0; k < kPipeStreams; ++k)
            HIPCHK(c, hipStreamCreateWithFlags(&c->pipe[k], mode == 2 ? hipStreamDefault : hipStreamNonBlocking));
        for (hipEvent_t &e : c->pipe_ev) HIPCHK(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
    }
    // mode 1: the caller's stream carries the even batches and one engine stream the odd ones; else two engine
    // streams.  fork: the engine streams start after the work already queued on `stream`
    hipStream_t q[kPipeStreams];
    for (int k = 0; k < kPipeStreams; ++k) q[k] = (mode == 1 && k == 0) ? s : c->pipe[k];
    HIPCHK(c, hipEventRecord(c->pipe_ev[kPipeStreams], s));
    for (int k = 0; k < kPipeStreams; ++k)
        if (q[k] != s) HIPCHK(c, hipStreamWaitEvent(q[k], c->pipe_ev[kPipeStreams], 0));
    // groups of up to PPE_MAX_BATCH non-empty batches per launch, launches alternating over the streams
    std::vector<ppe_batch_t> gin(std::min<uint32_t>(nbatch, PPE_MAX_RING));
    std::vector<ppe_result_t> gout(gin.size());
    uint32_t ng = 0, nl = 0;
    for (uint32_t i = 0; i <= nbatch; ++i) {
        if (i < nbatch && in[i].n == 0) continue;
        if (i < nbatch) {
            gin[ng] = in[i];
            gout[ng] = out[i];
            ++ng;
        }
        if (ng == per || (i == nbatch && ng)) {
            const int rc = launch(c, gin.data(), gout.data(), ng, cfg, q[nl % kPipeStreams], 0);
            if (rc != PPE_OK) return rc;
            ng = 0;
            ++nl;
        }
    }
    // join: `stream` continues after every batch
    for (int k = 0; k < kPipeStreams; ++k) {
        if (q[k] == s) continue;
        HIPCHK(c, hipEventRecord(c->pipe_ev[k], q[k]));
        HIPCHK(c, hipStreamWaitEvent(s, c->pipe_ev[k], 0));
    }
    return PPE_OK;
}

// device address of a pinned, device-mapped host buffer (hipHostMalloc / registered / torch pin_memory), or nullptr
static const void *mapped_host(const void *p) {
    if (!p) return nullptr;
    hipPointerAttribute_t at;
    if (hipPointerGetAttributes(&at, p) != hipSuccess) {
        (void)hipGetLastError();  // pageable memory: not an error for the caller
        return nullptr;
    }
    if (at.type != hipMemoryTypeHost || !at.devicePointer) return nullptr;
    return (const char *)at.devicePointer + ((const char *)p - (const char *)at.hostPointer);
}

int ppe_classify_host(ppe_ctx_t *c, const ppe_batch_t *in, const ppe_result_t *out, const ppe_cfg_t *cfg,
                      uint32_t chunk) {
    if (!c || !out) return PPE_EINVAL;
    int rc = check_batch(c, in, cfg);
    if (rc != PPE_OK || in->n == 0) return rc;
    HIPCHK(c, hipSetDevice(c->device));
    // Zero-copy: when every buffer is pinned and device-mapped, the kernel reads the windows and writes the results
    // across PCIe itself (C1: 822 vs 628 Mpps for the staged copies below, tools/host_zero_copy.py)
    if (env_int("PPE_HOST_ZEROCOPY", 1)) {
        ppe_batch_t b = *in;
        ppe_result_t r = *out;
        bool ok = (b.hdr = (const uint8_t *)mapped_host(in->hdr)) && (b.len = (const uint32_t *)mapped_host(in->len));
        if (in->ts) ok = ok && (b.ts = (const uint64_t *)mapped_host(in->ts));
        uint32_t **outs[] = {&r.verdict, &r.flow_hash, (uint32_t **)&r.acl_hit, &r.fw_idx, &r.drop_idx, &r.tile_cnt,
                             &r.tuple, (uint32_t **)&r.part8, (uint32_t **)&r.packed};
        for (uint32_t **o : outs)
            if (ok && *o) ok = (*o = (uint32_t *)mapped_host(*o)) != nullptr;
        if (ok) {
            rc = launch(c, &b, &r, 1, cfg, nullptr, 0);
            if (rc != PPE_OK) return rc;
            HIPCHK(c, hipStreamSynchronize(nullptr));
            return PPE_OK;
        }
    }
    if (out->packed && out->tuple)  // (the staged path keeps the packed words in the tuple's staging buffer)
        return fail(c, PPE_EINVAL, "ppe_classify_host: packed with tuple needs device-mapped host buffers");
    if (chunk == 0) chunk = 1u << 18;
    chunk = (chunk + 63u) & ~63u;
    chunk = std::min(chunk, (in->n + 63u) & ~63u);
    for (auto &h : c->hs) {
        if (!h.s) HIPCHK(c, hipStreamCreateWithFlags(&h.s, hipStreamNonBlocking));
        if (h.cap < chunk || h.stride != in->stride) {
            (void)hipFree(h.hdr); (void)hipFree(h.len); (void)hipFree(h.ts); (void)hipFree(h.verdict); (void)hipFree(h.fhash);
            (void)hipFree(h.hit); (void)hipFree(h.fw); (void)hipFree(h.drop); (void)hipFree(h.tcnt); (void)hipFree(h.tuple);
            h = HostStage{h.s};
            HIPCHK(c, hipMalloc(&h.hdr, (size_t)chunk * in->stride));
            HIPCHK(c, hipMalloc(&h.len, (size_t)chunk * 4));
            HIPCHK(c, hipMalloc(&h.ts, (size_t)chunk * 8));
            HIPCHK(c, hipMalloc(&h.verdict, (size_t)chunk * 4));
            HIPCHK(c, hipMalloc(&h.fhash, (size_t)chunk * 4));
            HIPCHK(c, hipMalloc(&h.hit, (size_t)chunk * 4));
            HIPCHK(c, hipMalloc(&h.fw, (size_t)chunk * 4));
            HIPCHK(c, hipMalloc(&h.drop, (size_t)chunk * 4));
            HIPCHK(c, hipMalloc(&h.tcnt, (size_t)(chunk / 64) * 4));
            HIPCHK(c, hipMalloc(&h.tuple, (size_t)chunk * 16));
            h.cap = chunk;
            h.stride = in->stride;
        }
    }
    const hipMemcpyKind h2d = hipMemcpyHostToDevice, d2h = hipMemcpyDeviceToHost;
    for (uint32_t base = 0, i = 0; base < in->n; base += chunk, ++i) {
        HostStage &h = c->hs[i % kHostStreams];
        const uint32_t m = std::min(chunk, in->n - base);
        HIPCHK(c, hipMemcpyAsync(h.hdr, in->hdr + (size_t)base * in->stride, (size_t)m * in->stride, h2d, h.s));
        HIPCHK(c, hipMemcpyAsync(h.len, in->len + base, (size_t)m * 4, h2d, h.s));
        if (in->ts) HIPCHK(c, hipMemcpyAsync(h.ts, in->ts + base, (size_t)m * 8, h2d, h.s));
        ppe_batch_t b = {h.hdr, h.len, in->ts ? h.ts : nullptr, m, in->stride};
        ppe_result_t r;
        r.verdict = out->verdict ? h.verdict : nullptr;
        r.flow_hash = out->flow_hash ? h.fhash : nullptr;
        r.acl_hit = out->acl_hit ? h.hit : nullptr;
        const bool part = out->fw_idx && out->fw_idx == out->drop_idx;  // partition layout: one list
        r.fw_idx = out->fw_idx ? h.fw : nullptr;
        r.drop_idx = part ? h.fw : (out->drop_idx ? h.drop : nullptr);
        r.tile_cnt = out->tile_cnt ? h.tcnt : nullptr;
        r.tuple = out->tuple ? h.tuple : nullptr;
        r.part8 = out->part8 ? (uint8_t *)h.fw : nullptr;  // (part8 excludes fw_idx: the staging list is free)
        r.packed = out->packed ? (uint64_t *)h.tuple : nullptr;
        rc = launch(c, &b, &r, 1, cfg, h.s, 1 + (int)(i % kHostStreams), base);
        if (rc != PPE_OK) return rc;
        if (out->verdict) HIPCHK(c, hipMemcpyAsync(out->verdict + base, h.verdict, (size_t)m * 4, d2h, h.s));
        if (out->flow_hash) HIPCHK(c, hipMemcpyAsync(out->flow_hash + base, h.fhash, (size_t)m * 4, d2h, h.s));
        if (out->acl_hit) HIPCHK(c, hipMemcpyAsync(out->acl_hit + base, h.hit, (size_t)m * 4, d2h, h.s));
        if (out->tuple) HIPCHK(c, hipMemcpyAsync(out->tuple + (size_t)base * 4, h.tuple, (size_t)m * 16, d2h, h.s));
        if (out->tile_cnt)
            HIPCHK(c, hipMemcpyAsync(out->tile_cnt + base / 64, h.tcnt, (size_t)((m + 63) / 64) * 4, d2h, h.s));
        // compacted indices carry the batch index (idx_base); chunk is a multiple of 64, so tiles line up
        if (out->fw_idx) HIPCHK(c, hipMemcpyAsync(out->fw_idx + base, h.fw, (size_t)m * 4, d2h, h.s));
        if (out->drop_idx && !part)
            HIPCHK(c, hipMemcpyAsync(out->drop_idx + base, h.drop, (size_t)m * 4, d2h, h.s));
        if (out->part8) HIPCHK(c, hipMemcpyAsync(out->part8 + base, h.fw, (size_t)m, d2h, h.s));
        if (out->packed) HIPCHK(c, hipMemcpyAsync(out->packed + base, h.tuple, (size_t)m * 8, d2h, h.s));
    }
    for (auto &h : c->hs) HIPCHK(c, hipStreamSynchronize(h.s));
    return PPE_OK;
}

int ppe_acl_lookup(ppe_ctx_t *c, const ppe_tuples_t *in, int32_t *hit, uint32_t *action, uint64_t now_seconds,
                   void *stream) {
    if (!c || !in) return PPE_EINVAL;
    if (in->n == 0) return PPE_OK;
    if (!in->tuple) return fail(c, PPE_EINVAL, "tuple required");
    HIPCHK(c, hipSetDevice(c->device));
    const int r = c->running;
    const uint32_t words = c->h_img[r][PPE_IMG_W_OFFBSEC];  // the binary walk's part of the image (no blocks)
    // staging the image into each workgroup's LDS pays off over many tuples; a few (one flow miss's lookup) walk it
    // from L2 / HBM in one workgroup
    const bool lds = (size_t)words * 4u + 1024u <= PPE_LDS_IMG_MAX && in->n >= 4096u;
    ppe_tuple_kargs a;
    std::memset(&a, 0, sizeof a);
    a.tuple = in->tuple;
    a.macs = in->macs;
    a.ts = in->ts;
    a.n = in->n;
    a.hit = hit;
    a.action = action;
    a.img = c->d_img[r];
    a.img_words = words;
    a.default_action = c->h_img[r][PPE_IMG_W_DEFACT];
    a.now = now_seconds;
    const uint32_t want = (in->n + PPE_BLOCK - 1) / PPE_BLOCK;
    const uint32_t grid = std::max(1u, std::min(want, c->n_cu * 8u));
    const int rc = ppe_launch_acl_tuples(&a, grid, lds ? 1 : 0, stream);
    if (rc != 0) return fail(c, PPE_EIO, "acl kernel launch failed: %s", hipGetErrorString((hipError_t)rc));
    return note_image_reader(c, r, (hipStream_t)stream);
}

int ppe_acl_lookup_host(ppe_ctx_t *c, const ppe_tuples_t *in, int32_t *hit, uint32_t *action,
                        uint64_t now_seconds) {
    if (!c || !in) return PPE_EINVAL;
    if (in->n == 0) return PPE_OK;
    if (!in->tuple) return fail(c, PPE_EINVAL, "tuple required");
    HIPCHK(c, use_device(c));
    LookupStage &L = c->lk;
    // the staging holds at most kLookupChunk entries (192 KB pinned per context, allocated by the first call); a
    // larger burst goes through it in chunks of that size
    constexpr uint32_t kLookupChunk = 4096;
    if (!L.s) HIPCHK(c, hipStreamCreateWithFlags(&L.s, hipStreamNonBlocking));
    if (!L.h) {
        HIPCHK(c, hipHostMalloc((void **)&L.h, (size_t)kLookupChunk * 48u, hipHostMallocMapped));
        HIPCHK(c, hipHostGetDevicePointer((void **)&L.d, L.h, 0));
        L.cap = kLookupChunk;
    }
    const size_t cap = L.cap;
    uint8_t *ht = L.h, *hm = L.h + cap * 16, *hts = L.h + cap * 32, *hh = L.h + cap * 40, *ha = L.h + cap * 44;
    for (uint32_t b = 0; b < in->n; b += (uint32_t)cap) {
        const size_t n = std::min<size_t>(cap, in->n - b);
        std::memcpy(ht, in->tuple + 4u * b, n * 16);
        if (in->macs) std::memcpy(hm, in->macs + 4u * b, n * 16);
        if (in->ts) std::memcpy(hts, in->ts + b, n * 8);
        uint8_t *d = L.d;
        ppe_tuples_t dv = {(const uint32_t *)d, in->macs ? (const uint32_t *)(d + cap * 16) : nullptr,
                           in->ts ? (const uint64_t *)(d + cap * 32) : nullptr, (uint32_t)n};
        int rc = ppe_acl_lookup(c, &dv, (int32_t *)(d + cap * 40), (uint32_t *)(d + cap * 44), now_seconds, L.s);
        if (rc != PPE_OK) return rc;
        // spin on this stream alone (a lookup is a few microseconds; a blocking wait would add the wake-up), then
        // block
        hipError_t q = hipErrorNotReady;
        const auto until = std::chrono::steady_clock::now() + std::chrono::milliseconds(2);
        while ((q = hipStreamQuery(L.s)) == hipErrorNotReady && std::chrono::steady_clock::now() < until)
            __builtin_ia32_pause();
        if (q == hipErrorNotReady) q = hipStreamSynchronize(L.s);
        if (q != hipSuccess) return fail(c, PPE_EIO, "acl lookup kernel failed: %s", hipGetErrorString(q));
        if (hit) std::memcpy(hit + b, hh, n * 4);
        if (action) std::memcpy(action + b, ha, n * 4);
    }
    return PPE_OK;
}

void *ppe_dev_alloc(ppe_ctx_t *c, size_t bytes) {
    void *p = nullptr;
    if (!c || hipSetDevice(c->device) != hipSuccess) return nullptr;
    if (hipMalloc(&p, bytes ? bytes : 1) != hipSuccess) return nullptr;
    return p;
}
void ppe_dev_free(ppe_ctx_t *c, void *p) {
    if (c && p && hipSetDevice(c->device) == hipSuccess) (void)hipFree(p);
}
void *ppe_host_alloc(ppe_ctx_t *c, size_t bytes) {
    void *p = nullptr;
    if (!c || hipSetDevice(c->device) != hipSuccess) return nullptr;
    if (hipHostMalloc(&p, bytes ? bytes : 1, hipHostMallocDefault) != hipSuccess) return nullptr;
    return p;
}
void ppe_host_free(ppe_ctx_t *c, void *p) {
    if (c && p) (void)hipHostFree(p);
}
int ppe_memcpy_h2d(ppe_ctx_t *c, void *dst, const void *src, size_t bytes) {
    if (!c) return PPE_EINVAL;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice));
    return PPE_OK;
}
int ppe_memcpy_d2h(ppe_ctx_t *c, void *dst, const void *src, size_t bytes) {
    if (!c) return PPE_EINVAL;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost));
    return PPE_OK;
}
int ppe_memset_d(ppe_ctx_t *c, void *dst, int value, size_t bytes) {
    if (!c) return PPE_EINVAL;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipMemset(dst, value, bytes));
    return PPE_OK;
}
int ppe_sync(ppe_ctx_t *c) {
    if (!c) return PPE_EINVAL;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipDeviceSynchronize());
    return PPE_OK;
}

int ppe_counters_read(ppe_ctx_t *c, ppe_counters_t *out) {
    if (!c || !out) return PPE_EINVAL;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipDeviceSynchronize());
    const size_t words = (size_t)kSlotSets * c->max_grid * PPE_CSLOT_WORDS;
    std::vector<unsigned long long> h(words);
    HIPCHK(c, hipMemcpy(h.data(), c->d_cslots, words * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    std::memset(out, 0, sizeof *out);
    for (size_t b = 0; b < (size_t)kSlotSets * c->max_grid; ++b)
        for (int i = 0; i < PPE_CSLOT_WORDS; ++i) out->c[i] += h[b * PPE_CSLOT_WORDS + i];
    return PPE_OK;
}

int ppe_counters_clear(ppe_ctx_t *c) {
    if (!c) return PPE_EINVAL;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipDeviceSynchronize());
    HIPCHK(c, hipMemset(c->d_cslots, 0,
                        (size_t)kSlotSets * c->max_grid * PPE_CSLOT_WORDS * sizeof(unsigned long long)));
    return PPE_OK;
}

int ppe_timing_enable(ppe_ctx_t *c, int on) {
    if (!c) return PPE_EINVAL;
    c->timing = on != 0;
    return PPE_OK;
}

int ppe_timing_read(ppe_ctx_t *c, double *total_ms, uint32_t *launches, int reset) {
    if (!c) return PPE_EINVAL;
    HIPCHK(c, hipSetDevice(c->device));
    double t = 0;
    for (size_t i = 0; i + 1 < c->ev_used; i += 2) {
        HIPCHK(c, hipEventSynchronize(c->ev[i + 1]));
        float ms = 0;
        HIPCHK(c, hipEventElapsedTime(&ms, c->ev[i], c->ev[i + 1]));
        t += ms;
    }
    if (total_ms) *total_ms = t;
    if (launches) *launches = (uint32_t)(c->ev_used / 2);
    if (reset) c->ev_used = 0;
    return PPE_OK;
}

int ppe_set_tuning(ppe_ctx_t *c, const ppe_tuning_t *t) {
    if (!c || !t) return PPE_EINVAL;
    if (t->block != 0 && t->block != 256 && t->block != 512 && t->block != 1024)
        return fail(c, PPE_EINVAL, "block must be 0 (auto), 256, 512 or 1024");
    if (t->pipeline != 0 && t->pipeline != 1 && t->pipeline != 3 && t->pipeline != 4 && t->pipeline != 5)
        return fail(c, PPE_EINVAL, "pipeline must be 0 (auto), 1 (first tile at the loop top), 3 (4 tiles per wave "
                                   "walking the block section together), 4 (first tile's loads before the image "
                                   "staging) or 5 (the cut lists of a v8 image)");
    if (t->blocks_per_cu > kMaxBlocksPerCU) return fail(c, PPE_EINVAL, "blocks_per_cu must be <= 32");
    if (t->batches_per_launch > PPE_MAX_RING) return fail(c, PPE_EINVAL, "batches_per_launch must be <= 4096");
    c->tune = *t;
    c->tune.pipeline = t->pipeline;
    c->tune.lds_image = t->lds_image ? 1u : 0u;
    return PPE_OK;
}

int ppe_get_tuning(ppe_ctx_t *c, ppe_tuning_t *t) {
    if (!c || !t) return PPE_EINVAL;
    *t = c->tune;
    return PPE_OK;
}

int ppe_acl_image(ppe_ctx_t *c, uint32_t *words, uint32_t *n_words) {
    if (!c || !n_words) return PPE_EINVAL;
    const std::vector<uint32_t> &img = c->h_img[c->running];
    if (words) std::memcpy(words, img.data(), std::min<size_t>(*n_words, img.size()) * 4u);
    *n_words = (uint32_t)img.size();
    return PPE_OK;
}

int ppe_launch_info(ppe_ctx_t *c, uint32_t *grid, uint32_t *block, uint32_t *lds_bytes, uint32_t *variant) {
    if (!c) return PPE_EINVAL;
    const StagePlan plan = stage_plan(c, c->h_img[c->running]);
    if (grid) *grid = std::min(c->n_cu * blocks_per_cu(c, plan), c->max_grid);
    if (block) *block = plan.block;
    if (lds_bytes)
        *lds_bytes = ppe_classify_fixed_lds((int)plan.block, plan.pipe, plan.mode) +
                     (plan.mode ? ((plan.stage_words * 4u + 1023u) & ~1023u) : 0u);
    if (variant) *variant = (uint32_t)plan.mode | ((uint32_t)plan.pipe << 4);
    return PPE_OK;
}

// ---------------------------------------------------------------------------------------------------------------
// Flow table (FlowInit / FlowHandlePacket / FlowAgeTimeoutCB / FlowRelease, dataplane/src/flow/flow.c)

static void flow_free_arrays(FlowArrays &a) {
    (void)hipFree(a.keys);
    (void)hipFree(a.creator);
    (void)hipFree(a.stats);
    (void)hipFree(a.recs);
    a = FlowArrays();
}

// allocate (if needed) and clear one slot-array set: every slot EMPTY with zero counters, no creator
static int flow_clear_arrays(ppe_ctx *c, FlowArrays &a, uint32_t nslots, hipStream_t s) {
    if (!a.keys) {
        if (hipMalloc(&a.keys, (size_t)nslots * 4u * PPE_FLOW_SLOT_WORDS) != hipSuccess ||
            hipMalloc(&a.recs, (size_t)nslots * 8u * PPE_FLOW_REC_WORDS) != hipSuccess ||
            hipMalloc(&a.creator, (size_t)nslots * 4u) != hipSuccess ||
            hipMalloc(&a.stats, (size_t)nslots * 32u) != hipSuccess) {
            flow_free_arrays(a);
            return fail(c, PPE_ENOMEM, "flow table: out of device memory (%u slots)", nslots);
        }
    }
    HIPCHK(c, hipMemsetAsync(a.keys, 0, (size_t)nslots * 4u * PPE_FLOW_SLOT_WORDS, s));
    HIPCHK(c, hipMemsetAsync(a.recs, 0, (size_t)nslots * 8u * PPE_FLOW_REC_WORDS, s));
    HIPCHK(c, hipMemsetAsync(a.creator, 0xff, (size_t)nslots * 4u, s));
    HIPCHK(c, hipMemsetAsync(a.stats, 0, (size_t)nslots * 32u, s));
    return PPE_OK;
}

static ppe_flowdev flow_dev(const FlowTable &t, int which) {
    ppe_flowdev d;
    std::memset(&d, 0, sizeof d);
    const FlowArrays &a = t.arr[which];
    d.keys = a.keys;
    d.stats = a.stats;
    d.packed = a.recs;
    d.miss_tiles = t.miss_tiles;
    d.parity = (uint32_t)(t.batches & 1u);
    d.fold_pkts = t.fold_pkts;
    d.fold_bytes = t.fold_bytes;
    d.snap = t.snap_d;
    d.seq = t.batches;
    d.creator = a.creator;
    d.ctl = t.ctl;
    d.rec = t.rec;
    d.tile_miss = t.tile_miss;
    d.tile_new = t.tile_new;
    d.rslot = t.rslot;
    d.gmask = t.nslots / PPE_FLOW_GROUP - 1u;
    d.capacity = t.capacity;
    d.upd = t.upd;
    d.ucnt = t.ucnt;
    d.upd_wgs = t.upd_wgs;
    d.upd_osh = t.upd_osh;
    d.upd_owners = t.upd_owners;
    d.upd_hmask = t.upd_hmask;
    return d;
}

static uint32_t flow_grid(const ppe_ctx *c, uint64_t items, uint32_t per_wg) {
    const uint64_t want = (items + per_wg - 1u) / per_wg;
    return (uint32_t)std::max<uint64_t>(1u, std::min<uint64_t>(want, (uint64_t)c->n_cu * 8u));
}

// exact live / tombstone counts (synchronises)
// Tighten the host's live / tombstone bounds from the latest snapshot the classify launches publish in pinned memory
// (seqlock: the sequence word is written last and re-read here).
static void flow_apply_snapshot(FlowTable &t) {
    const volatile unsigned long long *sh = t.snap_h;
    const uint64_t s0 = sh[0], live = sh[1], tombs = sh[2], s1 = sh[0];
    if (s0 == s1 && s0 > t.snap_used && s0 <= t.batches && t.batches - s0 < FlowTable::kSnapRing) {
        t.snap_used = s0;
        t.live_ub = std::min<uint64_t>(live + (t.tot_n - t.cum_n[s0 % FlowTable::kSnapRing]), t.capacity);
        t.tomb_ub = tombs + (t.tot_rev - t.cum_rev[s0 % FlowTable::kSnapRing]);
    }
}

static int flow_sync_counts(ppe_ctx *c, unsigned long long *ctl_out) {
    FlowTable &t = *c->flow;
    HIPCHK(c, hipDeviceSynchronize());
    HIPCHK(c, hipMemcpy(ctl_out, t.ctl, PPE_FCTL_WORDS * 8u, hipMemcpyDeviceToHost));
    if (ctl_out[PPE_FCTL_ERR]) {
        // reported once: the word is cleared, so only this call fails (the batches it covers may be inexact; the
        // table itself stays usable)
        HIPCHK(c, hipMemset(t.ctl + PPE_FCTL_ERR, 0, 8u));
        HIPCHK(c, hipDeviceSynchronize());
        return fail(c, PPE_EIO, "flow table: %llu finalize workgroup(s) timed out waiting for the revoke", ctl_out[PPE_FCTL_ERR]);
    }
    t.live_ub = ctl_out[PPE_FCTL_LIVE];
    t.tomb_ub = ctl_out[PPE_FCTL_TOMBS];
    t.snap_used = t.batches;  // (the device is idle: this is the state after every submitted batch)
    return PPE_OK;
}

// Rebuild the table without tombstones when they exceed a quarter of the slots (keeps every probe sequence short
// and an EMPTY slot on each).  Synchronises when the host bound says it may be needed.
static int flow_maybe_rehash(ppe_ctx *c) {
    FlowTable &t = *c->flow;
    if (t.tomb_ub <= t.nslots / 4u) return PPE_OK;
    unsigned long long ctl[PPE_FCTL_WORDS];
    int rc = flow_sync_counts(c, ctl);
    if (rc != PPE_OK || t.tomb_ub <= t.nslots / 4u) return rc;
    const int dst = 1 - t.cur;
    rc = flow_clear_arrays(c, t.arr[dst], t.nslots, nullptr);
    if (rc != PPE_OK) return rc;
    ppe_flow_kargs k;
    std::memset(&k, 0, sizeof k);
    k.f = flow_dev(t, t.cur);
    k.dst = flow_dev(t, dst);
    k.nslots = t.nslots;
    rc = ppe_launch_flow(PPE_FLOW_K_REHASH, &k, flow_grid(c, t.nslots, 256u), nullptr);
    if (rc != 0) return fail(c, PPE_EIO, "flow rehash launch failed: %s", hipGetErrorString((hipError_t)rc));
    HIPCHK(c, hipMemset(t.ctl + PPE_FCTL_TOMBS, 0, 8u));
    HIPCHK(c, hipDeviceSynchronize());
    t.cur = dst;
    t.tomb_ub = 0;
    ++t.rehashes;
    return PPE_OK;
}

// Test hook (tests/test_gpu_flow.py only, not in the public headers): the next `k` post-classify launches of
// ppe_classify_flow fail as a launch error would, after the batch's classify launch has run.
static uint32_t g_fail_post = 0;
extern "C" void ppe_flow_debug_fail_post(uint32_t k) { __atomic_store_n(&g_fail_post, k, __ATOMIC_RELAXED); }
static bool take_fail_post() {
    uint32_t k = __atomic_load_n(&g_fail_post, __ATOMIC_RELAXED);
    while (k)
        if (__atomic_compare_exchange_n(&g_fail_post, &k, k - 1, false, __ATOMIC_RELAXED, __ATOMIC_RELAXED)) return true;
    return false;
}

// the table exists and no batch was left half-done by a failed post-classify launch
static int flow_usable(ppe_ctx *c) {
    if (!c->flow) return fail(c, PPE_EINVAL, "no flow table (ppe_flow_create)");
    if (c->flow->broken)
        return fail(c, PPE_EIO, "flow table unusable: a batch's post-classify launch failed (ppe_flow_destroy it)");
    return PPE_OK;
}

int ppe_flow_destroy(ppe_ctx_t *c) {
    if (!c) return PPE_EINVAL;
    if (!c->flow) return PPE_OK;
    (void)hipSetDevice(c->device);
    (void)hipDeviceSynchronize();
    FlowTable *t = c->flow;
    for (FlowArrays &a : t->arr) flow_free_arrays(a);
    if (t->snap_h) (void)hipHostFree(t->snap_h);
    if (t->pre_launch) (void)hipEventDestroy(t->pre_launch);
    (void)hipFree(t->ctl);
    (void)hipFree(t->rec);
    (void)hipFree(t->rslot);
    (void)hipFree(t->miss_tiles);
    (void)hipFree(t->tile_miss);
    (void)hipFree(t->tile_new);
    (void)hipFree(t->upd);
    (void)hipFree(t->ucnt);
    delete t;
    c->flow = nullptr;
    return PPE_OK;
}

int ppe_flow_create(ppe_ctx_t *c, uint32_t capacity, uint32_t max_batch) {
    if (!c) return PPE_EINVAL;
    if (capacity == 0) capacity = 100000u;  // MEM_POOL_FLOW_NODE_NUM, dataplane/src/platform/mem_pool.h:72
    if (max_batch == 0) max_batch = 1u << 20;
    if (capacity > (1u << 26) || max_batch > (1u << 26))
        return fail(c, PPE_EINVAL, "flow table: capacity and max_batch must be <= 2^26");
    HIPCHK(c, hipSetDevice(c->device));
    ppe_flow_destroy(c);
    FlowTable *t = new (std::nothrow) FlowTable();
    if (!t) return PPE_ENOMEM;
    c->flow = t;
    t->capacity = capacity;
    t->max_batch = max_batch;
    t->use_event = env_int("PPE_FLOW_EVENT", 0) != 0;
    // finalize on half the CUs: the update workgroups (one per CU by their LDS) start on the other half at once
    // (F1 batch 67.1 -> 66.3 µs against one per CU, 69.3 / 71.9 at 64 / 32: profiles/r5_ab_runs.md r5aq)
    t->fin_cap = (uint32_t)std::max(0, env_int("PPE_FLOW_FIN_WGS", (int)std::max(1u, c->n_cu / 2u)));
    // test hook: lower fold thresholds so the fold path runs on small inputs (values <= the defaults only)
    const int fp = env_int("PPE_FLOW_FOLD_PKTS", 0), fb = env_int("PPE_FLOW_FOLD_BYTES", 0);
    if (fp > 0 && (unsigned long long)fp < t->fold_pkts) t->fold_pkts = (unsigned long long)fp;
    if (fb > 0 && (unsigned long long)fb < t->fold_bytes) t->fold_bytes = (unsigned long long)fb;
    // load <= 1/2 with the pool full and a whole batch of claims pending; tombstones are rehashed away at 1/4
    uint32_t ns = 64;
    while ((uint64_t)ns < 2ull * ((uint64_t)capacity + max_batch)) ns <<= 1;
    t->nslots = ns;
    const uint32_t tiles = (max_batch + 63u) / 64u;
    int rc = PPE_OK;
    if (hipMalloc(&t->ctl, PPE_FCTL_WORDS * 8u) != hipSuccess || hipMalloc(&t->rec, (size_t)max_batch * 16u) != hipSuccess ||
        hipMalloc(&t->rslot, (size_t)max_batch * 4u) != hipSuccess ||
        hipMalloc(&t->miss_tiles, (size_t)tiles * 4u) != hipSuccess ||
        hipMalloc(&t->tile_miss, (size_t)tiles * 8u) != hipSuccess ||
        hipMalloc(&t->tile_new, (size_t)tiles * 8u) != hipSuccess)
        rc = fail(c, PPE_ENOMEM, "flow table: out of device memory");
    if (rc == PPE_OK && hipMemset(t->ctl, 0, PPE_FCTL_WORDS * 8u) != hipSuccess) rc = fail(c, PPE_EIO, "memset");
    // owner-computed FlowUpdate: one bucket column per classify workgroup of a flow launch (at most 8 per CU and one
    // per 4 tiles of the largest batch; a workgroup past the columns updates its found flows by atomics);
    // PPE_FLOW_OWNER=0 turns it off (A/B)
    if (rc == PPE_OK && env_int("PPE_FLOW_OWNER", 1) != 0) {
        uint32_t owners = std::min<uint32_t>(PPE_UPD_OWNERS, ns), osh = 0;
        while ((ns >> osh) > owners) ++osh;
        t->upd_osh = osh;
        t->upd_owners = ns >> osh;
        t->upd_wgs = std::max(1u, std::min(c->n_cu * 8u, (tiles + 3u) / 4u));
        // test hook: a smaller LDS hash, so the update kernel's full-hash path runs on small inputs (power of two)
        const int hl = env_int("PPE_FLOW_UPD_HASH", 0);
        if (hl > 0 && hl < (int)PPE_UPD_HASH && (hl & (hl - 1)) == 0) t->upd_hmask = (uint32_t)hl - 1u;
        if (hipMalloc(&t->upd, (size_t)t->upd_owners * t->upd_wgs * PPE_UPD_CAP * 8u) != hipSuccess ||
            hipMalloc(&t->ucnt, (size_t)t->upd_owners * t->upd_wgs * 4u) != hipSuccess)
            rc = fail(c, PPE_ENOMEM, "flow table: out of device memory (update buckets)");
    }
    if (rc == PPE_OK && (hipHostMalloc(&t->snap_h, 64, hipHostMallocMapped) != hipSuccess ||
                         hipHostGetDevicePointer((void **)&t->snap_d, t->snap_h, 0) != hipSuccess))
        rc = fail(c, PPE_ENOMEM, "flow table: pinned snapshot buffer");
    if (rc == PPE_OK) std::memset(t->snap_h, 0, 64);
    if (rc == PPE_OK &&
        hipEventCreateWithFlags(&t->pre_launch, hipEventDisableTiming | hipEventBlockingSync) != hipSuccess)
        rc = fail(c, PPE_EIO, "flow table: event");
    t->cum_n.assign(FlowTable::kSnapRing, 0);
    t->cum_rev.assign(FlowTable::kSnapRing, 0);
    if (rc == PPE_OK) rc = flow_clear_arrays(c, t->arr[0], ns, nullptr);
    if (rc == PPE_OK && hipDeviceSynchronize() != hipSuccess) rc = fail(c, PPE_EIO, "flow table init failed");
    if (rc != PPE_OK) ppe_flow_destroy(c);
    return rc;
}

int ppe_classify_flow(ppe_ctx_t *c, const ppe_batch_t *in, const ppe_result_t *out, const ppe_cfg_t *cfg,
                      void *stream) {
    if (!c || !out) return PPE_EINVAL;
    if (const int u = flow_usable(c)) return u;
    if (!out->verdict) return fail(c, PPE_EINVAL, "ppe_classify_flow needs the verdict output");
    int rc = check_batch(c, in, cfg);
    if (rc != PPE_OK || in->n == 0) return rc;
    FlowTable &t = *c->flow;
    if (in->n > t.max_batch) return fail(c, PPE_EINVAL, "batch larger than the flow table's max_batch");
    HIPCHK(c, use_device(c));
    flow_apply_snapshot(t);
    if (t.tomb_ub > t.nslots / 4u && t.snap_used + 1u < t.batches) {
        // The tombstone bound counts every packet of every batch since the snapshot as a possible revocation, so with
        // the host several batches ahead it passes the rehash threshold long before the table does.  Wait (bounded)
        // for the latest submitted batch's classify launch to publish its snapshot — one batch stays in flight, the
        // queue does not drain — and decide on that tighter bound before synchronising.  The host polls the snapshot
        // the launch's first workgroup writes as it starts, yielding its core between polls (sched_yield: no busy
        // spin), at most 20 ms.  Until round 4 it first slept on an event recorded before each classify
        // launch; that marker cost the stream a 6-us gap per batch (PPE_FLOW_EVENT=1 restores it, for A/B).
        if (t.use_event) HIPCHK(c, hipEventSynchronize(t.pre_launch));
        const auto until = std::chrono::steady_clock::now() + std::chrono::milliseconds(20);
        while (t.snap_used + 1u < t.batches && std::chrono::steady_clock::now() < until) {
            if (t.use_event) __builtin_ia32_pause();
            else sched_yield();
            flow_apply_snapshot(t);
        }
    }
    rc = flow_maybe_rehash(c);
    if (rc != PPE_OK) return rc;
    const hipStream_t s = (hipStream_t)stream;
    const ppe_flowdev d = flow_dev(t, t.cur);
    if (t.use_event) HIPCHK(c, hipEventRecord(t.pre_launch, s));
    // 1. decode, hash, FlowFind; found flows are forwarded and their updates logged to the owners' buckets, the
    // rest get syn_check + ACL (would-be creators claim their slots)
    uint32_t cgrid = 0;
    rc = launch(c, in, out, 1, cfg, s, 0, 0, &d, &cgrid);
    if (rc != PPE_OK) return rc;
    ppe_flow_kargs k;
    std::memset(&k, 0, sizeof k);
    k.f = d;
    k.f.upd_grid = cgrid;
    k.len = in->len;
    k.verdict = out->verdict;
    k.hit = out->acl_hit;
    k.fw_idx = out->fw_idx;
    k.drop_idx = out->drop_idx;
    k.tile_cnt = out->tile_cnt;
    k.part8 = out->part8;
    k.n = in->n;
    k.unsup_fw = cfg ? cfg->unsupport_proto_action : 0u;
    k.now = cfg ? cfg->now_seconds : 0u;
    k.nslots = t.nslots;
    k.cslots = c->d_cslots;
    // 2. the post-classify launch: finalize (grid-stride over the miss-tile list, usually short: at most one
    // workgroup per CU) and, beside it, the found flows' counters and last-seen times, one workgroup per owner
    // (disjoint from the slots finalize touches).  When the host's bound says the pool may overflow, finalize checks
    // the exact counts and, on an overflow, marks the creators and has its workgroup 0 revoke those past the pool's
    // room first.
    const uint32_t fg = std::min(std::min(flow_grid(c, (in->n + 63u) / 64u, PPE_FLOW_POST_BLOCK / 64u), c->n_cu),
                                 t.fin_cap ? t.fin_cap : c->n_cu);
    const bool may_overflow = t.live_ub + in->n > t.capacity;
    k.revoke = may_overflow ? 1u : 0u;
    k.fin_wgs = fg;
    {
        const int e = take_fail_post() ? (int)hipErrorLaunchFailure
                                       : ppe_launch_flow(PPE_FLOW_K_POST, &k, fg + (t.upd_wgs ? t.upd_owners : 0u), (void *)s);
        if (e != 0) {
            t.broken = true;  // the classify launch above claimed slots that nothing will finalize
            return fail(c, PPE_EIO, "flow post-classify launch failed: %s", hipGetErrorString((hipError_t)e));
        }
    }
    t.cum_n[t.batches % FlowTable::kSnapRing] = t.tot_n;
    t.cum_rev[t.batches % FlowTable::kSnapRing] = t.tot_rev;
    t.tot_n += in->n;
    if (may_overflow) t.tot_rev += in->n;
    ++t.batches;
    t.live_ub = std::min<uint64_t>(t.live_ub + in->n, t.capacity);
    if (may_overflow) t.tomb_ub += in->n;  // revoked claims leave tombstones
    return PPE_OK;
}

int ppe_flow_age(ppe_ctx_t *c, uint64_t now_seconds, uint64_t timeout_seconds, uint64_t *deleted) {
    if (!c) return PPE_EINVAL;
    if (const int u = flow_usable(c)) return u;
    HIPCHK(c, use_device(c));
    FlowTable &t = *c->flow;
    unsigned long long before[PPE_FCTL_WORDS], after[PPE_FCTL_WORDS];
    int rc = flow_sync_counts(c, before);
    if (rc != PPE_OK) return rc;
    ppe_flow_kargs k;
    std::memset(&k, 0, sizeof k);
    k.f = flow_dev(t, t.cur);
    k.now = now_seconds;
    k.timeout = timeout_seconds;
    k.nslots = t.nslots;
    rc = ppe_launch_flow(PPE_FLOW_K_AGE, &k, flow_grid(c, t.nslots, 256u), nullptr);
    if (rc != 0) return fail(c, PPE_EIO, "flow age launch failed: %s", hipGetErrorString((hipError_t)rc));
    rc = flow_sync_counts(c, after);
    if (rc != PPE_OK) return rc;
    if (deleted) *deleted = after[PPE_FCTL_DEL_FLOW] - before[PPE_FCTL_DEL_FLOW];
    return flow_maybe_rehash(c);
}

int ppe_flow_info(ppe_ctx_t *c, ppe_flow_info_t *info) {
    if (!c || !info) return PPE_EINVAL;
    if (const int u = flow_usable(c)) return u;
    HIPCHK(c, use_device(c));
    unsigned long long ctl[PPE_FCTL_WORDS];
    const int rc = flow_sync_counts(c, ctl);
    if (rc != PPE_OK) return rc;
    std::memset(info, 0, sizeof *info);
    const FlowTable &t = *c->flow;
    info->live = ctl[PPE_FCTL_LIVE];
    info->new_flow = ctl[PPE_FCTL_NEW_FLOW];
    info->del_flow = ctl[PPE_FCTL_DEL_FLOW];
    info->capacity = t.capacity;
    info->max_batch = t.max_batch;
    info->slots = t.nslots;
    info->tombstones = (uint32_t)ctl[PPE_FCTL_TOMBS];
    info->rehashes = t.rehashes;
    return PPE_OK;
}

int ppe_flow_clear_stat(ppe_ctx_t *c) {
    if (!c) return PPE_EINVAL;
    if (const int u = flow_usable(c)) return u;
    HIPCHK(c, use_device(c));
    HIPCHK(c, hipDeviceSynchronize());
    HIPCHK(c, hipMemset(c->flow->ctl + PPE_FCTL_NEW_FLOW, 0, 16u));  // new_flow, del_flow
    return PPE_OK;
}

int ppe_flow_dump(ppe_ctx_t *c, ppe_flow_entry_t *entries, uint32_t max, uint32_t *n) {
    if (!c || !n) return PPE_EINVAL;
    if (const int u = flow_usable(c)) return u;
    HIPCHK(c, use_device(c));
    HIPCHK(c, hipDeviceSynchronize());
    const FlowTable &t = *c->flow;
    const FlowArrays &a = t.arr[t.cur];
    constexpr uint32_t W = PPE_FLOW_SLOT_WORDS;
    std::vector<uint32_t> keys((size_t)t.nslots * W);
    HIPCHK(c, hipMemcpy(keys.data(), a.keys, keys.size() * 4u, hipMemcpyDeviceToHost));
    std::vector<unsigned long long> stats, recs;
    if (entries && max) {
        stats.resize((size_t)t.nslots * 4u);
        HIPCHK(c, hipMemcpy(stats.data(), a.stats, stats.size() * 8u, hipMemcpyDeviceToHost));
        recs.resize((size_t)t.nslots * PPE_FLOW_REC_WORDS);
        HIPCHK(c, hipMemcpy(recs.data(), a.recs, recs.size() * 8u, hipMemcpyDeviceToHost));
    }
    uint32_t k = 0;
    for (uint32_t s = 0; s < t.nslots; ++s) {
        const uint32_t *kw = &keys[(size_t)W * s], st = kw[3];
        if ((st & (PPE_FS_PEND | 0xffu)) != PPE_FS_LIVE(0u)) continue;
        if (entries && k < max) {
            ppe_flow_entry_t &e = entries[k];
            std::memset(&e, 0, sizeof e);
            e.sip = kw[0];
            e.dip = kw[1];
            e.sport = (uint16_t)(kw[2] & 0xffffu);
            e.dport = (uint16_t)(kw[2] >> 16);
            e.protocol = (uint8_t)(st >> 8);
            e.slot = s;
            const unsigned long long *pr = &recs[(size_t)PPE_FLOW_REC_WORDS * s];  // packed counters, last-seen
            const unsigned long long bmask = (1ull << PPE_PK_SHIFT) - 1u, p0 = pr[0], p1 = pr[1];
            e.pktcnts2d = stats[4u * s] + (p0 >> PPE_PK_SHIFT);
            e.bytecnts2d = stats[4u * s + 1u] + (p0 & bmask);
            e.pktcntd2s = stats[4u * s + 2u] + (p1 >> PPE_PK_SHIFT);
            e.bytecntd2s = stats[4u * s + 3u] + (p1 & bmask);
            e.last_seen = pr[PPE_FLOW_REC_LAST];
        }
        ++k;
    }
    *n = k;
    return PPE_OK;
}

// ---------------------------------------------------------------------------------------------------------------
// Flow-hash steering across GPUs

int ppe_steer_partition(ppe_ctx_t *c, const uint32_t *verdict, const uint32_t *flow_hash, uint32_t n, uint32_t world,
                        uint32_t rank, uint32_t *perm, uint32_t *counts, void *stream) {
    if (!c) return PPE_EINVAL;
    if (world == 0 || world > PPE_STEER_MAX_WORLD || rank >= world)
        return fail(c, PPE_EINVAL, "world must be 1..%d and rank < world", PPE_STEER_MAX_WORLD);
    if (!counts || (n && (!verdict || !flow_hash || !perm))) return fail(c, PPE_EINVAL, "null argument");
    HIPCHK(c, use_device(c));
    const hipStream_t s = (hipStream_t)stream;
    if (n == 0) {
        HIPCHK(c, hipMemsetAsync(counts, 0, (size_t)world * 4u, s));
        return PPE_OK;
    }
    const uint32_t tiles = (n + 63u) / 64u;
    const size_t need = (size_t)tiles * world * 4u;
    if (need > c->steer_cap) {
        HIPCHK(c, hipStreamSynchronize(s));  // the old buffer may be in use by queued work
        if (c->d_steer) HIPCHK(c, hipFree(c->d_steer));
        c->d_steer = nullptr;
        c->steer_cap = 0;
        HIPCHK(c, hipMalloc(&c->d_steer, need));
        c->steer_cap = need;
    }
    ppe_steer_kargs k;
    std::memset(&k, 0, sizeof k);
    k.verdict = verdict;
    k.flow_hash = flow_hash;
    k.n = n;
    k.world = world;
    k.rank = rank;
    k.tcount = c->d_steer;
    k.perm = perm;
    k.counts = counts;
    const uint32_t grid = std::max(1u, std::min((tiles + 3u) / 4u, c->n_cu * 8u));
    for (int phase = 0; phase < 3; ++phase) {
        const int e = ppe_launch_steer(phase, &k, grid, (void *)s);
        if (e != 0) return fail(c, PPE_EIO, "steer kernel %d: %s", phase, hipGetErrorString((hipError_t)e));
    }
    return PPE_OK;
}

static int rows(ppe_ctx_t *c, const void *src, uint32_t row_bytes, const uint32_t *perm, uint32_t n, void *dst,
                int scatter, void *stream) {
    if (!c) return PPE_EINVAL;
    if (row_bytes == 0 || row_bytes % 4u || row_bytes > 256u) return fail(c, PPE_EINVAL, "row_bytes: 4..256, x4");
    if (n == 0) return PPE_OK;
    if (!src || !dst || !perm) return fail(c, PPE_EINVAL, "null argument");
    HIPCHK(c, use_device(c));
    ppe_rows_kargs k = {(const uint8_t *)src, (uint8_t *)dst, perm, n, row_bytes, (uint32_t)scatter, 0u};
    const uint64_t words = (uint64_t)n * (row_bytes / 4u);
    const uint32_t grid = (uint32_t)std::max<uint64_t>(1u, std::min<uint64_t>((words + 255u) / 256u, c->n_cu * 16u));
    const int e = ppe_launch_rows(&k, grid, stream);
    if (e != 0) return fail(c, PPE_EIO, "rows kernel: %s", hipGetErrorString((hipError_t)e));
    return PPE_OK;
}

int ppe_gather_rows(ppe_ctx_t *c, const void *src, uint32_t row_bytes, const uint32_t *perm, uint32_t n, void *dst,
                    void *stream) {
    return rows(c, src, row_bytes, perm, n, dst, 0, stream);
}

int ppe_scatter_rows(ppe_ctx_t *c, const void *src, uint32_t row_bytes, const uint32_t *perm, uint32_t n, void *dst,
                     void *stream) {
    return rows(c, src, row_bytes, perm, n, dst, 1, stream);
}

}  // extern "C"
