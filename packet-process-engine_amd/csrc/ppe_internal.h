/* ppe_internal.h — declarations shared between the engine (host) and the HIP kernel translation unit. */
#ifndef PPE_INTERNAL_H
#define PPE_INTERNAL_H

#include <stdint.h>

/* One batch of a launch: inputs, outputs (NULL = skipped) and sizes, as in ppe_batch_t / ppe_result_t. */
struct ppe_bdesc {
    const uint8_t *hdr;
    const uint32_t *len;
    const uint64_t *ts;
    uint32_t *verdict;
    uint32_t *fhash;
    int32_t *hit;
    uint32_t *fw_idx;
    uint32_t *drop_idx;
    uint32_t *tile_cnt;
    uint32_t *tuple;
    uint32_t n;
    uint32_t stride;
    uint32_t idx_base;        /* added to the packet indices written to fw_idx / drop_idx */
    uint32_t flags;           /* PPE_BD_PART8: tile_cnt carries the compact partition list (ppe_result_t.part8);
                                 PPE_BD_PACKED: verdict carries the 8-B packed results (ppe_result_t.packed) */
};
#define PPE_BD_PART8 1u
#define PPE_BD_PACKED 2u

/* Device flow table (ppe_classify_flow; ppe_kernels.hip "flow table").  Open addressing over groups of
 * PPE_FLOW_GROUP slots, linear probing from group flow_hash & gmask; a key lies before the first EMPTY slot of its
 * probe sequence (slots never return to EMPTY: deletions leave TOMBs, reclaimed by a rehash).  The probe array holds
 * only the keys, 16 B per slot {sip, dip, sport | dport << 16, state}, so a probe group of 4 slots is one 64-B
 * segment: one HBM request per probe (round 5; until then a 64-B slot record with the counters inside, a 128-B line
 * per probe group of 2).  The counters live in a record array of their own, 32 B per slot: the packed counters of
 * both directions and the last-seen time (`packed`). */
#define PPE_FLOW_GROUP 4u       /* slots per probe group */
#define PPE_FLOW_SLOT_WORDS 4u  /* u32 words per slot key */
#define PPE_FLOW_REC_WORDS 4u   /* u64 stride of the counter records {s2d, d2s, last-seen, 0} */
#define PPE_FLOW_REC_LAST 2u    /* the counter record's last-seen time */
#define PPE_FS_EMPTY 0u
#define PPE_FS_TOMB 1u
#define PPE_FS_LIVE(proto) (2u | ((proto) << 8))  /* key words valid */
#define PPE_FS_PEND 0x80000000u                   /* | packet index: claimed by this batch, key = rec[index] */
#define PPE_FLOW_NONE 0xffffffffu
#define PPE_FLOW_REVOKED 0x80000000u              /* creator word: pool exhausted, the claim is withdrawn */
enum { PPE_FCTL_LIVE = 0, PPE_FCTL_NEW_FLOW, PPE_FCTL_DEL_FLOW, PPE_FCTL_BATCH_NEW, PPE_FCTL_TOMBS,
       PPE_FCTL_MISS0, PPE_FCTL_MISS1, /* tiles with pending packets, by batch parity */
       PPE_FCTL_REVOKED_SEQ,           /* finalize: workgroup 0's revoke published for batch seq + 1 */
       PPE_FCTL_ERR,                   /* finalize: waits for the revoke flag that gave up (results not exact) */
       PPE_FCTL_LIVE_AT_BATCH,         /* LIVE as the batch's classify launch started: every finalize workgroup takes
                                          its overflow decision from this word, which nothing changes during finalize
                                          (LIVE itself grows as finalize workgroups finish) */
       PPE_FCTL_BATCH_NEW1,            /* BATCH_NEW of odd batches: the creators (slots claimed) the classify launch
                                          counts, by batch parity; finalize reads its batch's and zeroes the next's */
       PPE_FCTL_ARRIVE,                /* finalize, overflow batches: workgroups done marking their tiles' creators */
       PPE_FCTL_WORDS = 16 };
#define PPE_PK_SHIFT 40u                       /* packed counter: packets in bits 63:40, bytes in 39:0 */
#define PPE_PK_FOLD_PKTS (1ull << 23)          /* fold into `stats` once either field reaches half its range */
#define PPE_PK_FOLD_BYTES (1ull << 39)
/* Owner-computed FlowUpdate (flow_update_wg, ppe_flow_post_kernel): a found packet's counter update goes to a bucket of its slot's
 * owner (one of at most PPE_UPD_OWNERS slot ranges) in its classify workgroup's column, instead of a memory-side
 * atomic per packet; each owner's workgroup then sums its buckets in LDS and updates each touched slot once. */
#ifndef PPE_UPD_OWNERS
#define PPE_UPD_OWNERS 256u
#endif
#define PPE_UPD_CAP 16u        /* entries per (owner, classify workgroup) bucket; a full bucket: the direct atomic */
#ifndef PPE_UPD_HASH
#define PPE_UPD_HASH 4096u     /* LDS hash entries of an owner workgroup (slots it accumulates; more: direct atomics) */
#endif
#ifndef PPE_FLOW_POST_BLOCK
#define PPE_FLOW_POST_BLOCK 1024 /* workgroup size of the post-classify launch (finalize + update; 512: +1.4 µs per F1 batch) */
#endif
struct ppe_flowdev {
    uint32_t *keys;               /* nslots × {sip, dip, sport | dport << 16, state}: the key in the creating packet's
                                     orientation (the probe array)                                                     */
    unsigned long long *packed;   /* nslots × {s2d, d2s, last-seen, 0} (stride PPE_FLOW_REC_WORDS): packets << 40 |
                                     bytes per direction (FlowUpdate) and the last-seen time                          */
    unsigned long long *stats;    /* nslots × {pkts s2d, bytes s2d, pkts d2s, bytes d2s}: folded from `packed` before a
                                     field can overflow; a flow's counters = stats + the packed fields               */
    uint32_t *creator;            /* nslots: lowest index of the packets claiming the slot in this batch (| REVOKED)   */
    unsigned long long *ctl;      /* PPE_FCTL_* device counters                                                        */
    uint32_t *rec;                /* max_batch × {sip, dip, ports, proto | provisional status << 8} of pending packets */
    unsigned long long *tile_miss;  /* per tile: lanes whose flow was not found (pending resolution)                   */
    unsigned long long *tile_new;   /* per tile: lanes that create their flow                                          */
    uint32_t *rslot;              /* max_batch: the slot a pending packet's flow was claimed in, or PPE_FLOW_NONE       */
    uint32_t *miss_tiles;         /* tiles with pending packets (unordered), count in ctl[PPE_FCTL_MISS0 + parity]      */
    uint32_t parity;              /* batch sequence number & 1                                                         */
    unsigned long long fold_pkts, fold_bytes;  /* packed-counter fold thresholds (PPE_PK_FOLD_*; lowered by tests)   */
    unsigned long long *snap;     /* pinned host words {seq, live, tombstones}: written by the classify launch        */
    unsigned long long seq;       /* batches completed before this one                                                 */
    uint32_t gmask;               /* slot groups - 1                                                                   */
    uint32_t capacity;            /* flow pool size                                                                     */
    unsigned long long *upd;      /* [owner][upd_wgs][PPE_UPD_CAP]: slot | (wire length | dir << 31) << 32             */
    uint32_t *ucnt;               /* [upd_wgs][owner]: entries in each bucket (written by the classify launch)         */
    uint32_t upd_wgs;             /* classify workgroups with a bucket column (0: every found packet's atomic inline)  */
    uint32_t upd_osh;             /* owner of slot s = s >> upd_osh                                                      */
    uint32_t upd_owners;          /* owners (nslots >> upd_osh)                                                          */
    uint32_t upd_grid;            /* the update kernel: the batch's classify grid (bucket columns written)              */
    uint32_t upd_hmask;           /* the update kernel's LDS hash entries - 1 (PPE_UPD_HASH - 1; lowered by tests)       */
};

/* flow-table kernels after the classify kernel (one batch) */
struct ppe_flow_kargs {
    struct ppe_flowdev f;
    const uint32_t *len;          /* the batch's wire lengths (byte counters) */
    uint32_t *verdict;
    int32_t *hit;
    uint32_t *fw_idx, *drop_idx, *tile_cnt;
    uint8_t *part8;               /* compact partition list (ppe_result_t.part8) */
    uint32_t n;
    uint32_t unsup_fw;
    uint64_t now;
    uint64_t timeout;             /* aging */
    uint32_t nslots;
    uint32_t revoke;              /* finalize: the host's bound says the pool may overflow (check, rank, revoke) */
    uint32_t fin_wgs;             /* post-classify launch: workgroups [0, fin_wgs) finalize, the next upd_owners update */
    unsigned long long *cslots;   /* counter slots (one per workgroup) */
    struct ppe_flowdev dst;       /* rehash target */
};

/* batches per launch whose descriptors travel in the kernel arguments (32 × 96 B); a launch over more batches reads
 * them from a device descriptor ring (ppe_kargs.ring) */
#define PPE_MAX_BATCH 32
/* most batches one ring launch takes */
#define PPE_MAX_RING 4096

/* Kernel launch parameters, passed by value. */
struct ppe_kargs {
    struct ppe_bdesc batch[PPE_MAX_BATCH];  /* [0, nbatch) when nbatch <= PPE_MAX_BATCH.  The grid's waves split into
                                               G = min(waves, nbatch, max_groups) batch groups that run concurrently:
                                               group g takes batches g, g + G, ... in turn (no barrier between them),
                                               its waves striding over each batch's tiles */
    const struct ppe_bdesc *ring;           /* non-NULL: the nbatch descriptors are ring[0, nbatch) in device memory
                                               (one persistent launch over a whole queue of batches, nbatch beyond
                                               PPE_MAX_BATCH); batch[0] then repeats ring[0] */
    uint32_t nbatch;
    uint32_t max_tiles;       /* largest batch's tile count */
    const uint32_t *img;      /* device classifier image (ppe_image.h) */
    uint32_t img_words;
    uint32_t unsup_fw;        /* 1: unsupported protocols are forwarded */
    uint32_t syn_check;
    uint32_t default_action;
    uint64_t now;
    uint32_t lds_words;       /* image words [0, lds_words) in LDS at its image base (single-tile walks; the leaf
                                 lists / rule records of every walk are read from LDS when inside this prefix)   */
    uint32_t stage_src, stage_words; /* the kernel stages image words [stage_src, + stage_words) at its LDS image base */
    uint32_t lds_blocks;      /* multi-tile walks: 2-level blocks [0, lds_blocks) are in LDS                        */
    uint32_t bsec_lds, blk_lds; /* LDS byte offsets (from the LDS image base) of the block section / of block 0     */
    uint32_t off_bsec, off_blocks, max_bdepth; /* image header words 15, 17, 18                                  */
    uint32_t off_crec, off_idtab; /* image header words 19, 20: compact leaf records / slot → index table (0 = none) */
    uint32_t crec_lds, idtab_lds; /* their LDS byte offsets from the LDS image base, ~0u = read from global memory   */
    uint32_t cut;             /* cut-list walks (image v8): cut header word 0 (sip bits | dip bits << 8 | ids16)     */
    uint32_t cut_slc, cut_gbase, cut_fp, cut_ent;  /* word offsets of the length slices / group bases / fingerprints /
                                                      entry lines in the image                                       */
    uint32_t cut_epl, cut_div;  /* entries per 128-B line, and the divisor magic (e / epl = umulhi(e, cut_div))      */
    uint32_t cut_idrel;         /* without PPE_CUT_LINES: the id array's byte offset from the entry lines             */
    uint32_t cut_gbase_lds, cut_fp_lds, cut_ent_lds;  /* their LDS byte offsets from the LDS image base (the slices
                                                         are at it; the entry lines: IMG_LDS only)                   */
    uint32_t max_groups;      /* most batch groups of waves (concurrently streamed batches)                          */
    uint32_t part_layout;     /* 1: every batch writes verdict + flow hash + ACL hit and one partition list (fw_idx ==
                                 drop_idx), no tile counts, no tuple: the kernel variant with those checks compiled out */
    uint32_t lds_iters;       /* IMG_SPLIT: walk levels (node reads) whose nodes are all in the staged BFS prefix      */
    uint32_t max_depth;       /* deepest leaf: the walk reads max_depth + 1 nodes                                     */
    uint32_t max_leaf;        /* longest leaf candidate list: uniform trip count of the leaf scan                     */
    uint32_t root_ks;         /* the root node's key slot << 8 (image header word PPE_IMG_W_ROOTKS)                    */
    uint32_t jump;            /* jump root descriptor (image header word PPE_IMG_W_JUMP), 0 = none                    */
    uint32_t off_nodes;       /* image word offset of the nodes (after the jump table)                                */
    uint32_t off_leaf, off_rules, off_resid; /* image section offsets (words), from the image header: kernel arguments
                                                (scalar registers, no load in the loop)                               */
    unsigned long long *cslots; /* [grid][PPE_CSLOT_WORDS] counter slots, one per workgroup */
    /* the launch's completion, for the host's image / descriptor-ring reader bookkeeping (no event marker behind each
       launch): every workgroup, at its end, adds 1 to *done_cnt (a per-slot running count); the one that brings it to
       done_target writes done_seq to *done_host (pinned host memory).  done_cnt NULL: not tracked */
    unsigned long long *done_cnt, *done_host;
    unsigned long long done_target, done_seq;
    struct ppe_flowdev flow;    /* flow-table launches (ppe_classify_flow, one batch) */
};

/* flow-hash steering across GPUs (ppe_steer_partition / ppe_gather_rows / ppe_scatter_rows) */
#define PPE_STEER_MAX_WORLD 16
struct ppe_steer_kargs {
    const uint32_t *verdict;      /* stateless verdict words (PPE_F_L4 in the flags) */
    const uint32_t *flow_hash;
    uint32_t n, world, rank, pad;
    uint32_t *tcount;             /* [tiles][world]: per-tile owner counts, then exclusive offsets into perm */
    uint32_t *perm;               /* [n]: packet indices grouped by owner, ascending within an owner */
    uint32_t *counts;             /* [world] */
};
struct ppe_rows_kargs {
    const uint8_t *src;
    uint8_t *dst;
    const uint32_t *perm;
    uint32_t n, row_bytes;        /* row_bytes: a multiple of 4, <= 256 */
    uint32_t scatter;             /* 0: dst[i] = src[perm[i]]; 1: dst[perm[i]] = src[i] */
    uint32_t pad;
};

struct ppe_tuple_kargs {
    const uint32_t *tuple;    /* n × {sip, dip, sport | dport << 16, proto} */
    const uint32_t *macs;     /* optional n × {dmac lo, dmac hi, smac lo, smac hi} */
    const uint64_t *ts;
    uint32_t n;
    int32_t *hit;
    uint32_t *action;
    const uint32_t *img;
    uint32_t img_words;
    uint32_t default_action;
    uint64_t now;
};

#define PPE_CSLOT_WORDS 32
#define PPE_LDS_FIXED 1152u /* classify kernel LDS after the walk keys: 256 counter bins + 32 counters (u32) */
#define PPE_BLOCK 256
/* largest staged classifier image per workgroup (1024-thread workgroups, 2 per CU, each with 25 KB of keys + bins) */
#define PPE_LDS_IMG_MAX (54u * 1024u)

#ifdef __cplusplus
extern "C" {
#endif
/* Launch the classify kernel. grid = workgroups (persistent), lds_img = stage image in LDS. Returns hipError_t. */
/* mode: 0 image in global memory, 1 whole image in LDS, 2 prefix in LDS; pipe: 0 first tile loaded at the loop top,
 * 1 first tile's loads issued before the image staging (see ppe_kernels.hip) */
int ppe_launch_classify(const struct ppe_kargs *a, uint32_t grid, int mode, int pipe, int block, int flow,
                        void *stream, void *ev_start, void *ev_stop);
/* flow-table phases after a flow-mode classify launch (stream order): claim, resolve, finalize (+ revoke in its
 * workgroup 0 when the pool overflows) */
enum { PPE_FLOW_K_POST = 0, PPE_FLOW_K_AGE, PPE_FLOW_K_REHASH };
int ppe_launch_flow(int kind, const struct ppe_flow_kargs *a, uint32_t grid, void *stream);
#define PPE_FLOW_BLOCK 256      /* flow kernels' workgroup size */
/* steering: 0 count, 1 scan (one workgroup), 2 scatter the permutation; rows: gather / scatter of fixed rows */
int ppe_launch_steer(int phase, const struct ppe_steer_kargs *a, uint32_t grid, void *stream);
int ppe_launch_rows(const struct ppe_rows_kargs *a, uint32_t grid, void *stream);
#define PPE_FLOW_BLOCK_WAVES 4u /* waves (tiles in flight) per flow-kernel workgroup */
int ppe_classify_occupancy(uint32_t lds_words, int mode, int pipe, int block);
uint32_t ppe_classify_fixed_lds(int block, int pipe, int mode);
uint32_t ppe_flow_lds_extra(void);  /* classify LDS of a flow-table launch beyond the stateless kernel's (buckets) */
uint32_t ppe_flow_waves(void);      /* waves per SIMD of the flow-table classify kernel */
int ppe_classify_occupancy_flow(uint32_t lds_words, int mode, int block);  /* key slots (node walks only) + counter bins */
int ppe_launch_acl_tuples(const struct ppe_tuple_kargs *a, uint32_t grid, int lds_img, void *stream);
#ifdef __cplusplus
}
#endif

#endif
