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
    uint32_t pad;
};

/* batches per launch: the descriptors travel in the kernel arguments (8 × 96 B) */
#define PPE_MAX_BATCH 8

/* Kernel launch parameters, passed by value. */
struct ppe_kargs {
    struct ppe_bdesc batch[PPE_MAX_BATCH];  /* [0, nbatch): processed in order by every wave, no barrier between */
    uint32_t nbatch;
    uint32_t max_tiles;       /* largest batch's tile count */
    const uint32_t *img;      /* device classifier image (ppe_image.h) */
    uint32_t img_words;
    uint32_t unsup_fw;        /* 1: unsupported protocols are forwarded */
    uint32_t syn_check;
    uint32_t default_action;
    uint64_t now;
    uint32_t lds_words;       /* image words staged in LDS (IMG_LDS: all; IMG_SPLIT: header + top nodes [+ leaves]) */
    uint32_t lds_iters;       /* IMG_SPLIT: walk levels (node reads) whose nodes are all in the staged BFS prefix      */
    uint32_t max_depth;       /* deepest leaf: the walk reads max_depth + 1 nodes                                     */
    uint32_t max_leaf;        /* longest leaf candidate list: uniform trip count of the leaf scan                     */
    uint32_t root_ks;         /* the root node's key slot << 8 (image header word PPE_IMG_W_ROOTKS)                    */
    uint32_t jump;            /* jump root descriptor (image header word PPE_IMG_W_JUMP), 0 = none                    */
    uint32_t off_nodes;       /* image word offset of the nodes (after the jump table)                                */
    uint32_t off_leaf, off_rules, off_resid; /* image section offsets (words), from the image header: kernel arguments
                                                (scalar registers, no load in the loop)                               */
    unsigned long long *cslots; /* [grid][PPE_CSLOT_WORDS] counter slots, one per workgroup */
    unsigned long long *trace;  /* diagnostic builds (PPE_TRACE) only: per-wave phase timestamps, else unused */
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
int ppe_launch_classify(const struct ppe_kargs *a, uint32_t grid, int mode, int pipe, int block, void *stream,
                        void *ev_start, void *ev_stop);
int ppe_classify_occupancy(uint32_t lds_words, int mode, int pipe, int block);
uint32_t ppe_classify_fixed_lds(int block);
int ppe_launch_acl_tuples(const struct ppe_tuple_kargs *a, uint32_t grid, int lds_img, void *stream);
#ifdef __cplusplus
}
#endif

#endif
