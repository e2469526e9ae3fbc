/*
 * ppe_image.h — layout of the device classifier image (one flat array of u32 words).
 *
 * The image is a HyperSplit-style binary decision tree over the five header dimensions, flattened in BFS order
 * (children of node k are 2 consecutive nodes with index > k, so a walk strictly increases the node index and
 * always terminates), followed by the leaf rule lists, the compact rule records and their residual (MAC / time)
 * records.  The reference's tree engine (dp_acl.c / acl64.c, built by dataplane/src/acl/acl.mk:13-15) is absent;
 * its statistics names (gWstDepth, gAvgDepth, gNumTreeNode, gNumLeafNode: dataplane/src/common/dp_cmd.c:2032-2036)
 * are reproduced from this structure.
 *
 *  word 0   PPE_IMG_MAGIC
 *  word 1   PPE_IMG_VERSION
 *  word 2   n_nodes           word 3  n_leaf_entries      word 4  n_rules (slots)
 *  word 5   off_nodes         word 6  off_leaf            word 7  off_rules       word 8  off_resid   (word offsets)
 *  word 9   default_action    word 10 max_depth           word 11 total words     word 12 max leaf entries
 *  word 13..15 reserved
 *
 *  node (2 words, 8-B aligned):  y = (child << 11) | (dim << 8) | count
 *      internal: x = threshold, child = left, dim 0 sip, 1 dip, 2 sport, 3 dport, 4 proto, count 0
 *                key <= threshold → left, key > threshold → left + 1
 *      leaf:     dim = PPE_NODE_LEAF (5): the walk's key slot 5 holds 0, so "key > x" is false and the walk stays
 *                at child = the leaf itself (a fixed point: every lane can walk max_depth levels without a per-lane
 *                exit).  x = first leaf entry; count = number of entries, or PPE_LEAF_CNT_ESC when the count is
 *                stored in leaf entry x and the entries start at x + 1.
 *      The field positions let the walk form the key's LDS offset as y & 0x700 (slot stride 256 B) and the child's
 *      byte offset as (y >> 8) & ~7.
 *  leaf entry (1 word): rule slot | (certain << 31)      certain: the rule's 5-tuple box covers the leaf's region
 *                                                          and it has no residual field, so it matches unchecked
 *  rule (8 words, 32-B aligned), slot order == ascending rule index:
 *      sip_lo, sip_hi, dip_lo, dip_hi, sport_lo | sport_hi << 16, dport_lo | dport_hi << 16,
 *      proto_lo | proto_hi << 8 | action << 16, rule_index | resid << 29
 *  resid (8 words per slot; present only when at least one rule has a residual field, read only for those):
 *      dmac bytes 0-3 (LE), dmac bytes 4-5, smac bytes 0-3, smac bytes 4-5,
 *      time_start lo, hi, time_end lo, hi
 *      resid bits: 1 = dmac must equal, 2 = smac must equal, 4 = time_start <= ts <= time_end
 */
#ifndef PPE_IMAGE_H
#define PPE_IMAGE_H

#define PPE_IMG_MAGIC   0x41455050u /* "PPEA" */
#define PPE_IMG_VERSION 2u
#define PPE_IMG_HDR_WORDS 16u

#define PPE_IMG_W_NNODES   2
#define PPE_IMG_W_NLEAF    3
#define PPE_IMG_W_NRULES   4
#define PPE_IMG_W_OFFNODES 5
#define PPE_IMG_W_OFFLEAF  6
#define PPE_IMG_W_OFFRULES 7
#define PPE_IMG_W_OFFRESID 8
#define PPE_IMG_W_DEFACT   9
#define PPE_IMG_W_MAXDEPTH 10
#define PPE_IMG_W_TOTAL    11
#define PPE_IMG_W_MAXLEAF  12

#define PPE_NODE_LEAF 5u          /* leaf marker in the dim field; also the index of the walk's zero key slot */
#define PPE_NODE_CHILD_SHIFT 11u
#define PPE_NODE_DIM(y) (((y) >> 8) & 7u)
#define PPE_NODE_MAX (1u << 21)   /* child index field: 21 bits */
#define PPE_LEAF_CNT_ESC 255u     /* count field value meaning "count stored in the first leaf word" */
#define PPE_DIM_SIP   0u
#define PPE_DIM_DIP   1u
#define PPE_DIM_SPORT 2u
#define PPE_DIM_DPORT 3u
#define PPE_DIM_PROTO 4u
#define PPE_NDIMS     5

#define PPE_RESID_DMAC 1u
#define PPE_RESID_SMAC 2u
#define PPE_RESID_TIME 4u

#define PPE_LEAF_CERTAIN 0x80000000u

/* hard bound on walk length, enforced by the builder (max_depth) and by the kernel loop */
#define PPE_MAX_DEPTH 60

#endif
