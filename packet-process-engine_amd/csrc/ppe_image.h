/*
 * ppe_image.h — layout of the device classifier image (one flat array of u32 words), format v8.
 *
 * The image is a HyperSplit-style binary decision tree over the five header dimensions, flattened in BFS order
 * (children of node k are numbered after k, so a walk strictly descends and always terminates), followed by the
 * leaf candidate lists, the compact rule records and their residual (MAC / time) records.  The reference's tree
 * engine (dp_acl.c / acl64.c, built by dataplane/src/acl/acl.mk:13-15) is absent; its statistics names (gWstDepth,
 * gAvgDepth, gNumTreeNode, gNumLeafNode: dataplane/src/common/dp_cmd.c:2032-2036) are reproduced from this structure.
 *
 *  word 0   PPE_IMG_MAGIC
 *  word 1   PPE_IMG_VERSION
 *  word 2   n_nodes           word 3  n_leaf_entries      word 4  n_rules (slots, excluding the sentinel)
 *  word 5   off_nodes         word 6  off_leaf            word 7  off_rules       word 8  off_resid   (word offsets)
 *  word 9   default_action    word 10 max_depth           word 11 total words     word 12 max leaf entries
 *  word 13  root key slot << 8 (the dimension the root splits on; PPE_NODE_LEAF when the root is a leaf)
 *  word 14  jump root: dim | shift << 8 | bits << 16, or 0 for a single tree rooted at node 0
 *  word 15  off_bsec: word offset of the block section (v5)   word 16  n_blocks   word 17  off_blocks (word offset,
 *           32-B aligned)   word 18  max_bdepth: most blocks on a root-to-leaf path
 *  word 19  off_crec: word offset of the compact records (v6), 0 = the image has none
 *  word 20  off_idtab: word offset of the slot → rule index table, 0 = slot == rule index for every slot
 *  word 21  block levels: 2 (32-B blocks)
 *  word 22  off_cut: word offset of the cut-list section (v8), 0 = the image has none
 *  words 23..31 reserved
 *
 *  jump table (format v4; present iff word 14 != 0): 2^bits words right after the header.  A walk starts at
 *      bucket b = key[dim] >> shift: word b = the byte offset of that bucket's subtree root | its key slot << 24.
 *      The subtrees (a HyperCuts-style cut of the top bits of one dimension, each bucket then split HyperSplit-
 *      style) are laid out breadth-first as one forest, roots first, so whole levels of every subtree form a prefix
 *      of the node array (the LDS-staged top of the image).
 *
 *  node (4 words, 16-B aligned; node k at byte 4 * off_nodes + 16 k of the image):
 *      internal: { threshold, left child byte offset, right child byte offset, kslots }
 *                key <= threshold → left, key > threshold → right.  Child byte offsets are from the image start, so
 *                one offset addresses the node in LDS (staged image base + offset) and in global memory alike.
 *                kslots = (left child's key slot << 8) | (right child's key slot << 24): the dimension the CHILD
 *                splits on, known one level ahead, so a walk issues the key read and the node read of a level
 *                together (one LDS round trip per level).  Key slot d = dimension d (0 sip, 1 dip, 2 sport,
 *                3 dport, 4 proto); PPE_NODE_LEAF (5) for a leaf child: the walk's key slot 5 holds 0.
 *      leaf:     { 0xffffffff, own byte offset, payload, PPE_NODE_LEAF << 8 | PPE_NODE_LEAF << 24 }
 *                key 0 is never > 0xffffffff (no internal threshold is 0xffffffff), so a walk that reached a leaf
 *                stays there: every lane can run max_depth + 1 levels without a per-lane exit.
 *                payload, when max_leaf <= 1: the rule slot of the leaf's one candidate, or the sentinel slot
 *                n_rules (an always-matching record with rule index -1 and the default action) for an empty leaf.
 *                payload, when max_leaf > 1: first leaf entry | count << 24, count == PPE_LEAF_CNT_ESC meaning the
 *                count is stored in leaf entry `first` and the entries start at first + 1.
 *  leaf entry (1 word): rule slot, in ascending rule index (= priority) order
 *  rule (8 words, 32-B aligned), slot order == ascending rule index, slot n_rules = the sentinel:
 *      sip_lo, sip_hi - sip_lo, dip_lo, dip_hi - dip_lo, sport_lo | dport_lo << 16,
 *      (sport_hi - sport_lo) | (dport_hi - dport_lo) << 16, proto_lo | (proto_hi - proto_lo) << 8 | action << 16,
 *      rule_index (29-bit two's complement: the sentinel's is -1) | resid << 29
 *      A field matches iff (key - lo) mod 2^w <= span (w = the field width), i.e. lo <= key <= hi.
 *  resid (8 words per slot; present only when at least one rule has a residual field, read only for those):
 *      dmac bytes 0-3 (LE), dmac bytes 4-5, smac bytes 0-3, smac bytes 4-5,
 *      time_start lo, hi, time_end lo, hi
 *      resid bits: 1 = dmac must equal, 2 = smac must equal, 4 = time_start <= ts <= time_end
 *
 *  block section (v5, at off_bsec, after everything above): the same forest regrouped into 2-level BLOCKS, for the
 *  multi-tile walk, which reads the tree from L2 for large rule sets: one 32-B read resolves two levels, so a walk
 *  needs half the dependent memory round trips.
 *      block jump table (present iff word 14 != 0): 2^bits words, bucket → its root block index
 *      blocks (8 words, 32-B aligned; breadth-first by block depth: the LDS-staged prefix is whole block levels).
 *      A block holds 2 tree levels: positions p = 0 .. 2 in BFS order (position p's children are 2p + 1 and
 *      2p + 2), then 4 exits:
 *        w[p]    threshold of position p (w0..w2)
 *        w[3]    key slots: position p's at bits 4p..4p+3
 *        w[4..7] exits e = the 2 comparison bits, first level most significant (2 b0 + b1; b0: key(pos 0) > w0,
 *                b1: key(pos 1 + b0) > w[1 + b0]): PPE_BLK_LEAF | leaf payload (max_leaf <= 1: rule slot /
 *                sentinel, or the compact exit below; else first | count << 23), or the index of the block rooted
 *                at that position's child
 *        A leaf at a position is a pass-through: threshold 0xffffffff (no key is greater) and both of its children
 *        positions / exits carry the leaf, so every walk resolves exactly 2 levels per block.  (3-level 64-B blocks
 *        were an option until round 4: one L2 round trip fewer per three levels, measured slower on C3.)
 *
 *  compact leaves (v6; present iff word 19 != 0: one candidate per leaf (max_leaf <= 1) and no rule with a residual
 *  MAC / time field).  The block walk is the classify kernel's, and only TCP / UDP packets reach the ACL there
 *  (decode-ipv4.c:131-157), so a rule's protocol range matters only through "contains 6" and "contains 17".  A leaf
 *  exit then carries everything about its candidate except the address prefixes and port ranges:
 *      bits 0-23  rule slot (n_rules = the sentinel)         bit 24 DROP: the rule's action == ACL_RULE_ACTION_DROP
 *      bit 25     the protocol range contains 6 (TCP)       bit 26 contains 17 (UDP)
 *      bit 27     sip is a /32 (exact compare)              bit 28 dip is a /32
 *      bit 29     NOHIT: the sentinel (hit -1; bit 24 = the default action is DROP)
 *  compact record (4 words, 16 B, by slot; slot n_rules = the sentinel, matching every TCP / UDP key):
 *      sip: prefix | 1 << (31 - len) for len 0..31 (the lowest set bit marks the prefix end), the address for a /32
 *      dip: likewise;  sport_lo | dport_lo << 16;  (sport_hi - sport_lo) | (dport_hi - dport_lo) << 16
 *      The address matches iff (key ^ word) has no bit set above the marker bit (every bit for a /32).
 *  idtab (word 20 != 0): n_rules words, the rule index of each slot (when unused entries make slots != indices)
 *
 *  cut-list section (v8; present iff word 22 != 0: every rule without residual MAC / time fields).  A second,
 *  independent classifier for the classify kernel (TCP / UDP keys only): a HyperCuts-style cut of the top b0 bits
 *  of sip and the top b1 bits of dip into 2^(b0 + b1) buckets, bucket = (sip >> (32 - b0)) << b1 | dip >> (32 - b1)
 *  (b0 >= 3, b1 >= 2), and per bucket the list of the rules whose box meets it, in priority order, closed after the first
 *  rule that covers the whole bucket (every port, TCP and UDP).  The builder picks b0, b1 (b0 + b1 <= 16) by the
 *  expected list length (strongly preferring a cut whose groups, entries and ids fit half a CU's LDS) and rejects the
 *  section when a list would exceed 15 entries.  A lookup is one read of the bucket's group and one round of
 *  independent 16-B entry reads (LDS, or L2 for large sets): no dependent walk; a match reads its rule id.
 *      header (16 words at off_cut): b0 | b1 << 8 | PPE_CUT_IDS16, n_buckets, n_entries, max list length,
 *          off_slc, off_ent, n_groups, epl (entries per line), off_gbase, off_fp (word offsets from the image start),
 *          div (e / epl = umulhi(e, div) for e < 2^25), n_lines, off_id (0 with PPE_CUT_LINES), 0...
 *      groups of 32 buckets (group g = buckets 32 g .. 32 g + 31): slices (4 words, 16-B aligned, at off_slc + 4 g):
 *          bit k of word i = bit i of bucket 32 g + k's list length (0..15); base (1 word, at off_gbase + g): the
 *          group's first entry.  Bucket b's list = entries [first(b), first(b) + len(b)), first(b) = base +
 *          sum over i of 2^i popcount(slice i & (2^(b mod 32) - 1)).
 *      fingerprints (4 bits per entry, entry e at bits 4 (e mod 8) of word off_fp + e / 8; two spare words after):
 *          bit 0 = the rule's sip bit 31 - b0 (the first below the cut), bit 1 = its prefix fixes that bit, bits 2 / 3
 *          likewise for dip bit 31 - b1.  A lookup skips an entry whose fixed bits differ from the key's (it cannot
 *          match), so most entries that would not match are never read.
  *      entry lines (128 B each, 128-B aligned, at off_ent): epl entries (16 B each, entry e in line e / epl at slot
 *          e mod epl; contiguous per bucket in priority order).  PPE_CUT_LINES (cuts read from L2): then the line's
 *          rule ids (a matching entry's id shares its line: read right after it, from L1), epl = 7 with 16-bit ids,
 *          6 with 32-bit ids.  Otherwise (cuts that fit LDS) epl = 8 and the ids follow the last line, one per entry
 *          (at off_id).  16-bit ids when PPE_CUT_IDS16 (every index < 2^16), else 32-bit.  An entry:
 *          sip relative to the bucket | DROP | TCP: the prefix's bits below the top b0, shifted up by b0, then a
 *              marker bit (so the bits above the lowest set bit of the word without bits 0-1 must equal the key's
 *              sip << b0); a /32 puts the marker at bit b0 - 1 (>= 2); a prefix of at most b0 bits matches the whole
 *              bucket: 0x80000000.  Bit 0: the rule's protocol range contains 6; bit 1: its action is
 *              ACL_RULE_ACTION_DROP (the verdict needs no id read).
 *          dip relative to the bucket | UDP (bit 0: contains 17), likewise with b1 (marker at bit >= 1)
 *          sport_lo | dport_lo << 16;  (sport_hi - sport_lo) | (dport_hi - dport_lo) << 16
  */
#ifndef PPE_IMAGE_H
#define PPE_IMAGE_H

#define PPE_IMG_MAGIC   0x41455050u /* "PPEA" */
#define PPE_IMG_VERSION 8u
#define PPE_IMG_HDR_WORDS 32u

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
#define PPE_IMG_W_ROOTKS   13
#define PPE_IMG_W_JUMP     14
#define PPE_IMG_W_OFFBSEC  15
#define PPE_IMG_W_NBLOCKS  16
#define PPE_IMG_W_OFFBLOCKS 17
#define PPE_IMG_W_MAXBDEPTH 18
#define PPE_IMG_W_OFFCREC  19
#define PPE_IMG_W_OFFIDTAB 20
#define PPE_IMG_W_BLKLV    21
#define PPE_IMG_W_OFFCUT   22

#define PPE_BLK_WORDS 8u           /* 2-level block */
#define PPE_BLK_LEAF 0x80000000u  /* exit word: a leaf payload (else a block index) */
#define PPE_CX_SLOT   0x00ffffffu  /* compact leaf exit fields (v6) */
#define PPE_CX_DROP   (1u << 24)
#define PPE_CX_TCP    (1u << 25)
#define PPE_CX_UDP    (1u << 26)
#define PPE_CX_S32    (1u << 27)
#define PPE_CX_D32    (1u << 28)
#define PPE_CX_NOHIT  (1u << 29)
#define PPE_CREC_WORDS 4u
#define PPE_CUT_HDR_WORDS 16u
#define PPE_CUT_ENT_WORDS 4u      /* cut-list entry (16 B) */
#define PPE_CUT_LINE_WORDS 32u    /* cut-list entry line (128 B) */
#define PPE_CUT_IDS16 0x10000u    /* cut header word 0: 16-bit rule ids */
#define PPE_CUT_LINES 0x20000u    /* cut header word 0: rule ids inside the entry lines */
#define PPE_CUT_MAX_LIST 15u      /* longest bucket list (4-bit lengths) */
#define PPE_CUT_MAX_BITS 16u      /* b0 + b1: 2^16 buckets = 64 KB of groups */

#define PPE_NODE_WORDS 4u
#define PPE_NODE_LEAF 5u          /* key slot of a leaf: the walk's zero key */
#define PPE_LEAF_THR 0xffffffffu  /* threshold word of a leaf */
#define PPE_NODE_MAX (1u << 20)   /* node budget: child byte offsets stay below 16 MiB */
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

/* hard bound on walk length, enforced by the builder (max_depth) */
#define PPE_MAX_DEPTH 60

#endif
