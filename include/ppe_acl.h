/*
 * ppe_acl.h — PPE-compatible ACL rule model, rule store and ACL engine API.
 *
 * Drop-in surface for the reference's ACL path (royhunter/Packet-Process-Engine):
 *   - RCP_BLOCK_ACL_RULE_TUPLE   packed 60-B rule tuple       include/rpc-common.h:97-114
 *   - rule_entry_t / rule_list_t 10,000-entry rule store      include/acl_rule.h:27-41
 *   - ACL_RULE_ACTION_*, RULE_*  codes                        include/acl_rule.h:8-25
 *   - Rule_add / Rule_del_by_id / Rule_del_all /
 *     Rule_duplicate_check / Rule_Load_Line                   include/rule.h:25-31, rule/rule.c:176-431
 *   - DP_Acl_Rule_Init / DP_Acl_Load_Rule / DP_Acl_Rule_Clean /
 *     DP_Acl_Rule_Release / DP_Acl_Lookup / dp_acl_action_default
 *                                                             main.c:177, dataplane/src/common/dp_cmd.c:1963-2062,
 *                                                             dataplane/src/flow/flow.c:232,
 *                                                             dataplane/src/platform/oct-init.c:19,755
 *   - tree statistics gWstDepth/gAvgDepth/gChildCount/gNumTreeNode/gNumLeafNode
 *                                                             dataplane/src/common/dp_cmd.c:2032-2036
 *
 * The reference's ACL engine sources (dp_acl.c, acl64.c, dp_acl.h; built by dataplane/src/acl/acl.mk:13-15)
 * are absent from the reference tree, so the match semantics are defined here and frozen
 * by the golden fixtures under tests/golden/.  The classifier behind this API is a HyperSplit-style decision
 * tree built on the host and walked by the HIP kernel on the GPU.
 *
 * Plain C, no C++ or torch types across the boundary.
 */
#ifndef PPE_ACL_H
#define PPE_ACL_H

#include <stdint.h>
#include <stdio.h>
#include <pthread.h>

#include "ppe_rwlock.h"

#ifdef __cplusplus
extern "C" {
#endif

/* include/acl_rule.h:8 — the reference's fixed store size.  The extended store (ppe_rule_store_*) lifts it. */
#define RULE_ENTRY_MAX 10000

#define RULE_ENTRY_STATUS_FREE 0
#define RULE_ENTRY_STATUS_USED 1

#define RULE_BUILD_UNCOMMIT 0
#define RULE_BUILD_COMMIT   1

#define ACL_RULE_ACTION_FW   0
#define ACL_RULE_ACTION_DROP 1

#define RULE_OK        0
#define RULE_FULL      1
#define RULE_EXIST     2
#define RULE_NOT_EXIST 3

/* dataplane/src/include/sec-common.h:19-20 */
#ifndef SEC_OK
#define SEC_OK 0
#define SEC_NO 1
#endif

/* include/rpc-common.h:97-114 — 60 bytes, packed, host byte order.  IPs are numeric a<<24|b<<16|c<<8|d
 * (rule/rule.c:58-61); sip_mask/dip_mask are prefix LENGTHS 0..32; ports/protocol are inclusive ranges;
 * time (0,0) = any; all-zero MAC = any. */
typedef struct tag_RCP_BLOCK_ACL_RULE_TUPLE {
    uint64_t time_start;
    uint64_t time_end;
    uint8_t  smac[6];
    uint8_t  dmac[6];
    uint16_t sport_start;
    uint16_t sport_end;
    uint32_t sip;
    uint32_t dip;
    uint32_t sip_mask;
    uint32_t dip_mask;
    uint16_t dport_start;
    uint16_t dport_end;
    uint8_t  protocol_start;
    uint8_t  protocol_end;
    uint16_t action;
    uint32_t logable;
} __attribute__((__packed__)) RCP_BLOCK_ACL_RULE_TUPLE;

/* include/acl_rule.h:27-30 */
typedef struct {
    int8_t entry_status;
    RCP_BLOCK_ACL_RULE_TUPLE rule_tuple;
} rule_entry_t;

/* include/acl_rule.h:34-41 — ABI-compatible with the reference's POSIX-shm "RULE_LIST_SPACE" block. */
typedef struct {
    uint32_t rule_def_act;
    int rule_entry_free;
    int build_status;
    pthread_mutex_t rulelist_mutex;
    rule_entry_t rule_entry[RULE_ENTRY_MAX];
} rule_list_t;

/* The process-wide rule list the Rule_* functions operate on (include/acl_rule.h:43).  ppe_rule_list_init()
 * allocates it in process memory (the reference maps it from POSIX shm, mgrplane/src/srv/srvnet/srv_rule.c:56-89). */
extern rule_list_t *rule_list;

/* Opaque double-buffer halves of the running classifier (dataplane/src/common/dp_cmd.c:1963-1985). */
typedef struct ppe_tree_set  TreeSet;
typedef struct ppe_tree_node TreeNode;
typedef struct {
    TreeSet  *TreeSet;
    TreeNode *TreeNode;
} unit_tree_t;

/* The pair dp_cmd.c switches between (get_back_acltree / set_running_acltree, dp_cmd.c:1963-1985), owned here as the
 * absent ACL engine owned them: DP_Acl_Load_Rule(rl, &back->TreeSet, &back->TreeNode) builds and uploads the back
 * classifier without publishing it; g_acltree_running := &back (under acltree_running_rwlock) makes it the one the
 * next classify step and DP_Acl_Lookup use.  DP_Acl_Rule_Commit runs the whole protocol on this pair. */
extern unit_tree_t g_acltree_1, g_acltree_2;
extern unsigned long g_acltree_running;
extern rwlock_t acltree_running_rwlock;

/* ---- rule store (include/rule.h:25-31, rule/rule.c) ---- */
int  ppe_rule_list_init(void);          /* zeroed list, def_act DROP, build_status COMMIT (srv_rule.c:82-86) */
void ppe_rule_list_free(void);
int  Rule_add(RCP_BLOCK_ACL_RULE_TUPLE *rule, uint32_t *ruleid);
int  Rule_del_by_id(uint32_t id);
int  Rule_del_all(void);
int  Rule_duplicate_check(RCP_BLOCK_ACL_RULE_TUPLE *rule);
/* rule/rule.c:194-347: read the next '@' rule line from fp and Rule_add it.  Returns 0 on success or when no
 * rule line remains, -1 on a malformed line.  MACs are read as %2x hex (rule/rule.c:114). */
int  Rule_Load_Line(FILE *fp, int line);
/* Convenience: load every rule line of a file; returns the number of rules added or -1. */
int  ppe_rule_load_file(const char *path);

/* ---- ACL engine (reconstructed from call sites) ---- */
extern uint32_t dp_acl_action_default;     /* dataplane/src/common/dp_cmd.c:2062 */
extern int      gWstDepth;                 /* dataplane/src/common/dp_cmd.c:2032-2036 */
extern int      gAvgDepth;
extern int      gChildCount;
extern int      gNumTreeNode;
extern int      gNumLeafNode;

/* main.c:177 — create the engine context on the default device (PPE_DEVICE env, default 0). SEC_OK/SEC_NO. */
int      DP_Acl_Rule_Init(void);
/* dataplane/src/common/dp_cmd.c:2019 — build the classifier from every USED entry of rl into the given
 * double-buffer half and upload it to the GPU.  Returns SEC_OK on success. */
uint32_t DP_Acl_Load_Rule(rule_list_t *rl, TreeSet **tset, TreeNode **tnode);
/* dataplane/src/common/dp_cmd.c:2030 — free a (non-running) double-buffer half. */
void     DP_Acl_Rule_Clean(TreeSet **tset, TreeNode **tnode);
/* dataplane/src/platform/oct-init.c:755 */
void     DP_Acl_Rule_Release(void);
/* dp_acl_rule_commit equivalent (dataplane/src/common/dp_cmd.c:1987-2053): build into the back half, publish it
 * as running (pointer swap at a batch boundary), clean the old half, set build_status = COMMIT.
 * Returns SEC_OK / SEC_NO. */
int      DP_Acl_Rule_Commit(void);

#ifdef __cplusplus
}
#endif
#endif /* PPE_ACL_H */
