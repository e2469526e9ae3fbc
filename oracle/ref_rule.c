/* TEST INFRASTRUCTURE ONLY: storage for the reference's own rule store and '@' rule-file parser
 * (rule/rule.c + ipc/msgque.c, compiled unmodified from the reference tree by oracle/Makefile into
 * _ref/libref_rule.so).  Those two files need only the globals the reference defines elsewhere:
 *   rule_list        mgrplane/src/srv/srvnet/srv_rule.c:15 (mapped from POSIX shm there, :56-89; calloc here)
 *   dp_msg_queue_id  dataplane/src/common/dp_cmd.c:32      (only Rule_Notify_Dp_Build*, never called here)
 *   srv_dp_sync      dataplane/src/platform/oct-init.c:502 (idem)
 * tests/golden/gen_rule_golden.py drives Rule_Load_Line / Rule_add / Rule_del_by_id / Rule_duplicate_check /
 * Rule_del_all through ctypes and freezes the resulting rule_list_t images as fixtures for tests/test_rules.py. */
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#include "acl_rule.h"
#include "shm.h"

rule_list_t *rule_list;
int dp_msg_queue_id;
SRV_DP_SYNC *srv_dp_sync;

/* Rule_list_init's state after its memset (srv_rule.c:82-86); the zeroed mutex is glibc's default initializer */
int ref_rule_list_init(void) {
    if (!rule_list) rule_list = (rule_list_t *)malloc(sizeof(rule_list_t));
    if (!rule_list) return -1;
    memset(rule_list, 0, sizeof(rule_list_t));
    rule_list->rule_def_act = ACL_RULE_ACTION_DROP;
    rule_list->rule_entry_free = RULE_ENTRY_MAX;
    rule_list->build_status = RULE_BUILD_COMMIT;
    return 0;
}

void ref_rule_list_free(void) {
    free(rule_list);
    rule_list = NULL;
}

unsigned long ref_rule_list_size(void) { return sizeof(rule_list_t); }
