/*
 * rule_store.c — the PPE ACL rule store and '@' rule-file parser (include/rule.h, rule/rule.c).
 *
 * Same observable behaviour as the reference:
 *   - Rule_add        rule/rule.c:350-387  (FULL when no free entry, EXIST on a byte-identical USED tuple,
 *                                           first free index wins, build_status → UNCOMMIT, *ruleid = index)
 *   - Rule_del_by_id  rule/rule.c:389-414
 *   - Rule_del_all    rule/rule.c:176-192
 *   - Rule_duplicate_check rule/rule.c:416-431 (memcmp of the packed 60-B tuple)
 *   - Rule_Load_Line  rule/rule.c:194-347  (skip to '@', then smac dmac sip/len dip/len sp:sp dp:dp pr:pr
 *                                           t_start t_end action log; MACs as %2x hex)
 * The store lives in process memory (the reference maps it from POSIX shm, mgrplane/src/srv/srvnet/srv_rule.c:56-89).
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "ppe_acl.h"

rule_list_t *rule_list = NULL;

int ppe_rule_list_init(void) {
    if (rule_list) return 0;
    rule_list = (rule_list_t *)calloc(1, sizeof(rule_list_t));
    if (!rule_list) return -1;
    pthread_mutex_init(&rule_list->rulelist_mutex, NULL);
    rule_list->rule_def_act = ACL_RULE_ACTION_DROP;  /* srv_rule.c:84 */
    rule_list->rule_entry_free = RULE_ENTRY_MAX;     /* srv_rule.c:85 */
    rule_list->build_status = RULE_BUILD_COMMIT;     /* srv_rule.c:86 */
    return 0;
}

void ppe_rule_list_free(void) {
    if (!rule_list) return;
    pthread_mutex_destroy(&rule_list->rulelist_mutex);
    free(rule_list);
    rule_list = NULL;
}

static int first_free_entry(void) {
    for (int i = 0; i < RULE_ENTRY_MAX; i++)
        if (rule_list->rule_entry[i].entry_status == RULE_ENTRY_STATUS_FREE) return i;
    return -1;
}

/* caller holds the mutex */
static int duplicate_locked(const RCP_BLOCK_ACL_RULE_TUPLE *rule) {
    for (int i = 0; i < RULE_ENTRY_MAX; i++) {
        if (rule_list->rule_entry[i].entry_status == RULE_ENTRY_STATUS_FREE) continue;
        if (memcmp(rule, &rule_list->rule_entry[i].rule_tuple, sizeof(RCP_BLOCK_ACL_RULE_TUPLE)) == 0)
            return RULE_EXIST;
    }
    return RULE_OK;
}

int Rule_duplicate_check(RCP_BLOCK_ACL_RULE_TUPLE *rule) {
    if (!rule_list || !rule) return RULE_OK;
    return duplicate_locked(rule);
}

int Rule_add(RCP_BLOCK_ACL_RULE_TUPLE *rule, uint32_t *ruleid) {
    if (!rule_list && ppe_rule_list_init() != 0) return RULE_FULL;
    pthread_mutex_lock(&rule_list->rulelist_mutex);
    if (rule_list->rule_entry_free == 0) {
        pthread_mutex_unlock(&rule_list->rulelist_mutex);
        return RULE_FULL;
    }
    if (duplicate_locked(rule) == RULE_EXIST) {
        pthread_mutex_unlock(&rule_list->rulelist_mutex);
        return RULE_EXIST;
    }
    const int idx = first_free_entry();
    if (idx < 0) {
        pthread_mutex_unlock(&rule_list->rulelist_mutex);
        return RULE_FULL;
    }
    memcpy(&rule_list->rule_entry[idx].rule_tuple, rule, sizeof(RCP_BLOCK_ACL_RULE_TUPLE));
    rule_list->rule_entry_free--;
    rule_list->rule_entry[idx].entry_status = RULE_ENTRY_STATUS_USED;
    rule_list->build_status = RULE_BUILD_UNCOMMIT;
    pthread_mutex_unlock(&rule_list->rulelist_mutex);
    if (ruleid) *ruleid = (uint32_t)idx;
    return RULE_OK;
}

int Rule_del_by_id(uint32_t id) {
    if (!rule_list) return RULE_NOT_EXIST;
    pthread_mutex_lock(&rule_list->rulelist_mutex);
    int rc = RULE_OK;
    if (rule_list->rule_entry_free == RULE_ENTRY_MAX || id >= RULE_ENTRY_MAX ||
        rule_list->rule_entry[id].entry_status == RULE_ENTRY_STATUS_FREE) {
        rc = RULE_NOT_EXIST;
    } else {
        rule_list->rule_entry[id].entry_status = RULE_ENTRY_STATUS_FREE;
        rule_list->rule_entry_free++;
        rule_list->build_status = RULE_BUILD_UNCOMMIT;
    }
    pthread_mutex_unlock(&rule_list->rulelist_mutex);
    return rc;
}

int Rule_del_all(void) {
    if (!rule_list && ppe_rule_list_init() != 0) return RULE_OK;
    pthread_mutex_lock(&rule_list->rulelist_mutex);
    for (int i = 0; i < RULE_ENTRY_MAX; i++) rule_list->rule_entry[i].entry_status = RULE_ENTRY_STATUS_FREE;
    rule_list->rule_entry_free = RULE_ENTRY_MAX;
    rule_list->build_status = RULE_BUILD_UNCOMMIT;
    pthread_mutex_unlock(&rule_list->rulelist_mutex);
    return RULE_OK;
}

/* ---- '@' rule line parser: field readers follow rule/rule.c:27-173 ---- */

/* The reference reads every number with %d into an unsigned int (rule/rule.c:34,52,85,100): glibc converts with
 * strtol (saturating at LONG_MAX / LONG_MIN) and stores the low 32 bits.  %d into an int and a cast give the same bits
 * for every input, %u does not (it converts with strtoul: "9223372036854775808" is 0 there, 0xffffffff here).
 * Pinned against the reference's own rule.c by tests/test_rules.py (tests/golden/ref_rule_v1.npz). */
static int read_ip(FILE *fp, uint32_t *ip_out, uint32_t *mask_out) {
    int o[4], mask;
    char slash;
    if (fscanf(fp, "%d.%d.%d.%d", &o[0], &o[1], &o[2], &o[3]) != 4) return -1;
    if (fscanf(fp, "%c", &slash) != 1 || slash != '/') return -1;
    if (fscanf(fp, "%d", &mask) != 1) return -1;
    /* octets are shifted and OR'ed without range checks (rule/rule.c:58-61) */
    const uint32_t ip = ((uint32_t)o[0] << 24) | ((uint32_t)o[1] << 16) | ((uint32_t)o[2] << 8) | (uint32_t)o[3];
    if (ip == 0 && mask != 0) return -1;            /* rule/rule.c:63-68 */
    if (ip != 0 && (uint32_t)mask > 32u) return -1; /* rule/rule.c:69-73 (an unsigned compare there) */
    *ip_out = ip;
    *mask_out = (uint32_t)mask;
    return 0;
}

static int read_range(FILE *fp, unsigned int *from, unsigned int *to) {
    int a, b;
    if (fscanf(fp, "%d : %d", &a, &b) != 2) return -1;
    *from = (unsigned int)a;
    *to = (unsigned int)b;
    return 0;
}

static int read_mac(FILE *fp, uint8_t *mac) {
    unsigned int m[6];
    if (fscanf(fp, "%2x:%2x:%2x:%2x:%2x:%2x", &m[0], &m[1], &m[2], &m[3], &m[4], &m[5]) != 6) return -1;
    for (int i = 0; i < 6; i++) mac[i] = (uint8_t)m[i];
    return 0;
}

int Rule_Load_Line(FILE *fp, int line) {
    (void)line;
    RCP_BLOCK_ACL_RULE_TUPLE r;
    memset(&r, 0, sizeof r);
    int ch;
    while ((ch = fgetc(fp)) != EOF) {
        if (ch != '@') continue;  /* each rule begins with '@' (rule/rule.c:210-213) */
        unsigned int a, b;
        long t0, t1;
        int action, logable;
        if (read_mac(fp, r.smac) || read_mac(fp, r.dmac)) return -1;
        uint32_t ip, mask;
        if (read_ip(fp, &ip, &mask)) return -1;
        r.sip = ip;
        r.sip_mask = mask;
        if (read_ip(fp, &ip, &mask)) return -1;
        r.dip = ip;
        r.dip_mask = mask;
        if (read_range(fp, &a, &b)) return -1;
        r.sport_start = (uint16_t)a;
        r.sport_end = (uint16_t)b;
        if (r.sport_start > r.sport_end) return -1;
        if (read_range(fp, &a, &b)) return -1;
        r.dport_start = (uint16_t)a;
        r.dport_end = (uint16_t)b;
        if (r.dport_start > r.dport_end) return -1;
        if (read_range(fp, &a, &b)) return -1;
        r.protocol_start = (uint8_t)a;
        r.protocol_end = (uint8_t)b;
        if (r.protocol_start > r.protocol_end) return -1;
        if (fscanf(fp, "%ld", &t0) != 1 || fscanf(fp, "%ld", &t1) != 1) return -1;
        r.time_start = (uint64_t)t0;
        r.time_end = (uint64_t)t1;
        if (fscanf(fp, "%d", &action) != 1) return -1;
        /* ReadActionInfo stores the int into the uint16_t field first (rule/rule.c:146-158) and the 0/1 check reads
         * the narrowed field (rule/rule.c:320-324): "65537" is accepted as action 1 */
        r.action = (uint16_t)action;
        if (r.action != 0 && r.action != 1) return -1;
        if (fscanf(fp, "%d", &logable) != 1) return -1;
        if (logable != 0 && logable != 1) return -1;  /* rule/rule.c:334-338 */
        r.logable = (uint32_t)logable;
        uint32_t id;
        Rule_add(&r, &id);  /* result ignored, as in rule/rule.c:341 */
        return 0;
    }
    return 0;
}

int ppe_rule_load_file(const char *path) {
    FILE *fp = fopen(path, "r");
    if (!fp) return -1;
    if (!rule_list && ppe_rule_list_init() != 0) {
        fclose(fp);
        return -1;
    }
    const int before = RULE_ENTRY_MAX - rule_list->rule_entry_free;
    int line = 0, rc = 0;
    while (!feof(fp)) {
        long pos = ftell(fp);
        if (Rule_Load_Line(fp, ++line) != 0) {
            rc = -1;
            break;
        }
        if (ftell(fp) == pos) break;
    }
    fclose(fp);
    if (rc) return -1;
    return (RULE_ENTRY_MAX - rule_list->rule_entry_free) - before;
}
