/*
 * ppe_rwlock.h — the reference's platform reader / writer spin lock (dataplane/src/platform/rwlock.h: MIPS ll / sc
 * assembly on Octeon) with the compiler's atomic builtins, for a host build of dp_cmd.c's running-tree switch
 * (set_running_acltree, dp_cmd.c:1980-1985) against include/ppe_acl.h.  Same names, same lock word (readers count up
 * from 0, a writer holds bit 31), same trylock result (1 = acquired).  A host port includes this where the reference
 * includes "rwlock.h".
 */
#ifndef PPE_RWLOCK_H
#define PPE_RWLOCK_H

typedef struct {
    volatile unsigned int lock;
} rwlock_t;

#define PPE_RWLOCK_INITIALIZER {0u}

static inline void rwlock_init(rwlock_t *rw) { __atomic_store_n(&rw->lock, 0u, __ATOMIC_RELEASE); }
static inline int read_trylock(rwlock_t *rw) {
    unsigned int v = __atomic_load_n(&rw->lock, __ATOMIC_RELAXED);
    while (!(v & 0x80000000u))
        if (__atomic_compare_exchange_n(&rw->lock, &v, v + 1u, 1, __ATOMIC_ACQUIRE, __ATOMIC_RELAXED)) return 1;
    return 0;
}
static inline void read_lock(rwlock_t *rw) {
    while (!read_trylock(rw)) __builtin_ia32_pause();
}
static inline void read_unlock(rwlock_t *rw) { (void)__atomic_fetch_sub(&rw->lock, 1u, __ATOMIC_RELEASE); }
static inline int write_trylock(rwlock_t *rw) {
    unsigned int v = 0u;
    const int ok = __atomic_compare_exchange_n(&rw->lock, &v, 0x80000000u, 0, __ATOMIC_ACQUIRE, __ATOMIC_RELAXED);
    return ok;
}
static inline void write_lock(rwlock_t *rw) {
    while (!write_trylock(rw)) __builtin_ia32_pause();
}
static inline void write_unlock(rwlock_t *rw) { __atomic_store_n(&rw->lock, 0u, __ATOMIC_RELEASE); }

#endif
