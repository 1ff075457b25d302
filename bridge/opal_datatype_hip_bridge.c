/*
 * opal_datatype_hip_bridge.c -- Open MPI's convertor slots served by the MI355X engine.
 *
 * What the maintainer's copy of this file does inside opal/datatype/ (INTEGRATION.md §1):
 *   - opal_hip_bridge_attach() runs right after OPAL_CONVERTOR_PREPARE in
 *     opal_convertor_prepare_for_{send,recv} (opal_convertor.c:616-696) for accelerator
 *     convertors and installs fAdvance / fPosition, the way pack_description_sweep.c:877-965
 *     swaps the movers of a prepared convertor;
 *   - each committed opal_datatype_t is imported once (ddt_type_from_opal_desc on the
 *     convertor's use_desc, opal_convertor.c:533) into a cache keyed by the datatype
 *     pointer and a fingerprint of the description, dropped by
 *     opal_hip_bridge_datatype_destruct() from opal_datatype_destruct;
 *   - every fAdvance call resumes the engine at conv->bConverted (the engine's whole resume
 *     state), moves the iovecs, and writes bConverted / CONVERTOR_COMPLETED back with the
 *     return-code contract of opal_pack_accelerator_simple (_pack_accelerator.c:276-294)
 *     and opal_unpack_accelerator_simple (_unpack_accelerator.c:355-367).
 *
 * Engine convertors are per thread (the reference's contract is one thread per
 * convertor, opal_convertor.h:125; a thread serves many opal convertors in turn), so the
 * bridge keeps no per-convertor side table that could outlive an opal_convertor_t.
 */
#include <pthread.h>
#include <sched.h>
#include <stdlib.h>
#include <string.h>

#include "ddt_hip.h"
#include "opal_hip_bridge.h"

/* ------------------------------------------------------------------ import cache
 * Every fAdvance / fPosition / attach looks its datatype up here, from any thread.  Round 6
 * (scripts/bridgethreads.c, profiles/r6_threads.jsonl): one process-wide pthread mutex taken
 * twice per lookup convoyed under MPI_THREAD_MULTIPLE (4 threads: 5.4 us per call against 2.8
 * through the engine's own ABI), so each bucket has its own short spin lock -- threads moving
 * different datatypes never meet, and the critical sections are a few loads long -- and the
 * counters are atomics. */
typedef struct bridge_entry {
    const opal_datatype_t *key;
    const dt_elem_desc_t *desc;   /* fingerprint: the description the import was made from */
    size_t used, size;
    ptrdiff_t lb, ub, true_lb, true_ub;
    uint64_t sig;
    ddt_datatype_t *type;
    /* calls between bridge_type_of and bridge_release; an entry unlinked by a destruct or a
     * stale-address eviction while calls still use it is freed by the last of them */
    size_t inflight;
    int unlinked;
    unsigned bucket;
    struct bridge_entry *next;
} bridge_entry;

#define BRIDGE_BUCKETS 256
typedef struct {
    int lock;   /* 0 free, 1 held: __atomic test-and-set */
    bridge_entry *head;
} bridge_bucket;
static bridge_bucket g_buckets[BRIDGE_BUCKETS];
static size_t g_entries, g_imports, g_hits, g_stale;   /* __atomic counters */
/* bumped whenever an entry is unlinked: a thread's pinned entries (thread_state below) are
 * valid while it has not moved */
static unsigned long g_gen;

static void bucket_lock(bridge_bucket *b)
{
    for (unsigned spins = 0; __atomic_exchange_n(&b->lock, 1, __ATOMIC_ACQUIRE); ++spins) {
        while (__atomic_load_n(&b->lock, __ATOMIC_RELAXED)) {
            if (++spins > 256)
                sched_yield();   /* oversubscribed: let the holder run */
            else
                __builtin_ia32_pause();
        }
    }
}

static void bucket_unlock(bridge_bucket *b) { __atomic_store_n(&b->lock, 0, __ATOMIC_RELEASE); }

static void count(size_t *c, long d) { __atomic_fetch_add(c, (size_t) d, __ATOMIC_RELAXED); }

static unsigned bucket_of(const void *p)
{
    uintptr_t x = (uintptr_t) p;
    x ^= x >> 17;
    x *= 0x9E3779B97F4A7C15ull;
    return (unsigned) ((x >> 56) % BRIDGE_BUCKETS);
}

/* A 64-bit mix over the first and last (up to) 8 entries, 8 bytes at a time: catches a
 * different description that happens to sit at a recycled address without an O(entries) hash
 * per call. */
static uint64_t desc_sig(const dt_elem_desc_t *d, size_t used)
{
    uint64_t h = 0x9E3779B97F4A7C15ull ^ used;
    const size_t head = used < 8 ? used : 8;
    const size_t tail0 = used > head + 8 ? used - 8 : head;
    for (size_t r = 0; r < 2; ++r) {
        const size_t i0 = r ? tail0 : 0, i1 = r ? used : head;
        const unsigned char *b = (const unsigned char *) (d + i0);
        for (size_t k = 0; k < 32 * (i1 - i0); k += 8) {
            uint64_t w;
            memcpy(&w, b + k, 8);
            h = (h ^ w) * 0xBF58476D1CE4E5B9ull;
            h ^= h >> 31;
        }
    }
    return h;
}

static int same_fingerprint(const bridge_entry *e, const opal_datatype_t *dt, const dt_type_desc_t *ud,
                            uint64_t sig)
{
    return e->desc == ud->desc && e->used == ud->used && e->size == dt->size && e->lb == dt->lb
           && e->ub == dt->ub && e->true_lb == dt->true_lb && e->true_ub == dt->true_ub && e->sig == sig;
}

/* Called with the entry's bucket locked, on an entry already taken off the bucket list.  Returns
 * the entry when the caller must free it after unlocking (no call uses it), else NULL. */
static bridge_entry *retire_locked(bridge_entry *e)
{
    __atomic_fetch_add(&g_gen, 1, __ATOMIC_SEQ_CST);   /* before inflight is read: see thread_state */
    count(&g_entries, -1);
    if (e->inflight) {   /* a call on another thread still moves data with it */
        e->unlinked = 1;
        return NULL;
    }
    return e;
}

static void free_entry(bridge_entry *e)
{
    if (!e)
        return;
    ddt_type_destroy(&e->type);
    free(e);
}

static void bridge_release(bridge_entry *e)
{
    bridge_bucket *b = &g_buckets[e->bucket];
    bucket_lock(b);
    const int last = --e->inflight == 0 && e->unlinked;
    bucket_unlock(b);
    if (last)
        free_entry(e);
}

/* The entry of (dt, ud) in its bucket, bucket locked; a different description found at the same
 * address is unlinked on the way (the old datatype died unseen) and handed back in *dead. */
static bridge_entry *lookup_locked(bridge_bucket *b, const opal_datatype_t *dt, const dt_type_desc_t *ud,
                                   uint64_t sig, bridge_entry **dead)
{
    for (bridge_entry **pp = &b->head; *pp;) {
        if ((*pp)->key != dt) {
            pp = &(*pp)->next;
            continue;
        }
        if (same_fingerprint(*pp, dt, ud, sig))
            return *pp;
        bridge_entry *old = *pp;
        *pp = old->next;
        count(&g_stale, 1);
        bridge_entry *f = retire_locked(old);
        if (f) {   /* at most a few stale entries: chain them for the caller to free */
            f->next = *dead;
            *dead = f;
        }
    }
    return NULL;
}

static void free_chain(bridge_entry *d)
{
    while (d) {
        bridge_entry *n = d->next;
        free_entry(d);
        d = n;
    }
}

/* The cache entry of (dt, ud), imported on first use.  `hold`: keep it for the caller until
 * bridge_release (a destruct or an eviction on another thread in between only unlinks it).
 * The import itself -- seconds for a description of tens of millions of entries -- runs
 * outside the bucket lock, so other threads' calls never wait for it; two threads importing
 * the same datatype at once keep the first entry and drop the second. */
static bridge_entry *bridge_entry_of(const opal_datatype_t *dt, const dt_type_desc_t *ud, int hold, int *err)
{
    *err = OPAL_SUCCESS;
    if (!dt || !ud || !ud->desc || !(dt->flags & OPAL_DATATYPE_FLAG_COMMITTED)) {
        *err = OPAL_ERR_BAD_PARAM;
        return NULL;
    }
    const uint64_t sig = desc_sig(ud->desc, ud->used);
    const unsigned bi = bucket_of(dt);
    bridge_bucket *bk = &g_buckets[bi];
    bridge_entry *dead = NULL;
    bucket_lock(bk);
    bridge_entry *e = lookup_locked(bk, dt, ud, sig, &dead);
    if (e) {
        if (hold)
            ++e->inflight;
        bucket_unlock(bk);
        count(&g_hits, 1);
        free_chain(dead);
        return e;
    }
    bucket_unlock(bk);
    free_chain(dead);
    dead = NULL;

    ddt_datatype_t *t = NULL;
    const int rc = ddt_type_from_opal_desc(ud->desc, ud->used, dt->size, dt->lb, dt->ub, dt->true_lb,
                                           dt->true_ub, &t);
    if (rc != DDT_SUCCESS) {
        *err = rc == DDT_ERR_OUT_OF_RESOURCE ? OPAL_ERR_OUT_OF_RESOURCE : OPAL_ERR_BAD_PARAM;
        return NULL;
    }
    /* the import is this datatype's commit on the device side: a large index list gets its
     * address-ordered tables here (at commit or prepare), never in the first fAdvance */
    (void) ddt_type_prepare_device(t);
    bridge_entry *n = (bridge_entry *) calloc(1, sizeof(*n));
    if (!n) {
        ddt_type_destroy(&t);
        *err = OPAL_ERR_OUT_OF_RESOURCE;
        return NULL;
    }
    n->key = dt;
    n->desc = ud->desc;
    n->used = ud->used;
    n->size = dt->size;
    n->lb = dt->lb;
    n->ub = dt->ub;
    n->true_lb = dt->true_lb;
    n->true_ub = dt->true_ub;
    n->sig = sig;
    n->type = t;
    n->bucket = bi;

    bucket_lock(bk);
    e = lookup_locked(bk, dt, ud, sig, &dead);
    if (e) {   /* another thread imported it meanwhile */
        if (hold)
            ++e->inflight;
        bucket_unlock(bk);
        count(&g_hits, 1);
        free_chain(dead);
        ddt_type_destroy(&n->type);
        free(n);
        return e;
    }
    n->inflight = hold ? 1 : 0;
    n->next = bk->head;
    bk->head = n;
    bucket_unlock(bk);
    count(&g_entries, 1);
    count(&g_imports, 1);
    free_chain(dead);
    return n;
}

static void unpin_current_thread(void);

int opal_hip_bridge_datatype_commit(const opal_datatype_t *dt)
{
    if (!dt || !(dt->flags & OPAL_DATATYPE_FLAG_COMMITTED) || !dt->opt_desc.desc || dt->opt_desc.used == 0
        || dt->opt_desc.used < OPAL_HIP_BRIDGE_COMMIT_IMPORT_MIN)
        return OPAL_SUCCESS;   /* nothing to move, or cheap enough to import at first use */
    int err;
    (void) bridge_entry_of(dt, &dt->opt_desc, 0, &err);
    return err;
}

void opal_hip_bridge_datatype_destruct(const opal_datatype_t *dt)
{
    bridge_bucket *bk = &g_buckets[bucket_of(dt)];
    bridge_entry *dead = NULL;
    bucket_lock(bk);
    for (bridge_entry **pp = &bk->head; *pp;) {
        if ((*pp)->key == dt) {
            bridge_entry *old = *pp;
            *pp = old->next;
            bridge_entry *f = retire_locked(old);
            if (f) {
                f->next = dead;
                dead = f;
            }
        } else {
            pp = &(*pp)->next;
        }
    }
    bucket_unlock(bk);
    free_chain(dead);
}

void opal_hip_bridge_finalize(void)
{
    unpin_current_thread();   /* other threads' pins go at their next call or exit */
    for (size_t b = 0; b < BRIDGE_BUCKETS; ++b) {
        bridge_bucket *bk = &g_buckets[b];
        bridge_entry *dead = NULL;
        bucket_lock(bk);
        while (bk->head) {
            bridge_entry *old = bk->head;
            bk->head = old->next;
            bridge_entry *f = retire_locked(old);
            if (f) {
                f->next = dead;
                dead = f;
            }
        }
        bucket_unlock(bk);
        free_chain(dead);
    }
}

static size_t pin_hits_total(void);

void opal_hip_bridge_stats(size_t *out4)
{
    out4[0] = __atomic_load_n(&g_entries, __ATOMIC_RELAXED);
    out4[1] = __atomic_load_n(&g_imports, __ATOMIC_RELAXED);
    out4[2] = __atomic_load_n(&g_hits, __ATOMIC_RELAXED) + pin_hits_total();
    out4[3] = __atomic_load_n(&g_stale, __ATOMIC_RELAXED);
}

void opal_hip_bridge_layout(size_t *out8)
{
    out8[0] = sizeof(opal_datatype_t);
    out8[1] = offsetof(opal_datatype_t, opt_desc);
    out8[2] = sizeof(opal_convertor_t);
    out8[3] = offsetof(opal_convertor_t, bConverted);
    out8[4] = offsetof(opal_convertor_t, flags);
    out8[5] = offsetof(opal_convertor_t, fPosition);
    out8[6] = offsetof(opal_convertor_t, stream);
    out8[7] = sizeof(dt_elem_desc_t);
}

/* ------------------------------------------------------------------ per-thread state
 * Engine convertors are per thread (the reference's contract is one thread per convertor,
 * opal_convertor.h:125; a thread serves many opal convertors in turn).  Each thread also pins
 * the cache entries of the last two datatypes it moved (one reference each, taken by a normal
 * lookup), so its next calls on them touch no shared cache line at all; a pin is dropped when
 * the cache generation moved (an entry was unlinked somewhere: a destruct or a stale address),
 * when the slot is reused, and at thread exit.  A destruct of a pinned datatype therefore frees
 * its engine import at the pinning thread's next bridge call or exit. */
#define PIN_SLOTS 2
typedef struct {
    bridge_entry *e;
    const opal_datatype_t *key;
    const dt_type_desc_t *ud;
    uint64_t sig;
    unsigned long gen;
    unsigned long used;   /* LRU tick */
} pin_slot;

typedef struct thread_state {
    ddt_convertor_t *h;
    pin_slot pin[PIN_SLOTS];
    unsigned long tick;
    size_t pin_hits;   /* lookups served by a pin: written by the owner, summed by the stats */
    struct thread_state *next, *prev;
} thread_state;

static pthread_key_t g_key;
static pthread_once_t g_once = PTHREAD_ONCE_INIT;
/* live thread states (for the stats), and the pin hits of threads that exited */
static pthread_mutex_t g_ts_mu = PTHREAD_MUTEX_INITIALIZER;
static thread_state *g_ts_head;
static size_t g_exited_pin_hits;

static void unpin_all(thread_state *ts)
{
    for (int i = 0; i < PIN_SLOTS; ++i)
        if (ts->pin[i].e) {
            bridge_release(ts->pin[i].e);
            ts->pin[i].e = NULL;
        }
}

static void state_free(void *p)
{
    thread_state *ts = (thread_state *) p;
    pthread_mutex_lock(&g_ts_mu);
    g_exited_pin_hits += __atomic_load_n(&ts->pin_hits, __ATOMIC_RELAXED);
    if (ts->prev)
        ts->prev->next = ts->next;
    else
        g_ts_head = ts->next;
    if (ts->next)
        ts->next->prev = ts->prev;
    pthread_mutex_unlock(&g_ts_mu);
    unpin_all(ts);
    if (ts->h)
        ddt_convertor_destroy(ts->h);
    free(ts);
}

static void key_init(void) { (void) pthread_key_create(&g_key, state_free); }

static size_t pin_hits_total(void)
{
    pthread_mutex_lock(&g_ts_mu);
    size_t n = g_exited_pin_hits;
    for (thread_state *t = g_ts_head; t; t = t->next)
        n += __atomic_load_n(&t->pin_hits, __ATOMIC_RELAXED);
    pthread_mutex_unlock(&g_ts_mu);
    return n;
}

static void unpin_current_thread(void)
{
    (void) pthread_once(&g_once, key_init);
    thread_state *ts = (thread_state *) pthread_getspecific(g_key);
    if (ts)
        unpin_all(ts);
}

static thread_state *thread_state_get(void)
{
    (void) pthread_once(&g_once, key_init);
    thread_state *ts = (thread_state *) pthread_getspecific(g_key);
    if (!ts) {
        /* a line-aligned state of its own: the tick and pin counters written on every call must
         * not share a cache line with another thread's (r6 thread A/B) */
        const size_t tsz = (sizeof(*ts) + 127) & ~(size_t) 127;
        ts = (thread_state *) aligned_alloc(128, tsz);
        if (ts)
            memset(ts, 0, tsz);
        if (ts && pthread_setspecific(g_key, ts) != 0) {
            free(ts);
            ts = NULL;
        }
        if (ts) {
            pthread_mutex_lock(&g_ts_mu);
            ts->next = g_ts_head;
            if (g_ts_head)
                g_ts_head->prev = ts;
            g_ts_head = ts;
            pthread_mutex_unlock(&g_ts_mu);
        }
    }
    return ts;
}

static ddt_convertor_t *thread_convertor(void)
{
    thread_state *ts = thread_state_get();
    if (!ts)
        return NULL;
    if (!ts->h)
        ts->h = ddt_convertor_create();
    return ts->h;
}

/* The entry of the convertor's datatype for one call: from this thread's pins when the cache
 * generation has not moved since they were taken (no lock, no shared write; *pinned = 1: do
 * not release), else a normal held lookup (*pinned = 0 unless it was kept as a new pin). */
static bridge_entry *bridge_type_of_call(const opal_convertor_t *conv, int *err, int *pinned)
{
    *pinned = 0;
    const opal_datatype_t *dt = conv->pDesc;
    const dt_type_desc_t *ud = conv->use_desc ? conv->use_desc : (dt ? &dt->opt_desc : NULL);
    thread_state *ts = thread_state_get();
    if (!ts || !dt || !ud || !ud->desc || !(dt->flags & OPAL_DATATYPE_FLAG_COMMITTED))
        return bridge_entry_of(dt, ud, 1, err);
    const uint64_t sig = desc_sig(ud->desc, ud->used);
    const unsigned long gen = __atomic_load_n(&g_gen, __ATOMIC_SEQ_CST);
    for (int i = 0; i < PIN_SLOTS; ++i) {
        pin_slot *p = &ts->pin[i];
        if (!p->e)
            continue;
        if (p->gen != gen) {   /* something was unlinked: this pin may be stale */
            bridge_release(p->e);
            p->e = NULL;
            continue;
        }
        if (p->key == dt && p->ud == ud && p->sig == sig && same_fingerprint(p->e, dt, ud, sig)) {
            p->used = ++ts->tick;
            __atomic_store_n(&ts->pin_hits, ts->pin_hits + 1, __ATOMIC_RELAXED);
            *err = OPAL_SUCCESS;
            *pinned = 1;
            return p->e;
        }
    }
    bridge_entry *e = bridge_entry_of(dt, ud, 1, err);
    if (!e)
        return NULL;
    /* keep the held reference as a pin in the least recently used slot, unless an entry was
     * unlinked meanwhile (then this one may be the unlinked one: release it after the call) */
    if (__atomic_load_n(&g_gen, __ATOMIC_SEQ_CST) != gen)
        return e;
    int v = 0;
    for (int i = 1; i < PIN_SLOTS; ++i)
        if (!ts->pin[i].e || (ts->pin[v].e && ts->pin[i].used < ts->pin[v].used))
            v = i;
    if (ts->pin[v].e)
        bridge_release(ts->pin[v].e);
    ts->pin[v] = (pin_slot){e, dt, ud, sig, gen, ++ts->tick};
    *pinned = 1;
    return e;
}

static void bridge_done(bridge_entry *e, int pinned)
{
    if (!pinned)
        bridge_release(e);
}

static int32_t opal_code(int rc)
{
    switch (rc) {
    case DDT_ERR_OUT_OF_RESOURCE: return OPAL_ERR_OUT_OF_RESOURCE;
    case DDT_ERR_BAD_PARAM: return OPAL_ERR_BAD_PARAM;
    case DDT_ERR_NOT_SUPPORTED: return OPAL_ERR_NOT_SUPPORTED;
    default: return OPAL_ERROR;
    }
}

/* The hipStream_t of an accelerator stream object: the rocm component keeps it in a malloc'ed
 * cell that opal_accelerator_stream_t::stream points to (GET_STREAM,
 * accelerator_rocm_module.c:80; created at :176-182). */
static void *hip_stream_of(const opal_accelerator_stream_t *s)
{
    if (!s || s == OPAL_ACCELERATOR_STREAM_DEFAULT || !s->stream)
        return NULL;
    return *(void *const *) s->stream;
}

static int32_t bridge_move(opal_convertor_t *conv, ddt_datatype_t *t, struct iovec *iov,
                           uint32_t *out_size, size_t *max_data, int pack)
{
    ddt_convertor_t *h = thread_convertor();
    if (!h)
        return OPAL_ERR_OUT_OF_RESOURCE;
    int rc = pack ? ddt_convertor_prepare_for_send(h, t, conv->count, conv->pBaseBuf)
                  : ddt_convertor_prepare_for_recv(h, t, conv->count, conv->pBaseBuf);
    if (rc != DDT_SUCCESS)
        return opal_code(rc);
    size_t pos = conv->bConverted;
    if ((rc = ddt_convertor_set_position(h, &pos)) != DDT_SUCCESS)
        return opal_code(rc);
    /* CONVERTOR_ACCELERATOR_ASYNC: queue on convertor->stream and return; the PML records
     * its completion event on that stream (pml_ob1_recvreq.c:627-663) */
    void *stream = NULL;
    int async = 0;
    if (conv->flags & CONVERTOR_ACCELERATOR_ASYNC) {
        async = 1;
        stream = hip_stream_of(conv->stream);
    }
    ddt_convertor_set_stream(h, stream, async);
    int32_t r = pack ? ddt_convertor_pack(h, iov, out_size, max_data)
                     : ddt_convertor_unpack(h, iov, out_size, max_data);
    ddt_convertor_set_stream(h, NULL, 0);
    return r < 0 ? opal_code(r) : r;
}

static int32_t bridge_advance(opal_convertor_t *conv, struct iovec *iov, uint32_t *out_size,
                              size_t *max_data, int pack)
{
    if (!conv || !out_size || !max_data || (*out_size && !iov))
        return OPAL_ERR_BAD_PARAM;
    if (conv->flags & CONVERTOR_COMPLETED) {   /* opal_convertor_pack/unpack guard (:258-261) */
        if (*out_size)
            iov[0].iov_len = 0;
        *out_size = 0;
        *max_data = 0;
        return 1;
    }
    if (!(conv->flags & CONVERTOR_HOMOGENEOUS))   /* as the accelerator movers assert (:180) */
        return OPAL_ERR_NOT_SUPPORTED;
    int err, pinned;
    bridge_entry *e = bridge_type_of_call(conv, &err, &pinned);
    if (!e)
        return err;
    int32_t r = bridge_move(conv, e->type, iov, out_size, max_data, pack);
    bridge_done(e, pinned);
    if (r < 0)
        return r;
    conv->bConverted += *max_data;
    conv->partial_length = 0;
    if (conv->bConverted == conv->local_size) {
        conv->flags |= CONVERTOR_COMPLETED;
        return 1;
    }
    return 0;
}

int32_t opal_pack_hip(opal_convertor_t *conv, struct iovec *iov, uint32_t *out_size, size_t *max_data)
{
    return bridge_advance(conv, iov, out_size, max_data, 1);
}

int32_t opal_unpack_hip(opal_convertor_t *conv, struct iovec *iov, uint32_t *out_size, size_t *max_data)
{
    return bridge_advance(conv, iov, out_size, max_data, 0);
}

int32_t opal_position_hip(opal_convertor_t *conv, size_t *position)
{
    if (!conv || !position)
        return OPAL_ERR_BAD_PARAM;
    /* opal_convertor_set_position has clamped to the packed size and cleared COMPLETED.
     * opal_convertor_position_generic (opal_convertor.c:445-471) walks the description to the
     * position (opal_datatype_position.c:167-367); a send convertor then drops the partial
     * predefined element (bConverted -= partial_length) and reports the snapped position.
     * The snap follows the imported use_desc, so a UINT4 blen 5 carrier snaps to 4 bytes. */
    size_t p = *position;
    if (conv->flags & CONVERTOR_SEND) {
        int err, pinned;
        bridge_entry *e = bridge_type_of_call(conv, &err, &pinned);
        if (!e)
            return err;
        const int rc = ddt_type_snap_position(e->type, p, &p);
        bridge_done(e, pinned);
        if (rc != DDT_SUCCESS)
            return opal_code(rc);
    }
    conv->bConverted = p;
    conv->partial_length = 0;
    conv->stack_pos = 0;
    *position = p;
    return OPAL_SUCCESS;
}

int opal_hip_bridge_attach(opal_convertor_t *conv)
{
    if (!conv)
        return OPAL_ERR_BAD_PARAM;
    if (!(conv->flags & CONVERTOR_ACCELERATOR) || !(conv->flags & CONVERTOR_HOMOGENEOUS))
        return OPAL_ERR_NOT_SUPPORTED;   /* host buffers keep the reference movers */
    int err, pinned;
    bridge_entry *e = bridge_type_of_call(conv, &err, &pinned);
    if (!e)
        return err;
    bridge_done(e, pinned);
    conv->fAdvance = (conv->flags & CONVERTOR_SEND) ? opal_pack_hip : opal_unpack_hip;
    conv->fPosition = opal_position_hip;
    return OPAL_SUCCESS;
}
