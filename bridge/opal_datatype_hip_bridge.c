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
#include <stdlib.h>
#include <string.h>

#include "ddt_hip.h"
#include "opal_hip_bridge.h"

/* ------------------------------------------------------------------ import cache */
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
    struct bridge_entry *next;
} bridge_entry;

#define BRIDGE_BUCKETS 256
static bridge_entry *g_buckets[BRIDGE_BUCKETS];
static pthread_mutex_t g_mu = PTHREAD_MUTEX_INITIALIZER;
static size_t g_entries, g_imports, g_hits, g_stale;

static size_t bucket_of(const void *p)
{
    uintptr_t x = (uintptr_t) p;
    x ^= x >> 17;
    x *= 0x9E3779B97F4A7C15ull;
    return (size_t) (x >> 56) % BRIDGE_BUCKETS;
}

/* FNV-1a over the first and last (up to) 8 entries: catches a different description that
 * happens to sit at a recycled address without an O(entries) hash per call. */
static uint64_t desc_sig(const dt_elem_desc_t *d, size_t used)
{
    uint64_t h = 1469598103934665603ull ^ used;
    const size_t head = used < 8 ? used : 8;
    const size_t tail0 = used > head + 8 ? used - 8 : head;
    for (size_t r = 0; r < 2; ++r) {
        const size_t i0 = r ? tail0 : 0, i1 = r ? used : head;
        const unsigned char *b = (const unsigned char *) (d + i0);
        for (size_t k = 0; k < 32 * (i1 - i0); ++k)
            h = (h ^ b[k]) * 1099511628211ull;
    }
    return h;
}

static int same_fingerprint(const bridge_entry *e, const opal_datatype_t *dt, const dt_type_desc_t *ud,
                            uint64_t sig)
{
    return e->desc == ud->desc && e->used == ud->used && e->size == dt->size && e->lb == dt->lb
           && e->ub == dt->ub && e->true_lb == dt->true_lb && e->true_ub == dt->true_ub && e->sig == sig;
}

/* Called with g_mu held on an entry already taken off its bucket list. */
static void retire_locked(bridge_entry *e)
{
    --g_entries;
    if (e->inflight) {   /* a call on another thread still moves data with it */
        e->unlinked = 1;
        return;
    }
    ddt_type_destroy(&e->type);
    free(e);
}

static void bridge_release(bridge_entry *e)
{
    pthread_mutex_lock(&g_mu);
    if (--e->inflight == 0 && e->unlinked) {
        ddt_type_destroy(&e->type);
        free(e);
    }
    pthread_mutex_unlock(&g_mu);
}

/* The entry of (dt, ud) in its bucket, with g_mu held; a different description found at the
 * same address is retired on the way (the old datatype died unseen). */
static bridge_entry *lookup_locked(const opal_datatype_t *dt, const dt_type_desc_t *ud, uint64_t sig)
{
    for (bridge_entry **pp = &g_buckets[bucket_of(dt)]; *pp;) {
        if ((*pp)->key != dt) {
            pp = &(*pp)->next;
            continue;
        }
        if (same_fingerprint(*pp, dt, ud, sig))
            return *pp;
        bridge_entry *old = *pp;
        *pp = old->next;
        retire_locked(old);
        ++g_stale;
    }
    return NULL;
}

/* The cache entry of (dt, ud), imported on first use.  `hold`: keep it for the caller until
 * bridge_release (a destruct or an eviction on another thread in between only unlinks it).
 * The import itself -- seconds for a description of tens of millions of entries -- runs
 * outside the cache lock, so other threads' calls on other datatypes never wait for it; two
 * threads importing the same datatype at once keep the first entry and drop the second. */
static bridge_entry *bridge_entry_of(const opal_datatype_t *dt, const dt_type_desc_t *ud, int hold, int *err)
{
    *err = OPAL_SUCCESS;
    if (!dt || !ud || !ud->desc || !(dt->flags & OPAL_DATATYPE_FLAG_COMMITTED)) {
        *err = OPAL_ERR_BAD_PARAM;
        return NULL;
    }
    const uint64_t sig = desc_sig(ud->desc, ud->used);
    pthread_mutex_lock(&g_mu);
    bridge_entry *e = lookup_locked(dt, ud, sig);
    if (e) {
        ++g_hits;
        if (hold)
            ++e->inflight;
        pthread_mutex_unlock(&g_mu);
        return e;
    }
    pthread_mutex_unlock(&g_mu);

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

    pthread_mutex_lock(&g_mu);
    e = lookup_locked(dt, ud, sig);
    if (e) {   /* another thread imported it meanwhile */
        ++g_hits;
        if (hold)
            ++e->inflight;
        pthread_mutex_unlock(&g_mu);
        ddt_type_destroy(&n->type);
        free(n);
        return e;
    }
    const size_t b = bucket_of(dt);
    n->inflight = hold ? 1 : 0;
    n->next = g_buckets[b];
    g_buckets[b] = n;
    ++g_entries;
    ++g_imports;
    pthread_mutex_unlock(&g_mu);
    return n;
}

static bridge_entry *bridge_type_of(const opal_convertor_t *conv, int *err)
{
    const opal_datatype_t *dt = conv->pDesc;
    return bridge_entry_of(dt, conv->use_desc ? conv->use_desc : (dt ? &dt->opt_desc : NULL), 1, err);
}

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
    pthread_mutex_lock(&g_mu);
    for (bridge_entry **pp = &g_buckets[bucket_of(dt)]; *pp;) {
        if ((*pp)->key == dt) {
            bridge_entry *old = *pp;
            *pp = old->next;
            retire_locked(old);
        } else {
            pp = &(*pp)->next;
        }
    }
    pthread_mutex_unlock(&g_mu);
}

void opal_hip_bridge_finalize(void)
{
    pthread_mutex_lock(&g_mu);
    for (size_t b = 0; b < BRIDGE_BUCKETS; ++b) {
        while (g_buckets[b]) {
            bridge_entry *old = g_buckets[b];
            g_buckets[b] = old->next;
            retire_locked(old);
        }
    }
    pthread_mutex_unlock(&g_mu);
}

void opal_hip_bridge_stats(size_t *out4)
{
    pthread_mutex_lock(&g_mu);
    out4[0] = g_entries;
    out4[1] = g_imports;
    out4[2] = g_hits;
    out4[3] = g_stale;
    pthread_mutex_unlock(&g_mu);
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

/* ------------------------------------------------------------------ per-thread engine convertor */
static pthread_key_t g_key;
static pthread_once_t g_once = PTHREAD_ONCE_INIT;

static void conv_free(void *p) { ddt_convertor_destroy((ddt_convertor_t *) p); }
static void key_init(void) { (void) pthread_key_create(&g_key, conv_free); }

static ddt_convertor_t *thread_convertor(void)
{
    (void) pthread_once(&g_once, key_init);
    ddt_convertor_t *h = (ddt_convertor_t *) pthread_getspecific(g_key);
    if (!h) {
        h = ddt_convertor_create();
        if (h && pthread_setspecific(g_key, h) != 0) {
            ddt_convertor_destroy(h);
            h = NULL;
        }
    }
    return h;
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
    int err;
    bridge_entry *e = bridge_type_of(conv, &err);
    if (!e)
        return err;
    int32_t r = bridge_move(conv, e->type, iov, out_size, max_data, pack);
    bridge_release(e);
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
        int err;
        bridge_entry *e = bridge_type_of(conv, &err);
        if (!e)
            return err;
        const int rc = ddt_type_snap_position(e->type, p, &p);
        bridge_release(e);
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
    int err;
    bridge_entry *e = bridge_type_of(conv, &err);
    if (!e)
        return err;
    bridge_release(e);
    conv->fAdvance = (conv->flags & CONVERTOR_SEND) ? opal_pack_hip : opal_unpack_hip;
    conv->fPosition = opal_position_hip;
    return OPAL_SUCCESS;
}
