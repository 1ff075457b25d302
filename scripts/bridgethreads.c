/*
 * bridgethreads.c -- the drop-in under MPI_THREAD_MULTIPLE: T threads (1, 2, 4, 8), each with its
 * own opal-shaped convertor and its own HIP stream, pack and unpack 512 KiB faces of a 256^3
 * double field (the y face: FLOAT8 count 256 blen 256 extent 524288) through Open MPI's own path
 * (prepare, opal_hip_bridge_attach, conv->fAdvance = opal_pack_hip / opal_unpack_hip), the way
 * ob1 drives accelerator convertors from several threads.  The reference's convertor takes no
 * lock on this path (no opal_mutex in opal/datatype), so aggregate calls per second should
 * grow with the threads until the device or HIP's own launch path is the limit.
 *
 * Per T: every thread's host microseconds per call (the calls only enqueue, ACCELERATOR_ASYNC),
 * device microseconds per operation on its stream (one event pair around its loop), and the
 * aggregate host calls per second = all calls / the slowest thread's loop time.
 *
 *   ./scripts/bridgethreads [iters] [own|shared] [sync|async] [face|tiny]
 *     own     each thread its own opal_datatype_t (own import, plan, descriptor sets; default)
 *     shared  one datatype for all threads (one plan: the threads share its descriptor sets)
 *     sync    no ACCELERATOR_ASYNC: every call returns with the data in place (MPI_Pack's
 *             contract), so host time per call is the whole synchronous operation
 *   [direct|bridge] [slots|noslots]   (bisection of the per-call path)
 *     direct  the engine's own convertor ABI (ddt_convertor_prepare_* + pack / unpack on a
 *             per-thread ddt_convertor_t and a per-type ddt_datatype_t imported once) instead of
 *             the opal bridge's fAdvance
 *     noslots ddt_tune("slots", 0): every launch carries its kernel arguments
 *     tiny    16 doubles at a 2 KiB stride (128 packed bytes) instead of the 512 KiB y face: the
 *             device time per call is the launch alone, so host scaling is not hidden behind the
 *             device's own throughput
 * Not part of the library.
 */
#include <hip/hip_runtime_api.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "ddt_hip.h"
#include "opal_hip_bridge.h"

#define N 256
#define FIELD_BYTES ((size_t) N * N * N * 8)
#define FACE_BYTES ((size_t) N * N * 8)
#define MAXT 8

static double now_us(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec * 1e6 + t.tv_nsec * 1e-3;
}

typedef struct {
    dt_elem_desc_t desc[2];
    opal_datatype_t dt;
} face_type;

static size_t g_bytes = FACE_BYTES;   /* packed bytes per call */

static void make_face(face_type *f, int tiny)
{
    memset(f, 0, sizeof(*f));
    f->desc[0].elem.common.flags = OPAL_DATATYPE_FLAG_DATA | OPAL_DATATYPE_FLAG_CONTIGUOUS;
    f->desc[0].elem.common.type = 16;   /* OPAL_DATATYPE_FLOAT8 */
    f->desc[0].elem.count = tiny ? 16 : N;
    f->desc[0].elem.blocklen = tiny ? 1 : N;
    f->desc[0].elem.extent = tiny ? (ptrdiff_t) N * 8 : (ptrdiff_t) N * N * 8;
    f->desc[1].end_loop.common.type = OPAL_DATATYPE_END_LOOP;
    f->desc[1].end_loop.size = g_bytes;
    opal_datatype_t *dt = &f->dt;
    dt->super.obj_reference_count = 1;
    dt->flags = OPAL_DATATYPE_FLAG_COMMITTED | OPAL_DATATYPE_FLAG_DATA;
    dt->size = g_bytes;
    dt->ub = FIELD_BYTES;
    dt->true_ub = tiny ? (ptrdiff_t) 15 * N * 8 + 8 : (ptrdiff_t) (N - 1) * N * N * 8 + N * 8;
    dt->desc.length = dt->opt_desc.length = 2;
    dt->desc.used = dt->opt_desc.used = 1;
    dt->desc.desc = dt->opt_desc.desc = f->desc;
}

static void prepare(opal_convertor_t *c, opal_datatype_t *dt, void *buf, int send, opal_accelerator_stream_t *s,
                    int async)
{
    memset(c, 0, sizeof(*c));
    c->super.obj_reference_count = 1;
    c->pStack = c->static_stack;
    c->stack_size = DT_STATIC_STACK_SIZE;
    c->flags = (send ? CONVERTOR_SEND : CONVERTOR_RECV) | CONVERTOR_ACCELERATOR
               | (async ? CONVERTOR_ACCELERATOR_ASYNC : 0);
    c->local_size = dt->size;
    c->pBaseBuf = (unsigned char *) buf;
    c->count = 1;
    c->pDesc = dt;
    c->use_desc = &dt->opt_desc;
    c->flags |= (CONVERTOR_DATATYPE_MASK & dt->flags) | CONVERTOR_HOMOGENEOUS;
    c->remote_size = c->local_size;
    c->stream = s;
}

typedef struct {
    int id, iters, async, direct;
    opal_datatype_t *dt;
    ddt_datatype_t *edt;   /* direct: the engine's import of dt */
    ddt_convertor_t *ec;
    void *grid, *packed;
    hipStream_t hs;
    opal_accelerator_stream_t sobj;
    hipEvent_t a, b;
    pthread_barrier_t *bar;
    double host_us;   /* loop time */
    float dev_ms;
    int err;
} worker;

static int run_calls(worker *w, int n)
{
    if (w->direct) {
        for (int i = 0; i < n; ++i) {
            for (int dir = 0; dir < 2; ++dir) {
                struct iovec iov = {w->packed, g_bytes};
                uint32_t cnt = 1;
                size_t md = 0;
                int rc = dir == 0 ? ddt_convertor_prepare_for_send(w->ec, w->edt, 1, w->grid)
                                  : ddt_convertor_prepare_for_recv(w->ec, w->edt, 1, w->grid);
                if (rc != 0)
                    return 4;
                rc = dir == 0 ? ddt_convertor_pack(w->ec, &iov, &cnt, &md) : ddt_convertor_unpack(w->ec, &iov, &cnt, &md);
                if (rc != 1 || md != g_bytes)
                    return 5;
            }
        }
        return 0;
    }
    for (int i = 0; i < n; ++i) {
        for (int dir = 0; dir < 2; ++dir) {   /* pack, then unpack into the same field */
            opal_convertor_t c;
            prepare(&c, w->dt, w->grid, dir == 0, &w->sobj, w->async);
            if (opal_hip_bridge_attach(&c) != OPAL_SUCCESS)
                return 1;
            struct iovec iov = {w->packed, g_bytes};
            uint32_t cnt = 1;
            size_t md = 0;
            if (c.fAdvance(&c, &iov, &cnt, &md) != 1 || md != g_bytes)
                return 2;
        }
    }
    return 0;
}

static void *thread_main(void *p)
{
    worker *w = (worker *) p;
    (void) hipSetDevice(0);
    w->err = run_calls(w, 20);   /* warm-up: imports, descriptor sets, slot binds */
    if (hipStreamSynchronize(w->hs) != hipSuccess)
        w->err = 3;
    pthread_barrier_wait(w->bar);
    (void) hipEventRecord(w->a, w->hs);
    const double t0 = now_us();
    if (!w->err)
        w->err = run_calls(w, w->iters);
    w->host_us = now_us() - t0;
    (void) hipEventRecord(w->b, w->hs);
    (void) hipStreamSynchronize(w->hs);
    (void) hipEventElapsedTime(&w->dev_ms, w->a, w->b);
    return NULL;
}

int main(int argc, char **argv)
{
    const int iters = argc > 1 ? atoi(argv[1]) : 2000;
    const int shared = argc > 2 && !strcmp(argv[2], "shared");
    const int async = !(argc > 3 && !strcmp(argv[3], "sync"));
    const int tiny = argc > 4 && !strcmp(argv[4], "tiny");
    const int direct = argc > 5 && !strcmp(argv[5], "direct");
    if (argc > 6 && !strcmp(argv[6], "noslots"))
        (void) ddt_tune("slots", 0);
    if (tiny)
        g_bytes = 128;
    if (hipSetDevice(0) != hipSuccess)
        return 2;
    static face_type types[MAXT];
    for (int t = 0; t < MAXT; ++t)
        make_face(&types[t], tiny);
    static worker W[MAXT];
    for (int t = 0; t < MAXT; ++t) {
        worker *w = &W[t];
        w->id = t;
        w->async = async;
        if (hipMalloc(&w->grid, FIELD_BYTES) != hipSuccess || hipMalloc(&w->packed, FACE_BYTES) != hipSuccess
            || hipMemset(w->grid, 1 + t, FIELD_BYTES) != hipSuccess
            || hipStreamCreateWithFlags(&w->hs, hipStreamNonBlocking) != hipSuccess
            || hipEventCreate(&w->a) != hipSuccess || hipEventCreate(&w->b) != hipSuccess)
            return 2;
        hipStream_t *cell = (hipStream_t *) malloc(sizeof(hipStream_t));   /* the rocm component's cell */
        *cell = w->hs;
        memset(&w->sobj, 0, sizeof(w->sobj));
        w->sobj.stream = cell;
        w->dt = &types[shared ? 0 : t].dt;
        w->direct = direct;
        if (direct) {
            const opal_datatype_t *d = w->dt;
            if (shared && t > 0) {
                w->edt = W[0].edt;
            } else if (ddt_type_from_opal_desc(d->opt_desc.desc, d->opt_desc.used, d->size, d->lb, d->ub, d->true_lb,
                                               d->true_ub, &w->edt) != 0) {
                return 3;
            }
            w->ec = ddt_convertor_create();
            if (!w->ec || ddt_convertor_set_stream(w->ec, w->hs, async) != 0)
                return 3;
        }
    }
    const int Ts[] = {1, 2, 4, 8};
    double base_rate = 0;
    for (size_t ti = 0; ti < sizeof(Ts) / sizeof(Ts[0]); ++ti) {
        const int T = Ts[ti];
        /* the same total work per thread: a thread's loop is `iters` pack + unpack pairs */
        pthread_barrier_t bar;
        pthread_barrier_init(&bar, NULL, (unsigned) T);
        pthread_t th[MAXT];
        for (int t = 0; t < T; ++t) {
            W[t].iters = iters;
            W[t].bar = &bar;
            W[t].err = 0;
            pthread_create(&th[t], NULL, thread_main, &W[t]);
        }
        for (int t = 0; t < T; ++t)
            pthread_join(th[t], NULL);
        pthread_barrier_destroy(&bar);
        double maxh = 0, sumh = 0, maxd = 0, sumd = 0;
        for (int t = 0; t < T; ++t) {
            if (W[t].err) {
                fprintf(stderr, "thread %d failed: %d\n", t, W[t].err);
                return 1;
            }
            const double h = W[t].host_us / (2.0 * iters), d = W[t].dev_ms * 1e3 / (2.0 * iters);
            maxh = h > maxh ? h : maxh;
            sumh += h;
            maxd = d > maxd ? d : maxd;
            sumd += d;
        }
        double maxloop = 0;
        for (int t = 0; t < T; ++t)
            maxloop = W[t].host_us > maxloop ? W[t].host_us : maxloop;
        const double rate = 2.0 * iters * T / (maxloop * 1e-6);
        if (T == 1)
            base_rate = rate;
        int64_t si[4] = {0, 0, 0, 0};
        (void) ddt_slot_info(si);
        printf("{\"what\": \"%s %s pack+unpack, %s, %s%s\", \"threads\": %d, \"bytes\": %zu, "
               "\"calls_per_thread\": %d, \"host_us_per_call\": {\"mean\": %.3f, \"max\": %.3f}, "
               "\"device_us_per_op\": {\"mean\": %.3f, \"max\": %.3f}, \"aggregate_calls_per_s\": %.0f, "
               "\"speedup_vs_1\": %.3f, \"slots\": [%lld, %lld, %lld, %lld]}\n",
               direct ? "engine ABI" : "bridge", tiny ? "16 doubles at 2 KiB" : "y face",
               shared ? "one shared datatype" : "a datatype per thread", async ? "ACCELERATOR_ASYNC" : "synchronous",
               argc > 6 && !strcmp(argv[6], "noslots") ? ", no launch slots" : "", T, g_bytes, 2 * iters, sumh / T, maxh, sumd / T, maxd, rate, rate / base_rate,
               (long long) si[0], (long long) si[1], (long long) si[2], (long long) si[3]);
        fflush(stdout);
    }
    for (int t = 0; t < MAXT; ++t)
        opal_hip_bridge_datatype_destruct(&types[t].dt);
    return 0;
}
