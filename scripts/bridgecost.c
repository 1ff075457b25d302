/*
 * bridgecost.c -- the drop-in's host cost per call: Open MPI's own convertor path
 * (opal_convertor_prepare_for_send + opal_convertor_pack -> conv->fAdvance = opal_pack_hip)
 * on opal-shaped objects with CONVERTOR_ACCELERATOR_ASYNC and a rocm-style stream object, the
 * way ob1 drives an accelerator pack, for one 512 KiB face of a 256^3 double field (the y face:
 * FLOAT8 count 256 blen 256 extent 524288).  Per call: host microseconds (the calls only
 * enqueue) and device microseconds (one event pair around the loop).  Not part of the library.
 *
 *   ./scripts/bridgecost [iters]
 */
#include <hip/hip_runtime_api.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "opal_hip_bridge.h"

#define N 256
#define FIELD_BYTES ((size_t) N * N * N * 8)
#define FACE_BYTES ((size_t) N * N * 8)

#define CHECK(x)                                                                        \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                     \
            return 2;                                                                   \
        }                                                                               \
    } while (0)

static double now_us(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec * 1e6 + t.tv_nsec * 1e-3;
}

static void prepare(opal_convertor_t *c, opal_datatype_t *dt, void *buf, int send, opal_accelerator_stream_t *s)
{
    memset(c, 0, sizeof(*c));
    c->super.obj_reference_count = 1;
    c->pStack = c->static_stack;
    c->stack_size = DT_STATIC_STACK_SIZE;
    c->flags = (send ? CONVERTOR_SEND : CONVERTOR_RECV) | CONVERTOR_ACCELERATOR | CONVERTOR_ACCELERATOR_ASYNC;
    c->local_size = dt->size;
    c->pBaseBuf = (unsigned char *) buf;
    c->count = 1;
    c->pDesc = dt;
    c->use_desc = &dt->opt_desc;
    c->flags |= (CONVERTOR_DATATYPE_MASK & dt->flags) | CONVERTOR_HOMOGENEOUS;
    c->remote_size = c->local_size;
    c->stream = s;
}

int main(int argc, char **argv)
{
    const int iters = argc > 1 ? atoi(argv[1]) : 2000;
    dt_elem_desc_t desc[2];
    memset(desc, 0, sizeof(desc));
    desc[0].elem.common.flags = OPAL_DATATYPE_FLAG_DATA | OPAL_DATATYPE_FLAG_CONTIGUOUS;
    desc[0].elem.common.type = 16;   /* OPAL_DATATYPE_FLOAT8 */
    desc[0].elem.count = N;
    desc[0].elem.blocklen = N;
    desc[0].elem.extent = (ptrdiff_t) N * N * 8;
    desc[0].elem.disp = 0;
    desc[1].end_loop.common.type = OPAL_DATATYPE_END_LOOP;
    desc[1].end_loop.size = FACE_BYTES;
    opal_datatype_t dt;
    memset(&dt, 0, sizeof(dt));
    dt.super.obj_reference_count = 1;
    dt.flags = OPAL_DATATYPE_FLAG_COMMITTED | OPAL_DATATYPE_FLAG_DATA;
    dt.size = FACE_BYTES;
    dt.lb = 0;
    dt.ub = FIELD_BYTES;
    dt.true_lb = 0;
    dt.true_ub = (ptrdiff_t) (N - 1) * N * N * 8 + N * 8;
    dt.desc.length = dt.opt_desc.length = 2;
    dt.desc.used = dt.opt_desc.used = 1;
    dt.desc.desc = dt.opt_desc.desc = desc;

    void *d_grid, *d_packed;
    CHECK(hipMalloc(&d_grid, FIELD_BYTES));
    CHECK(hipMalloc(&d_packed, FACE_BYTES));
    CHECK(hipMemset(d_grid, 1, FIELD_BYTES));
    hipStream_t hs;
    CHECK(hipStreamCreateWithFlags(&hs, hipStreamNonBlocking));
    hipStream_t *cell = (hipStream_t *) malloc(sizeof(hipStream_t));   /* the rocm component's cell */
    *cell = hs;
    opal_accelerator_stream_t sobj;
    memset(&sobj, 0, sizeof(sobj));
    sobj.stream = cell;
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));

    for (int dir = 0; dir < 2; ++dir) {
        opal_convertor_t c;
        double host = 0;
        for (int phase = 0; phase < 2; ++phase) {   /* 20 warm-up calls, then the timed loop */
            const int n = phase ? iters : 20;
            if (phase)
                CHECK(hipEventRecord(a, hs));
            const double t0 = now_us();
            for (int i = 0; i < n; ++i) {
                prepare(&c, &dt, d_grid, dir == 0, &sobj);
                if (opal_hip_bridge_attach(&c) != OPAL_SUCCESS)
                    return 1;
                struct iovec iov = {d_packed, FACE_BYTES};
                uint32_t cnt = 1;
                size_t md = 0;
                const int32_t rc = c.fAdvance(&c, &iov, &cnt, &md);
                if (rc != 1 || md != FACE_BYTES) {
                    fprintf(stderr, "fAdvance rc %d moved %zu\n", rc, md);
                    return 1;
                }
            }
            host = (now_us() - t0) / n;
            if (phase)
                CHECK(hipEventRecord(b, hs));
            CHECK(hipStreamSynchronize(hs));
        }
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, a, b));
        printf("{\"what\": \"bridge %s y face (prepare + attach + fAdvance)\", \"bytes\": %zu, \"host_us\": %.3f, "
               "\"device_us\": %.3f}\n", dir ? "unpack" : "pack", FACE_BYTES, host, ms * 1e3 / iters);
    }
    opal_hip_bridge_datatype_destruct(&dt);
    return 0;
}
