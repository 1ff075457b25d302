/*
 * bridge_demo.c -- the fAdvance bridge driven from C, the way Open MPI's own code drives a
 * convertor: an opal_datatype_t with a committed opt_desc, an opal_convertor_t prepared as
 * OPAL_CONVERTOR_PREPARE + opal_convertor_prepare_for_{send,recv} leave it
 * (opal_convertor.c:526-696), the movers swapped by opal_hip_bridge_attach() (the
 * pack_description_sweep.c:877-965 precedent), then opal_convertor_pack/unpack's call into
 * conv->fAdvance (:255-349) in BTL-sized fragments, with opal_convertor_set_position
 * (opal_convertor.h:357-394) for out-of-order receives.
 *
 * Workload: the x face of a 64^3 double grid, 5 fields (the SURVEY App. A description
 * FLOAT8 count 4096 blen 1 extent 512, resized to the field).  Checks against the closed
 * form on the host: packed[f][r] = grid[f][r*64 + 0].  Exit status 0 = bit-exact.
 * Test infrastructure (tests/test_gpu_bridge.py builds and runs it); not part of the library.
 */
#include <hip/hip_runtime_api.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "opal_hip_bridge.h"

#define N 64
#define FIELDS 5
#define FIELD_BYTES ((size_t) N * N * N * 8)
#define FACE (N * N)

#define CHECK(x)                                                                        \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                     \
            return 2;                                                                   \
        }                                                                               \
    } while (0)

static void prepare(opal_convertor_t *c, opal_datatype_t *dt, size_t count, void *buf, int send)
{
    /* opal_convertor_construct + prepare_for_{send,recv}: check_addr said "device" */
    memset(c, 0, sizeof(*c));
    c->super.obj_reference_count = 1;
    c->pStack = c->static_stack;
    c->stack_size = DT_STATIC_STACK_SIZE;
    c->flags = (send ? CONVERTOR_SEND : CONVERTOR_RECV) | CONVERTOR_ACCELERATOR;
    c->local_size = count * dt->size;
    c->pBaseBuf = (unsigned char *) buf;
    c->count = count;
    c->pDesc = dt;
    c->bConverted = 0;
    c->use_desc = &dt->opt_desc;
    c->flags |= (CONVERTOR_DATATYPE_MASK & dt->flags) | CONVERTOR_HOMOGENEOUS;
    c->remote_size = c->local_size;
}

/* opal_convertor_pack / _unpack for a non-NO_OP convertor: the COMPLETED guard, then fAdvance */
static int32_t conv_advance(opal_convertor_t *c, void *p, size_t n, size_t *moved)
{
    struct iovec iov = {p, n};
    uint32_t cnt = 1;
    *moved = 0;
    if (c->flags & CONVERTOR_COMPLETED)
        return 1;
    return c->fAdvance(c, &iov, &cnt, moved);
}

static void set_position(opal_convertor_t *c, size_t pos)
{
    if (c->local_size <= pos) {
        c->flags |= CONVERTOR_COMPLETED;
        c->bConverted = c->local_size;
        return;
    }
    if (pos == c->bConverted)
        return;
    c->flags &= ~CONVERTOR_COMPLETED;
    c->fPosition(c, &pos);
}

int main(void)
{
    /* the committed description: one DATA entry + the END_LOOP sentinel */
    dt_elem_desc_t desc[2];
    memset(desc, 0, sizeof(desc));
    desc[0].elem.common.flags = OPAL_DATATYPE_FLAG_DATA | OPAL_DATATYPE_FLAG_CONTIGUOUS;
    desc[0].elem.common.type = 16;   /* OPAL_DATATYPE_FLOAT8 */
    desc[0].elem.count = FACE;
    desc[0].elem.blocklen = 1;
    desc[0].elem.extent = N * 8;
    desc[0].elem.disp = 0;
    desc[1].end_loop.common.type = OPAL_DATATYPE_END_LOOP;
    desc[1].end_loop.size = FACE * 8;
    opal_datatype_t dt;
    memset(&dt, 0, sizeof(dt));
    dt.super.obj_reference_count = 1;
    dt.flags = OPAL_DATATYPE_FLAG_COMMITTED | OPAL_DATATYPE_FLAG_DATA;
    dt.size = FACE * 8;
    dt.lb = 0;
    dt.ub = FIELD_BYTES;                    /* resized to the field */
    dt.true_lb = 0;
    dt.true_ub = (ptrdiff_t) (FACE - 1) * N * 8 + 8;
    dt.desc.length = dt.opt_desc.length = 2;
    dt.desc.used = dt.opt_desc.used = 1;
    dt.desc.desc = dt.opt_desc.desc = desc;

    const size_t span = FIELDS * FIELD_BYTES, packed_bytes = FIELDS * FACE * 8;
    double *h = (double *) malloc(span), *back = (double *) malloc(span);
    double *hp = (double *) malloc(packed_bytes);
    for (size_t i = 0; i < span / 8; ++i)
        h[i] = (double) (i * 2654435761u % 1000003u) + 0.25;
    void *d_grid, *d_packed, *d_out;
    CHECK(hipMalloc(&d_grid, span));
    CHECK(hipMalloc(&d_packed, packed_bytes));
    CHECK(hipMalloc(&d_out, span));
    CHECK(hipMemcpy(d_grid, h, span, hipMemcpyHostToDevice));
    CHECK(hipMemset(d_out, 0, span));

    /* pack in 7000-byte fragments (not a multiple of 8: the pack stops on elements) */
    opal_convertor_t c;
    prepare(&c, &dt, FIELDS, d_grid, 1);
    if (opal_hip_bridge_attach(&c) != OPAL_SUCCESS || c.fAdvance != opal_pack_hip) {
        fprintf(stderr, "attach failed\n");
        return 1;
    }
    size_t pos = 0, moved;
    int32_t rc = 0;
    while (rc == 0) {
        size_t cap = packed_bytes - pos < 7000 ? packed_bytes - pos : 7000;
        rc = conv_advance(&c, (char *) d_packed + pos, cap, &moved);
        if (rc < 0 || moved % 8 || (moved == 0 && cap >= 8)) {
            fprintf(stderr, "pack rc %d moved %zu at %zu\n", rc, moved, pos);
            return 1;
        }
        pos += moved;
    }
    if (pos != packed_bytes || !(c.flags & CONVERTOR_COMPLETED)) {
        fprintf(stderr, "pack ended at %zu\n", pos);
        return 1;
    }
    CHECK(hipMemcpy(hp, d_packed, packed_bytes, hipMemcpyDeviceToHost));
    for (size_t f = 0; f < FIELDS; ++f)
        for (size_t r = 0; r < FACE; ++r)
            if (memcmp(&hp[f * FACE + r], &h[f * (FIELD_BYTES / 8) + r * N], 8) != 0) {
                fprintf(stderr, "packed mismatch field %zu row %zu\n", f, r);
                return 1;
            }

    /* unpack out of order: fragments of 4099 bytes (mid-element cuts), last to first */
    opal_convertor_t u;
    prepare(&u, &dt, FIELDS, d_out, 0);
    if (opal_hip_bridge_attach(&u) != OPAL_SUCCESS || u.fAdvance != opal_unpack_hip)
        return 1;
    const size_t frag = 4099;
    for (size_t k = (packed_bytes + frag - 1) / frag; k-- > 0;) {
        const size_t a = k * frag, n = packed_bytes - a < frag ? packed_bytes - a : frag;
        set_position(&u, a);
        rc = conv_advance(&u, (char *) d_packed + a, n, &moved);
        if (rc < 0 || moved != n) {
            fprintf(stderr, "unpack rc %d moved %zu of %zu at %zu\n", rc, moved, n, a);
            return 1;
        }
    }
    CHECK(hipMemcpy(back, d_out, span, hipMemcpyDeviceToHost));
    for (size_t i = 0; i < span / 8; ++i) {
        const int on_face = ((i % (FIELD_BYTES / 8)) % N) == 0;
        const double want = on_face ? h[i] : 0.0;
        if (memcmp(&back[i], &want, 8) != 0) {
            fprintf(stderr, "unpack mismatch at double %zu\n", i);
            return 1;
        }
    }
    opal_hip_bridge_datatype_destruct(&dt);
    size_t st[4];
    opal_hip_bridge_stats(st);
    printf("bridge_demo ok: %zu bytes packed in fragments and unpacked out of order; imports %zu hits %zu\n",
           packed_bytes, st[1], st[2]);
    CHECK(hipFree(d_grid));
    CHECK(hipFree(d_packed));
    CHECK(hipFree(d_out));
    free(h);
    free(back);
    free(hp);
    return 0;
}
