/*
 * halo26.c -- a 26-neighbour halo exchange of a 256^3 double field through the engine's
 * convertor ABI, back to back from C: per iteration 26 asynchronous packs (6 faces of 512 KiB,
 * 12 edges of 2 KiB, 8 corners of 8 bytes, each its own committed subarray type) from field A
 * into 26 packed buffers, then 26 asynchronous unpacks into the opposite boundary of field B,
 * all on one stream -- the call pattern of a 3-D stencil code's exchange through ob1
 * (pml_ob1_sendreq.c:535,579 pack each message with its own convertor).  Reports host
 * microseconds per iteration (the calls only enqueue) and device microseconds per iteration
 * (one event pair around the timed iterations), with the launch-slot counters.
 *
 *   ./scripts/halo26 [iters] [slots 0|1] [label]
 * Not part of the library.
 */
#include <hip/hip_runtime_api.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "ddt_hip.h"

#define N 256
#define NB 26

static double now_us(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec * 1e6 + t.tv_nsec * 1e-3;
}

#define CK(x)                                                                            \
    do {                                                                                 \
        int r_ = (int) (x);                                                              \
        if (r_ != 0) {                                                                   \
            fprintf(stderr, "%s failed (%d): %s\n", #x, r_, ddt_last_error());           \
            return 1;                                                                    \
        }                                                                                \
    } while (0)

int main(int argc, char **argv)
{
    const int iters = argc > 1 ? atoi(argv[1]) : 500;
    const int slots = argc > 2 ? atoi(argv[2]) : 1;
    const char *label = argc > 3 ? argv[3] : "engine";
    CK(ddt_tune("slots", slots));
    const size_t field = (size_t) N * N * N * 8;
    void *A, *B;
    CK(hipMalloc(&A, field));
    CK(hipMalloc(&B, field));
    CK(hipMemset(A, 1, field));
    CK(hipMemset(B, 0, field));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    ddt_datatype_t *snd[NB], *rcv[NB];
    ddt_convertor_t *cp[NB], *cu[NB];
    void *pk[NB];
    size_t bytes[NB];
    int nb = 0, kinds[4] = {0, 0, 0, 0};
    for (int dz = -1; dz <= 1; ++dz)
        for (int dy = -1; dy <= 1; ++dy)
            for (int dx = -1; dx <= 1; ++dx) {
                if (!dx && !dy && !dz)
                    continue;
                const int d[3] = {dz, dy, dx};   /* C order: [z][y][x] */
                size_t sizes[3] = {N, N, N}, sub[3], st_s[3], st_r[3];
                int zeros = 0;
                for (int a = 0; a < 3; ++a) {
                    sub[a] = d[a] ? 1 : N;
                    st_s[a] = d[a] < 0 ? 0 : (d[a] > 0 ? N - 1 : 0);   /* our boundary layer */
                    st_r[a] = d[a] < 0 ? N - 1 : (d[a] > 0 ? 0 : 0);   /* the neighbour's opposite side */
                    zeros += d[a] == 0;
                }
                kinds[zeros]++;
                CK(ddt_type_create_subarray(3, sizes, sub, st_s, 0, ddt_predefined(DDT_FLOAT8), &snd[nb]));
                CK(ddt_type_create_subarray(3, sizes, sub, st_r, 0, ddt_predefined(DDT_FLOAT8), &rcv[nb]));
                CK(ddt_type_commit(snd[nb]));
                CK(ddt_type_commit(rcv[nb]));
                CK(ddt_type_size(snd[nb], &bytes[nb]));
                CK(hipMalloc(&pk[nb], bytes[nb]));
                cp[nb] = ddt_convertor_create();
                cu[nb] = ddt_convertor_create();
                CK(ddt_convertor_set_stream(cp[nb], s, 1));
                CK(ddt_convertor_set_stream(cu[nb], s, 1));
                ++nb;
            }
    size_t total = 0;
    for (int i = 0; i < nb; ++i)
        total += bytes[i];
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    int64_t si0[4], si1[4];
    double host = 0;
    for (int phase = 0; phase < 2; ++phase) {   /* 10 warm-up iterations, then the timed ones */
        const int n = phase ? iters : 10;
        if (phase) {
            CK(ddt_slot_info(si0));
            CK(hipEventRecord(e0, s));
        }
        const double t0 = now_us();
        for (int it = 0; it < n; ++it) {
            for (int i = 0; i < nb; ++i) {
                struct iovec iov = {pk[i], bytes[i]};
                uint32_t c = 1;
                size_t md = 0;
                CK(ddt_convertor_prepare_for_send(cp[i], snd[i], 1, A));
                if (ddt_convertor_pack(cp[i], &iov, &c, &md) != 1 || md != bytes[i])
                    return 1;
            }
            for (int i = 0; i < nb; ++i) {
                struct iovec iov = {pk[i], bytes[i]};
                uint32_t c = 1;
                size_t md = 0;
                CK(ddt_convertor_prepare_for_recv(cu[i], rcv[i], 1, B));
                if (ddt_convertor_unpack(cu[i], &iov, &c, &md) != 1 || md != bytes[i])
                    return 1;
            }
        }
        host = (now_us() - t0) / n;
        if (phase)
            CK(hipEventRecord(e1, s));
        CK(hipStreamSynchronize(s));
    }
    CK(ddt_slot_info(si1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    /* spot check: field B's received corners and faces hold field A's bytes (all 0x01) */
    unsigned char probe[8];
    CK(hipMemcpy(probe, (char *) B + field - 8, 8, hipMemcpyDeviceToHost));
    const int ok = probe[0] == 1 && probe[7] == 1;
    printf("{\"what\": \"26-neighbour halo, 256^3 double, %d faces %d edges %d corners, %s\", \"slots\": %d, "
           "\"bytes_per_iter\": %zu, \"calls_per_iter\": %d, \"iters\": %d, \"host_us_per_iter\": %.2f, "
           "\"device_us_per_iter\": %.2f, \"device_us_per_call\": %.3f, \"slot_launches_per_iter\": %.1f, "
           "\"pack_slots_bound\": %lld, \"unpack_slots_bound\": %lld, \"received_ok\": %s}\n",
           kinds[2], kinds[1], kinds[0], label, slots, 2 * total, 2 * nb, iters, host, ms * 1e3 / iters,
           ms * 1e3 / iters / (2 * nb), (double) (si1[3] - si0[3]) / iters, (long long) si1[0], (long long) si1[1],
           ok ? "true" : "false");
    for (int i = 0; i < nb; ++i) {
        ddt_convertor_destroy(cp[i]);
        ddt_convertor_destroy(cu[i]);
        ddt_type_destroy(&snd[i]);
        ddt_type_destroy(&rcv[i]);
    }
    return ok ? 0 : 1;
}
