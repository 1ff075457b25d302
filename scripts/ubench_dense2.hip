// ubench_dense2.hip -- round 3: kernel shapes for line-dense records (BASELINE config 5:
// 20-byte records at a 32-byte stride, 128 Mi records, 4 GiB user span, 2.5 GiB packed),
// pack AND unpack, to choose what the move kernel builds in.  Not part of the product.
//   pack  A: one 4-byte unit per lane (the engine's affine loop today)
//         B: workgroup stages R records through LDS with 16-byte loads, writes 16-byte stores
//         C: each lane owns 4 records: 4 x (16 + 4)-byte loads, 5 x 16-byte stores
//   unpack A: one 4-byte unit per lane
//          B: workgroup stages R records of packed stream through LDS (16-byte loads), each
//             lane writes whole records as one 16-byte + one 4-byte store
//          C: each lane owns 4 records: 5 x 16-byte loads, 4 x (16 + 4)-byte stores
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHK(x)                                                                          \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);            \
            exit(1);                                                                    \
        }                                                                               \
    } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr uint64_t NREC = 128ull << 20;
constexpr uint32_t REC = 20, STRIDE = 32, WPR = REC / 4;

template <int DIR, int K>
__global__ __launch_bounds__(256) void units(uint32_t *__restrict__ user, uint32_t *__restrict__ packed,
                                             uint32_t per_task)
{
    const uint64_t u0 = uint64_t(blockIdx.x) * per_task, u1 = u0 + per_task;
    for (uint64_t base = u0 + threadIdx.x; base < u1; base += 256 * K) {
        uint32_t v[K];
        uint64_t ua[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint64_t u = base + uint64_t(k) * 256;
            const uint64_t r = u / WPR, w = u - r * WPR;
            ua[k] = r * (STRIDE / 4) + w;
            v[k] = DIR == 0 ? __builtin_nontemporal_load(user + ua[k]) : packed[u];
        }
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint64_t u = base + uint64_t(k) * 256;
            if (DIR == 0) packed[u] = v[k];
            else user[ua[k]] = v[k];
        }
    }
}

template <uint32_t R>
__global__ __launch_bounds__(256) void pack_lds(const u32x4 *__restrict__ user, u32x4 *__restrict__ packed)
{
    __shared__ uint32_t lds[R * STRIDE / 4];
    const uint64_t r0 = uint64_t(blockIdx.x) * R;
    const u32x4 *src = user + r0 * (STRIDE / 16);
    constexpr uint32_t NV = R * STRIDE / 16, PV = NV / 256 > 0 ? NV / 256 : 1;
    u32x4 v[PV];
#pragma unroll
    for (uint32_t k = 0; k < PV; ++k) v[k] = __builtin_nontemporal_load(src + threadIdx.x + k * 256);
#pragma unroll
    for (uint32_t k = 0; k < PV; ++k) *reinterpret_cast<u32x4 *>(&lds[4 * (threadIdx.x + k * 256)]) = v[k];
    __syncthreads();
    constexpr uint32_t NO = R * REC / 16;
    u32x4 *dst = packed + r0 * REC / 16;
    for (uint32_t c = threadIdx.x; c < NO; c += 256) {
        uint32_t d[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint32_t q = 4 * c + uint32_t(i), r = q / WPR, w = q - r * WPR;
            d[i] = lds[r * (STRIDE / 4) + w];
        }
        dst[c] = u32x4{d[0], d[1], d[2], d[3]};
    }
}

template <uint32_t R>
__global__ __launch_bounds__(256) void unpack_lds(u32x4 *__restrict__ user, const u32x4 *__restrict__ packed)
{
    __shared__ uint32_t lds[R * REC / 4];
    const uint64_t r0 = uint64_t(blockIdx.x) * R;
    const u32x4 *src = packed + r0 * REC / 16;
    constexpr uint32_t NV = R * REC / 16;
    for (uint32_t i = threadIdx.x; i < NV; i += 256)
        *reinterpret_cast<u32x4 *>(&lds[4 * i]) = __builtin_nontemporal_load(src + i);
    __syncthreads();
    for (uint32_t r = threadIdx.x; r < R; r += 256) {
        const uint32_t *l = &lds[r * WPR];
        uint32_t *d = reinterpret_cast<uint32_t *>(user + (r0 + r) * (STRIDE / 16));
        *reinterpret_cast<u32x4 *>(d) = u32x4{l[0], l[1], l[2], l[3]};
        d[4] = l[4];
    }
}

// C: lane owns 4 records (80 packed bytes = 5 vectors)
template <int DIR>
__global__ __launch_bounds__(256) void quad(u32x4 *__restrict__ user, u32x4 *__restrict__ packed)
{
    const uint64_t q = uint64_t(blockIdx.x) * 256 + threadIdx.x;   // record quad
    u32x4 *pk = packed + q * 5;
    uint32_t w[20];
    if (DIR == 0) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const uint32_t *s = reinterpret_cast<const uint32_t *>(user + (q * 4 + r) * 2);
            const u32x4 a = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(s));
            w[5 * r] = a.x; w[5 * r + 1] = a.y; w[5 * r + 2] = a.z; w[5 * r + 3] = a.w;
            w[5 * r + 4] = __builtin_nontemporal_load(s + 4);
        }
#pragma unroll
        for (int i = 0; i < 5; ++i) pk[i] = u32x4{w[4 * i], w[4 * i + 1], w[4 * i + 2], w[4 * i + 3]};
    } else {
#pragma unroll
        for (int i = 0; i < 5; ++i) {
            const u32x4 a = __builtin_nontemporal_load(pk + i);
            w[4 * i] = a.x; w[4 * i + 1] = a.y; w[4 * i + 2] = a.z; w[4 * i + 3] = a.w;
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            uint32_t *d = reinterpret_cast<uint32_t *>(user + (q * 4 + r) * 2);
            *reinterpret_cast<u32x4 *>(d) = u32x4{w[5 * r], w[5 * r + 1], w[5 * r + 2], w[5 * r + 3]};
            d[4] = w[5 * r + 4];
        }
    }
}

template <typename F>
float timeit(F f, int iters)
{
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    f();
    CHK(hipDeviceSynchronize());
    CHK(hipEventRecord(a));
    for (int i = 0; i < iters; ++i) f();
    CHK(hipEventRecord(b));
    CHK(hipEventSynchronize(b));
    float ms;
    CHK(hipEventElapsedTime(&ms, a, b));
    return ms * 1000.f / iters;
}

int main(int argc, char **argv)
{
    const int iters = argc > 1 ? atoi(argv[1]) : 10;
    const uint64_t ubytes = NREC * STRIDE, pbytes = NREC * REC;
    void *u, *p;
    CHK(hipMalloc(&u, ubytes));
    CHK(hipMalloc(&p, pbytes));
    CHK(hipMemset(u, 7, ubytes));
    CHK(hipMemset(p, 9, pbytes));
    const uint32_t units_total = uint32_t(pbytes / 4);
    auto gbs = [&](float us) { return (ubytes + pbytes) / (us * 1e3); };
    for (int dir = 0; dir < 2; ++dir) {
        const char *nm = dir ? "unpack" : "pack  ";
        for (uint32_t per : {4096u, 8192u}) {
            const uint32_t grid = units_total / per;
            float t = dir ? timeit([&] { hipLaunchKernelGGL((units<1, 8>), dim3(grid), dim3(256), 0, 0, (uint32_t *) u, (uint32_t *) p, per); }, iters)
                          : timeit([&] { hipLaunchKernelGGL((units<0, 8>), dim3(grid), dim3(256), 0, 0, (uint32_t *) u, (uint32_t *) p, per); }, iters);
            printf("%s A units K=8, %5u units/task: %7.1f us (%4.0f GB/s lines r+w)\n", nm, per, t, gbs(t));
        }
#define LDSV(RR)                                                                                                  \
        {                                                                                                         \
            float t = dir ? timeit([&] { hipLaunchKernelGGL(unpack_lds<RR>, dim3(uint32_t(NREC / RR)), dim3(256), 0, 0, \
                                                            (u32x4 *) u, (const u32x4 *) p); }, iters)             \
                          : timeit([&] { hipLaunchKernelGGL(pack_lds<RR>, dim3(uint32_t(NREC / RR)), dim3(256), 0, 0,   \
                                                            (const u32x4 *) u, (u32x4 *) p); }, iters);            \
            printf("%s B LDS, %4d records/workgroup: %7.1f us (%4.0f GB/s)\n", nm, RR, t, gbs(t));             \
        }
        LDSV(128) LDSV(256) LDSV(512)
        float tq = dir ? timeit([&] { hipLaunchKernelGGL(quad<1>, dim3(uint32_t(NREC / 1024)), dim3(256), 0, 0, (u32x4 *) u, (u32x4 *) p); }, iters)
                       : timeit([&] { hipLaunchKernelGGL(quad<0>, dim3(uint32_t(NREC / 1024)), dim3(256), 0, 0, (u32x4 *) u, (u32x4 *) p); }, iters);
        printf("%s C 4 records per lane: %7.1f us (%4.0f GB/s)\n", nm, tq, gbs(tq));
    }
    return 0;
}
