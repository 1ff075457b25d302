// ubench_dense.hip -- is a line-dense pack (BASELINE config 5: 20-byte records at a 32-byte
// stride, 128 Mi records) faster when a workgroup stages its user span through LDS with
// whole-line 16-byte loads and writes the packed stream as 16-byte stores, than with one
// 4-byte unit per lane (the engine's affine path, U = 4)?  Not part of the product.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHK(x)                                                                          \
    do {                                                                                \
        hipError_t e = (x);                                                             \
        if (e != hipSuccess) {                                                          \
            printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);             \
            exit(1);                                                                    \
        }                                                                               \
    } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr uint64_t NREC = 128ull << 20;
constexpr uint32_t REC = 20, STRIDE = 32, WPR = REC / 4;   // dwords per record

// A: one 4-byte unit per lane, K units in flight (the engine's affine loop)
template <int K>
__global__ __launch_bounds__(256) void pack_units(const uint32_t *__restrict__ user, uint32_t *__restrict__ packed,
                                                  uint64_t units, uint32_t per_task)
{
    const uint64_t u0 = uint64_t(blockIdx.x) * per_task, u1 = u0 + per_task < units ? u0 + per_task : units;
    for (uint64_t base = u0 + threadIdx.x; base < u1; base += 256 * K) {
        uint32_t v[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint64_t u = base + uint64_t(k) * 256;
            if (u < u1) {
                const uint64_t r = u / WPR, w = u - r * WPR;
                v[k] = user[r * (STRIDE / 4) + w];
            }
        }
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint64_t u = base + uint64_t(k) * 256;
            if (u < u1)
                packed[u] = v[k];
        }
    }
}

// B: a workgroup stages RPT records (RPT * 32 bytes) through LDS with 16-byte loads, then
// writes RPT * 20 bytes of packed stream as 16-byte stores (RPT a multiple of 4: 80-byte
// aligned packed chunks)
template <uint32_t RPT>
__global__ __launch_bounds__(256) void pack_lds(const u32x4 *__restrict__ user, u32x4 *__restrict__ packed)
{
    __shared__ uint32_t lds[RPT * STRIDE / 4];
    const uint64_t r0 = uint64_t(blockIdx.x) * RPT;
    const u32x4 *src = user + r0 * (STRIDE / 16);
    constexpr uint32_t NV = RPT * STRIDE / 16;
#pragma unroll 4
    for (uint32_t i = threadIdx.x; i < NV; i += 256) {
        const u32x4 v = __builtin_nontemporal_load(src + i);
        lds[4 * i] = v.x;
        lds[4 * i + 1] = v.y;
        lds[4 * i + 2] = v.z;
        lds[4 * i + 3] = v.w;
    }
    __syncthreads();
    constexpr uint32_t NO = RPT * REC / 16;
    u32x4 *dst = packed + r0 * REC / 16;
    for (uint32_t c = threadIdx.x; c < NO; c += 256) {
        uint32_t d[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint32_t q = 4 * c + uint32_t(i);   // dword of the packed chunk
            const uint32_t r = q / WPR, w = q - r * WPR;
            d[i] = lds[r * (STRIDE / 4) + w];
        }
        dst[c] = u32x4{d[0], d[1], d[2], d[3]};
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
    void *u, *p, *q;
    CHK(hipMalloc(&u, ubytes));
    CHK(hipMalloc(&p, pbytes));
    CHK(hipMalloc(&q, pbytes));
    CHK(hipMemset(u, 7, ubytes));
    const uint64_t units = pbytes / 4;
    auto gbs = [&](float us) { return (ubytes + pbytes) / (us * 1e3); };
    for (uint32_t per : {4096u, 8192u, 16384u}) {
        const uint32_t grid = uint32_t((units + per - 1) / per);
        const float t4 = timeit([&] { hipLaunchKernelGGL(pack_units<4>, dim3(grid), dim3(256), 0, 0, (const uint32_t *) u,
                                                         (uint32_t *) p, units, per); }, iters);
        const float t8 = timeit([&] { hipLaunchKernelGGL(pack_units<8>, dim3(grid), dim3(256), 0, 0, (const uint32_t *) u,
                                                         (uint32_t *) p, units, per); }, iters);
        printf("units/lane, %5u units per task: K=4 %.1f us (%.0f GB/s lines r+w) | K=8 %.1f us (%.0f GB/s)\n", per, t4,
               gbs(t4), t8, gbs(t8));
    }
    const float l256 = timeit([&] { hipLaunchKernelGGL(pack_lds<256>, dim3(uint32_t(NREC / 256)), dim3(256), 0, 0,
                                                       (const u32x4 *) u, (u32x4 *) q); }, iters);
    const float l512 = timeit([&] { hipLaunchKernelGGL(pack_lds<512>, dim3(uint32_t(NREC / 512)), dim3(256), 0, 0,
                                                       (const u32x4 *) u, (u32x4 *) q); }, iters);
    const float l1024 = timeit([&] { hipLaunchKernelGGL(pack_lds<1024>, dim3(uint32_t(NREC / 1024)), dim3(256), 0, 0,
                                                        (const u32x4 *) u, (u32x4 *) q); }, iters);
    printf("LDS-staged, records per workgroup 256: %.1f us (%.0f GB/s) | 512: %.1f us (%.0f) | 1024: %.1f us (%.0f)\n",
           l256, gbs(l256), l512, gbs(l512), l1024, gbs(l1024));
    // same bytes?
    bool same = true;
    {
        uint32_t *hp = (uint32_t *) malloc(1 << 20), *hq = (uint32_t *) malloc(1 << 20);
        CHK(hipMemcpy(hp, p, 1 << 20, hipMemcpyDeviceToHost));
        CHK(hipMemcpy(hq, q, 1 << 20, hipMemcpyDeviceToHost));
        for (int i = 0; i < (1 << 18); ++i) same = same && hp[i] == hq[i];
    }
    printf("outputs equal: %s\n", same ? "yes" : "NO");
    return 0;
}
