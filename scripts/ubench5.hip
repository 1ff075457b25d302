// ubench5.hip -- random 4-byte gather/scatter rate vs the size of the region the
// accesses fall in (tuning evidence for the index-list engine, not product).
// 64 Mi elements; element i belongs to region i / R (regions consecutive in blockIdx),
// inside which it maps to a pseudo-random bijective position.  The packed side is
// coalesced.  "xcd" variants give each region to the workgroups of one XCD
// (blockIdx % 8) so that its lines stay in that XCD's 4 MiB L2.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

constexpr uint32_t N = 64u << 20;      // elements
constexpr uint32_t PER_WG = 4096;      // elements per workgroup
constexpr int K = 8;

__device__ __forceinline__ uint32_t mix(uint32_t x, uint32_t bits)
{
    const uint32_t m = bits >= 32 ? 0xffffffffu : ((1u << bits) - 1);
    const uint32_t h = bits / 2 + 1;
    x = (x ^ (x >> h)) & m;
    x = (x * 0x9E3779B1u) & m;
    x = (x ^ (x >> h)) & m;
    x = (x * 0x85EBCA77u) & m;
    x = (x ^ (x >> h)) & m;
    return x;
}

// workgroup -> first element, optionally XCD-grouped: the workgroups of one region all
// have the same blockIdx % 8.
__device__ __forceinline__ uint32_t wg_base(uint32_t b, uint32_t rbits, bool xcd)
{
    if (!xcd) return b * PER_WG;
    const uint32_t wgs_per_region = (1u << rbits) / PER_WG;       // >= 1
    const uint32_t x = b & 7, j = b >> 3;                           // XCD, index within XCD
    const uint32_t region = (j / wgs_per_region) * 8 + x;
    return region * (1u << rbits) + (j % wgs_per_region) * PER_WG;
}

template <bool XCD>
__global__ __launch_bounds__(256) void gat(const uint32_t *__restrict__ in, uint32_t *__restrict__ out, uint32_t rbits)
{
    const uint32_t base = wg_base(blockIdx.x, rbits, XCD);
    for (uint32_t e0 = base + threadIdx.x; e0 < base + PER_WG; e0 += 256 * K) {
        uint32_t v[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint32_t e = e0 + k * 256;
            const uint32_t r = e >> rbits, w = e & ((1u << rbits) - 1);
            v[k] = in[(r << rbits) | mix(w, rbits)];
        }
#pragma unroll
        for (int k = 0; k < K; ++k) out[e0 + k * 256] = v[k];
    }
}

template <bool XCD>
__global__ __launch_bounds__(256) void sca(const uint32_t *__restrict__ in, uint32_t *__restrict__ out, uint32_t rbits)
{
    const uint32_t base = wg_base(blockIdx.x, rbits, XCD);
    for (uint32_t e0 = base + threadIdx.x; e0 < base + PER_WG; e0 += 256 * K) {
        uint32_t v[K];
#pragma unroll
        for (int k = 0; k < K; ++k) v[k] = in[e0 + k * 256];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint32_t e = e0 + k * 256;
            const uint32_t r = e >> rbits, w = e & ((1u << rbits) - 1);
            out[(r << rbits) | mix(w, rbits)] = v[k];
        }
    }
}

template <typename F> float timeit(F f, int it)
{
    hipEvent_t a, b; CHK(hipEventCreate(&a)); CHK(hipEventCreate(&b));
    f(); CHK(hipDeviceSynchronize());
    CHK(hipEventRecord(a)); for (int i = 0; i < it; ++i) f(); CHK(hipEventRecord(b));
    CHK(hipEventSynchronize(b)); float ms; CHK(hipEventElapsedTime(&ms, a, b)); return ms * 1000.f / it;
}

int main(int argc, char **argv)
{
    const int it = argc > 1 ? atoi(argv[1]) : 5;
    uint32_t *a, *b;
    CHK(hipMalloc(&a, size_t(N) * 4)); CHK(hipMalloc(&b, size_t(N) * 4));
    CHK(hipMemset(a, 1, size_t(N) * 4)); CHK(hipMemset(b, 2, size_t(N) * 4));
    const dim3 grid(N / PER_WG), blk(256);
    for (uint32_t rbits : {16u, 18u, 19u, 20u, 21u, 22u, 24u, 26u}) {   // region 256 KiB .. 256 MiB
        float tg = timeit([&] { hipLaunchKernelGGL((gat<false>), grid, blk, 0, 0, a, b, rbits); }, it);
        float ts = timeit([&] { hipLaunchKernelGGL((sca<false>), grid, blk, 0, 0, b, a, rbits); }, it);
        float tgx = 0, tsx = 0;
        if ((1u << rbits) >= PER_WG && rbits <= 23) {
            tgx = timeit([&] { hipLaunchKernelGGL((gat<true>), grid, blk, 0, 0, a, b, rbits); }, it);
            tsx = timeit([&] { hipLaunchKernelGGL((sca<true>), grid, blk, 0, 0, b, a, rbits); }, it);
        }
        printf("region %7u KiB | gather %7.1f us %6.1f G/s | scatter %7.1f us %6.1f G/s | xcd gather %7.1f us scatter %7.1f us\n",
               (1u << rbits) * 4 / 1024, tg, N / tg / 1e3, ts, N / ts / 1e3, tgx, tsx);
    }
    return 0;
}
