// ubench_copy.hip -- streaming-copy ceiling of one MI355X (round 2): which launch shape
// reaches the highest read+write rate for a copy far beyond the 256 MiB Infinity Cache.
// Sweeps chunked grids (one contiguous chunk per workgroup) and persistent grid-stride
// grids, unroll depth, workgroup size and load/store cache policy.  Also read-only and
// write-only rates.  Not part of the product; the result sets the copy ceiling quoted in
// DESIGN.md and the per-face targets.
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

template <bool NT> __device__ __forceinline__ u32x4 ld(const u32x4 *p)
{
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}
template <bool NT> __device__ __forceinline__ void st(u32x4 *p, u32x4 v)
{
    if constexpr (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// chunked: workgroup b copies vectors [b*per, (b+1)*per); per % (BS*K) == 0
template <int BS, int K, bool NTL, bool NTS>
__global__ __launch_bounds__(BS) void copy_chunk(const u32x4 *__restrict__ a, u32x4 *__restrict__ b, uint32_t per)
{
    const size_t base = size_t(blockIdx.x) * per;
    for (uint32_t i = threadIdx.x; i < per; i += BS * K) {
        u32x4 v[K];
#pragma unroll
        for (int k = 0; k < K; ++k) v[k] = ld<NTL>(a + base + i + k * BS);
#pragma unroll
        for (int k = 0; k < K; ++k) st<NTS>(b + base + i + k * BS, v[k]);
    }
}

// persistent grid-stride over tiles of BS*K vectors; n % (BS*K) == 0
template <int BS, int K, bool NTL, bool NTS>
__global__ __launch_bounds__(BS) void copy_stride(const u32x4 *__restrict__ a, u32x4 *__restrict__ b, size_t ntiles)
{
    for (size_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const size_t base = t * (BS * K) + threadIdx.x;
        u32x4 v[K];
#pragma unroll
        for (int k = 0; k < K; ++k) v[k] = ld<NTL>(a + base + k * BS);
#pragma unroll
        for (int k = 0; k < K; ++k) st<NTS>(b + base + k * BS, v[k]);
    }
}

template <int BS, int K>
__global__ __launch_bounds__(BS) void read_chunk(const u32x4 *__restrict__ a, u32x4 *__restrict__ sink, uint32_t per)
{
    const size_t base = size_t(blockIdx.x) * per;
    u32x4 acc = {0, 0, 0, 0};
    for (uint32_t i = threadIdx.x; i < per; i += BS * K) {
        u32x4 v[K];
#pragma unroll
        for (int k = 0; k < K; ++k) v[k] = __builtin_nontemporal_load(a + base + i + k * BS);
#pragma unroll
        for (int k = 0; k < K; ++k) acc ^= v[k];
    }
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) sink[threadIdx.x] = acc;
}

template <int BS, int K>
__global__ __launch_bounds__(BS) void write_chunk(u32x4 *__restrict__ b, uint32_t per)
{
    const size_t base = size_t(blockIdx.x) * per;
    const u32x4 v = {blockIdx.x, 1u, 2u, 3u};
    for (uint32_t i = threadIdx.x; i < per; i += BS * K) {
#pragma unroll
        for (int k = 0; k < K; ++k) b[base + i + k * BS] = v;
    }
}

template <typename F>
float timeit(F f, int iters)
{
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    f();
    f();
    CHK(hipDeviceSynchronize());
    CHK(hipEventRecord(a));
    for (int i = 0; i < iters; ++i) f();
    CHK(hipEventRecord(b));
    CHK(hipEventSynchronize(b));
    float ms;
    CHK(hipEventElapsedTime(&ms, a, b));
    CHK(hipEventDestroy(a));
    CHK(hipEventDestroy(b));
    return ms * 1000.f / iters;
}

static u32x4 *A, *B;
static size_t NV;   // vectors copied

template <int BS, int K, bool NTL, bool NTS>
void chunk(uint32_t per_bytes, int it)
{
    const uint32_t per = per_bytes / 16;
    if (per % (BS * K) || NV % per) return;   // shape does not tile this chunk
    const uint32_t g = uint32_t(NV / per);
    float t = timeit([&] { hipLaunchKernelGGL((copy_chunk<BS, K, NTL, NTS>), dim3(g), dim3(BS), 0, 0, A, B, per); }, it);
    printf("chunk  bs %4d K %d ntl %d nts %d per %7u B grid %7u: %8.1f us  %6.0f GB/s r+w\n", BS, K, NTL, NTS,
           per_bytes, g, t, 2.0 * NV * 16 / t / 1e3);
}

template <int BS, int K, bool NTL, bool NTS>
void stride(uint32_t wg_per_cu, int it)
{
    const size_t tiles = NV / (BS * K);
    if (tiles * BS * K != NV) { printf("bad tiles\n"); exit(1); }
    const uint32_t g = 256 * wg_per_cu;
    float t = timeit([&] { hipLaunchKernelGGL((copy_stride<BS, K, NTL, NTS>), dim3(g), dim3(BS), 0, 0, A, B, tiles); }, it);
    printf("stride bs %4d K %d ntl %d nts %d wg/cu %2u grid %7u: %8.1f us  %6.0f GB/s r+w\n", BS, K, NTL, NTS,
           wg_per_cu, g, t, 2.0 * NV * 16 / t / 1e3);
}

int main(int argc, char **argv)
{
    const size_t bytes = (argc > 1 ? size_t(atol(argv[1])) : 2048ull) << 20;
    NV = bytes / 16;
    CHK(hipMalloc(&A, bytes));
    CHK(hipMalloc(&B, bytes));
    CHK(hipMemset(A, 1, bytes));
    CHK(hipMemset(B, 2, bytes));
    const int it = 10;
    printf("copy of %zu MiB (src and dst each, beyond the 256 MiB Infinity Cache)\n", bytes >> 20);
    for (uint32_t per : {16384u, 65536u, 262144u}) {
        chunk<256, 4, false, false>(per, it);
        chunk<256, 8, false, false>(per, it);
        chunk<256, 4, true, false>(per, it);
        chunk<256, 4, false, true>(per, it);
        chunk<256, 4, true, true>(per, it);
        chunk<512, 4, false, false>(per, it);
        chunk<1024, 4, false, false>(per, it);
    }
    for (uint32_t w : {1u, 2u, 4u, 8u}) {
        stride<256, 4, false, false>(w, it);
        stride<256, 4, true, true>(w, it);
        stride<512, 4, false, false>(w, it);
        stride<1024, 2, false, false>(w, it);
        stride<256, 8, false, false>(w, it);
    }
    for (uint32_t per : {65536u, 262144u}) {
        const uint32_t pv = per / 16, g = uint32_t(NV / pv);
        float tr = timeit([&] { hipLaunchKernelGGL((read_chunk<256, 8>), dim3(g), dim3(256), 0, 0, A, B, pv); }, it);
        float tw = timeit([&] { hipLaunchKernelGGL((write_chunk<256, 8>), dim3(g), dim3(256), 0, 0, B, pv); }, it);
        printf("read-only per %u B: %.1f us %.0f GB/s | write-only: %.1f us %.0f GB/s\n", per, tr,
               NV * 16.0 / tr / 1e3, tw, NV * 16.0 / tw / 1e3);
    }
    // 32 MiB (Infinity-Cache resident when looped) for the face-sized moves
    NV = (32ull << 20) / 16;
    printf("copy of 32 MiB (cache-resident when looped)\n");
    chunk<256, 4, false, false>(65536, 50);
    chunk<256, 4, false, false>(16384, 50);
    stride<256, 4, false, false>(2, 50);
    return 0;
}
