// ubench_face.hip -- ceilings for the per-face figure with a cold, clean cache (round 3).
// Each repetition first reads a 1 GiB scribble buffer (4x the 256 MiB Infinity Cache), then
// times ONE kernel with events: the same protocol as bench.face_throughput(flush="read").
// Shapes (256 MiB moved each way, the 256^3 double faces of 512 fields):
//   z: a contiguous copy, 16 KiB chunks per workgroup (the engine's streaming task size);
//   y: 2 KiB rows at a 512 KiB stride gathered to / scattered from a contiguous stream.
// Variants: load/store cache policy, chunk size, rows per workgroup.  Not part of the product.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

#define CHK(x)                                                                          \
    do {                                                                                \
        hipError_t e = (x);                                                             \
        if (e != hipSuccess) {                                                          \
            printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);             \
            exit(1);                                                                    \
        }                                                                               \
    } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int NT> __device__ __forceinline__ u32x4 ld(const u32x4 *p)
{
    if constexpr (NT == 1) return __builtin_nontemporal_load(p);
    else return *p;
}
template <int NT> __device__ __forceinline__ void st(u32x4 *p, u32x4 v)
{
    if constexpr (NT == 1) __builtin_nontemporal_store(v, p);
    else *p = v;
}

__global__ __launch_bounds__(256) void flush_write(u32x4 *__restrict__ a, size_t nv, uint32_t v)
{
    for (size_t i = size_t(blockIdx.x) * 256 + threadIdx.x; i < nv; i += size_t(gridDim.x) * 256)
        a[i] = u32x4{v, v, v, v};
}

static bool g_write_flush = false;

__global__ __launch_bounds__(256) void flush_read(const u32x4 *__restrict__ a, u32x4 *__restrict__ sink, size_t nv)
{
    u32x4 acc = {0, 0, 0, 0};
    for (size_t i = size_t(blockIdx.x) * 256 + threadIdx.x; i < nv; i += size_t(gridDim.x) * 256)
        acc ^= a[i];
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) sink[threadIdx.x] = acc;
}

// z: workgroup b copies vectors [b*per, (b+1)*per)
template <int K, int NTL, int NTS>
__global__ __launch_bounds__(256) void copy_chunk(const u32x4 *__restrict__ a, u32x4 *__restrict__ b, uint32_t per)
{
    const size_t base = size_t(blockIdx.x) * per;
    for (uint32_t i = threadIdx.x; i < per; i += 256 * K) {
        u32x4 v[K];
#pragma unroll
        for (int k = 0; k < K; ++k) v[k] = ld<NTL>(a + base + i + k * 256);
#pragma unroll
        for (int k = 0; k < K; ++k) st<NTS>(b + base + i + k * 256, v[k]);
    }
}

// y: R rows of 2 KiB (128 vectors) per workgroup; row r at user + r * stride_v; packed r*128.
// DIR 0 gathers (pack), DIR 1 scatters (unpack).  XCD: blocks are renumbered so that each XCD
// (blockIdx % 8) takes a contiguous range of rows when SLAB is set.
template <int R, int DIR, int NTL, int NTS, bool SLAB>
__global__ __launch_bounds__(256) void rows(u32x4 *__restrict__ user, u32x4 *__restrict__ packed, uint32_t nrows,
                                            uint32_t stride_v)
{
    uint32_t b = blockIdx.x;
    if (SLAB) {
        const uint32_t g = gridDim.x, per = g / 8;
        b = (b % 8) * per + b / 8;
    }
    constexpr int PER = R * 128 / 256;   // vectors per thread
    u32x4 v[PER];
    const uint32_t r0 = b * R;
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        const uint32_t e = threadIdx.x + k * 256, r = r0 + e / 128, c = e % 128;
        if (DIR == 0) v[k] = ld<NTL>(user + size_t(r) * stride_v + c);
        else v[k] = ld<NTL>(packed + size_t(r) * 128 + c);
    }
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        const uint32_t e = threadIdx.x + k * 256, r = r0 + e / 128, c = e % 128;
        if (DIR == 0) st<NTS>(packed + size_t(r) * 128 + c, v[k]);
        else st<NTS>(user + size_t(r) * stride_v + c, v[k]);
    }
}

static u32x4 *F, *SINK;
static const size_t FV = (1ull << 30) / 16;

template <typename L>
float cold(L launch, int reps)
{
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    std::vector<float> ts;
    for (int i = 0; i < reps + 2; ++i) {
        if (g_write_flush)
            hipLaunchKernelGGL(flush_write, dim3(4096), dim3(256), 0, 0, F, FV, uint32_t(i));
        else
            hipLaunchKernelGGL(flush_read, dim3(4096), dim3(256), 0, 0, F, SINK, FV);
        CHK(hipEventRecord(a));
        launch();
        CHK(hipEventRecord(b));
        CHK(hipEventSynchronize(b));
        float ms;
        CHK(hipEventElapsedTime(&ms, a, b));
        if (i >= 2) ts.push_back(ms * 1000.f);
    }
    std::sort(ts.begin(), ts.end());
    CHK(hipEventDestroy(a));
    CHK(hipEventDestroy(b));
    return ts[ts.size() / 2];
}

int main(int argc, char **argv)
{
    g_write_flush = argc > 1 && argv[1][0] == 'w';   // "write": the flush writes its 1 GiB instead
    const size_t bytes = 256ull << 20, NV = bytes / 16;
    u32x4 *A, *B, *G;
    CHK(hipMalloc(&F, FV * 16));
    CHK(hipMalloc(&SINK, 4096));
    CHK(hipMalloc(&A, bytes));
    CHK(hipMalloc(&B, bytes));
    CHK(hipMemset(F, 1, FV * 16));
    CHK(hipMemset(A, 1, bytes));
    CHK(hipMemset(B, 2, bytes));
    const int reps = 15;
    auto rate = [&](float us) { return 2.0 * bytes / us / 1e6; };   // TB/s read + write
    printf("cold 256 MiB moves after a 1 GiB %s flush (median of %d), TB/s r+w and frac of 8 TB/s\n",
           g_write_flush ? "WRITE" : "read", reps);
#define Z(K, NTL, NTS, PERB)                                                                                \
    {                                                                                                       \
        const uint32_t per = PERB / 16;                                                                     \
        if (per % (256 * K) == 0) {                                                                         \
        float t = cold([&] { hipLaunchKernelGGL((copy_chunk<K, NTL, NTS>), dim3(NV / per), dim3(256), 0, 0, \
                                                A, B, per); }, reps);                                       \
        printf("z copy   K %d ntl %d nts %d chunk %6d B: %7.1f us %5.2f TB/s %.3f\n", K, NTL, NTS, PERB, t, \
               rate(t), rate(t) / 8.0);                                                                     \
        }                                                                                                   \
    }
    Z(4, 0, 0, 16384) Z(4, 1, 0, 16384) Z(4, 1, 1, 16384) Z(4, 0, 1, 16384) Z(8, 1, 0, 16384)
    Z(2, 1, 0, 8192) Z(4, 1, 0, 32768) Z(4, 1, 0, 65536)
    // y: user grid of 512 fields x 256 planes of 512 KiB, one 2 KiB row per plane (the y face)
    const size_t gbytes = 64ull << 30;
    u32x4 *U;
    CHK(hipMalloc(&U, gbytes));
    CHK(hipMemset(U, 3, gbytes));
    G = U;
    const uint32_t nrows = 512 * 256, sv = (512u << 10) / 16;
#define Y(R, DIR, NTL, NTS, SLAB)                                                                              \
    {                                                                                                          \
        float t = cold([&] { hipLaunchKernelGGL((rows<R, DIR, NTL, NTS, SLAB>), dim3(nrows / R), dim3(256), 0, \
                                                0, G, B, nrows, sv); }, reps);                                 \
        printf("y %s R %2d ntl %d nts %d slab %d: %7.1f us %5.2f TB/s %.3f\n", DIR ? "scatter" : "gather ", R, \
               NTL, NTS, SLAB, t, rate(t), rate(t) / 8.0);                                                      \
    }
    Y(8, 0, 0, 0, false) Y(8, 0, 1, 0, false) Y(8, 0, 1, 0, true) Y(4, 0, 1, 0, false) Y(16, 0, 1, 0, false)
    Y(8, 1, 0, 0, false) Y(8, 1, 1, 0, false) Y(8, 1, 0, 1, false) Y(8, 1, 1, 0, true) Y(4, 1, 1, 0, false)
    Y(16, 1, 1, 0, false)
    return 0;
}
