// ubench_masked.hip -- does reading a line before a partial write make the write cheaper?
// (round 2, cfg4's unpack scatter and the x-face unpack).  Not part of the product.
//
// The engine's scatters write a few elements per 128-byte line (cfg4: 4-byte elements, a
// quarter of the slots, in address order; x faces: 8 bytes per 2 KiB).  Each such write
// reaches memory as a byte-masked request, a read-modify-write there.  Variants over the
// same touched set:
//   mask   : masked stores only (what the engine does)
//   ld+mask: each lane first loads the 16 bytes around its slots (whole lines valid in L2),
//            then stores only its touched slots (legal: gap bytes are never written)
//   full   : load 16 B, merge, store 16 B (writes the gap bytes back: NOT legal for MPI,
//            the upper bound a whole-line write would give)
// Dense: 1 GiB, 4-byte slots, slot touched when hash(slot) % 4 == 0 (~1/4, like cfg4).
// Sparse: 2 Mi lines at a 2 KiB stride, one 8-byte element each (the x face).
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
constexpr size_t DENSE = size_t(1) << 30;
constexpr uint32_t CHUNK = 16384;   // bytes per workgroup (one engine chunk)

__device__ __forceinline__ bool touched(uint32_t slot)
{
    uint32_t h = slot * 0x9e3779b1u;
    h ^= h >> 15;
    h *= 0x85ebca77u;
    h ^= h >> 13;
    return (h & 3u) == 0;
}

// MODE 0 mask, 1 ld+mask, 2 full
template <int MODE>
__global__ __launch_bounds__(256) void dense(uint32_t *__restrict__ g, uint32_t val)
{
    const size_t base = size_t(blockIdx.x) * CHUNK;
#pragma unroll
    for (int pass = 0; pass < int(CHUNK / 4096); ++pass) {
        const size_t off = base + size_t(pass) * 4096 + threadIdx.x * 16u;
        u32x4 *p = reinterpret_cast<u32x4 *>(reinterpret_cast<uint8_t *>(g) + off);
        const uint32_t s0 = uint32_t(off >> 2);
        if constexpr (MODE == 0) {
            uint32_t *q = reinterpret_cast<uint32_t *>(p);
            for (int k = 0; k < 4; ++k)
                if (touched(s0 + k)) q[k] = val + s0 + k;
        } else {
            u32x4 v = *p;
            if constexpr (MODE == 1) {
                uint32_t *q = reinterpret_cast<uint32_t *>(p);
                if (v.x != 0xdeadbeefu)   // always true: keeps the load
                    for (int k = 0; k < 4; ++k)
                        if (touched(s0 + k)) q[k] = val + s0 + k;
            } else {
                if (touched(s0 + 0)) v.x = val + s0;
                if (touched(s0 + 1)) v.y = val + s0 + 1;
                if (touched(s0 + 2)) v.z = val + s0 + 2;
                if (touched(s0 + 3)) v.w = val + s0 + 3;
                *p = v;
            }
        }
    }
}

constexpr uint32_t LINES = 2u << 20;
constexpr size_t STRIDE = 2048;

// MODE 0 mask (8 B), 1 one lane loads the line's first 16 B then stores 8 B, 2 8 lanes load
// the whole 128-byte line, lane 0 stores 8 B
template <int MODE>
__global__ __launch_bounds__(256) void sparse(uint8_t *__restrict__ g, uint64_t val)
{
    constexpr int LPL = MODE == 2 ? 8 : 1;
    const uint32_t gid = blockIdx.x * 256u + threadIdx.x;
    const uint32_t line = gid / LPL, sub = gid % LPL;
    if (line >= LINES)
        return;
    uint8_t *p = g + size_t(line) * STRIDE;
    if constexpr (MODE == 0) {
        *reinterpret_cast<uint64_t *>(p) = val + line;
    } else {
        const u32x4 v = reinterpret_cast<const u32x4 *>(p)[sub];
        if (sub == 0 && v.x != 0xdeadbeefu)
            *reinterpret_cast<uint64_t *>(p) = val + line;
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
    uint32_t *d;
    uint8_t *s;
    CHK(hipMalloc(&d, DENSE));
    CHK(hipMalloc(&s, size_t(LINES) * STRIDE));
    CHK(hipMemset(d, 1, DENSE));
    CHK(hipMemset(s, 1, size_t(LINES) * STRIDE));
    const uint32_t nb = uint32_t(DENSE / CHUNK);
    uint32_t k = 7;
    const float m0 = timeit([&] { hipLaunchKernelGGL(dense<0>, dim3(nb), dim3(256), 0, 0, d, k++); }, iters);
    const float m1 = timeit([&] { hipLaunchKernelGGL(dense<1>, dim3(nb), dim3(256), 0, 0, d, k++); }, iters);
    const float m2 = timeit([&] { hipLaunchKernelGGL(dense<2>, dim3(nb), dim3(256), 0, 0, d, k++); }, iters);
    printf("dense 1 GiB, 1/4 of 4-byte slots: mask %.1f us | ld+mask %.1f us | full (illegal) %.1f us\n", m0, m1, m2);
    // check: every touched slot holds the last value, untouched slots are 0x01010101
    {
        const size_t n = 1 << 20;
        uint32_t *h = (uint32_t *) malloc(n * 4);
        CHK(hipMemcpy(h, d, n * 4, hipMemcpyDeviceToHost));
        size_t bad = 0;
        for (size_t i = 0; i < n; ++i) {
            uint32_t x = uint32_t(i) * 0x9e3779b1u;
            x ^= x >> 15;
            x *= 0x85ebca77u;
            x ^= x >> 13;
            const uint32_t want = (x & 3u) == 0 ? (k - 1) + uint32_t(i) : 0x01010101u;
            bad += h[i] != want;
        }
        printf("dense check: %zu mismatches in the first 4 MiB\n", bad);
        free(h);
    }
    const uint32_t b1 = LINES / 256, b8 = LINES * 8 / 256;
    uint64_t v = 11;
    const float s0 = timeit([&] { hipLaunchKernelGGL(sparse<0>, dim3(b1), dim3(256), 0, 0, s, v++); }, iters);
    const float s1 = timeit([&] { hipLaunchKernelGGL(sparse<1>, dim3(b1), dim3(256), 0, 0, s, v++); }, iters);
    const float s2 = timeit([&] { hipLaunchKernelGGL(sparse<2>, dim3(b8), dim3(256), 0, 0, s, v++); }, iters);
    printf("sparse 2 Mi lines, 8 B at a 2 KiB stride: mask %.1f us (%.1f G/s) | ld16+mask %.1f us | "
           "ld128+mask %.1f us\n",
           s0, LINES / s0 / 1e3, s1, s2);
    return 0;
}
