// ubench.hip -- standalone gfx950 micro-benchmarks for the x-face access pattern
// (8-byte elements at a 2 KiB stride, 16 fields at 128 MiB stride) and plain
// streaming, to choose load/store forms for ddt_kernels.hip.  Not part of the product.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHK(x)                                                                          \
    do {                                                                                \
        hipError_t e = (x);                                                             \
        if (e != hipSuccess) {                                                          \
            printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);             \
            exit(1);                                                                    \
        }                                                                               \
    } while (0)

constexpr size_t FIELD = 256ull * 256 * 256 * 8;   // 128 MiB
constexpr int NF = 16;
constexpr uint32_t ROWS = 65536;                    // rows per field (x face elements)

enum Mode { PLAIN = 0, NT = 1, SC1 = 2, SC0SC1 = 3, LDS = 4 };

template <int MODE, int K, int FACES>
__global__ __launch_bounds__(256) void gather_x(const uint8_t *__restrict__ grid, uint64_t *__restrict__ out,
                                                uint32_t per_wg)
{
    // element e in [0, FACES*NF*ROWS): face f = e / (NF*ROWS), field = .., row = ..
    const uint32_t base = blockIdx.x * per_wg, end = base + per_wg;
    for (uint32_t e0 = base + threadIdx.x; e0 < end; e0 += 256 * K) {
        uint64_t v[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            uint32_t e = e0 + k * 256;
            if (e >= end) e = base;   // in-range dummy (result discarded below)
            uint32_t row = e % ROWS, rest = e / ROWS, field = rest % NF, face = rest / NF;
            const uint64_t *p = reinterpret_cast<const uint64_t *>(
                grid + size_t(field) * FIELD + size_t(row) * 2048 + (face ? 2040 : 0));
            if constexpr (MODE == NT)
                v[k] = __builtin_nontemporal_load(p);
            else if constexpr (MODE == SC1)
                v[k] = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            else if constexpr (MODE == SC0SC1)
                v[k] = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            else
                v[k] = *p;
        }
#pragma unroll
        for (int k = 0; k < K; ++k)
            if (e0 + k * 256 < end) out[e0 + k * 256] = v[k];
    }
}

template <int K, int FACES>
__global__ __launch_bounds__(256) void scatter_x(uint8_t *__restrict__ grid, const uint64_t *__restrict__ in,
                                                 uint32_t per_wg, int nt)
{
    const uint32_t base = blockIdx.x * per_wg, end = base + per_wg;
    for (uint32_t e0 = base + threadIdx.x; e0 < end; e0 += 256 * K) {
        uint64_t v[K];
#pragma unroll
        for (int k = 0; k < K; ++k)
            v[k] = in[(e0 + k * 256 < end) ? e0 + k * 256 : base];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            uint32_t e = e0 + k * 256;
            if (e >= end) continue;
            uint32_t row = e % ROWS, rest = e / ROWS, field = rest % NF, face = rest / NF;
            uint64_t *p = reinterpret_cast<uint64_t *>(grid + size_t(field) * FIELD + size_t(row) * 2048 + (face ? 2040 : 0));
            if (nt) __builtin_nontemporal_store(v[k], p);
            else *p = v[k];
        }
    }
}

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
template <int K>
__global__ __launch_bounds__(256) void stream_copy(const u32x4 *__restrict__ a, u32x4 *__restrict__ b, uint32_t per_wg)
{
    const uint32_t base = blockIdx.x * per_wg, end = base + per_wg;
    for (uint32_t i = base + threadIdx.x; i < end; i += 256 * K) {
        u32x4 v[K];
#pragma unroll
        for (int k = 0; k < K; ++k) v[k] = a[(i + k * 256 < end) ? i + k * 256 : base];
#pragma unroll
        for (int k = 0; k < K; ++k) if (i + k * 256 < end) b[i + k * 256] = v[k];
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

int main()
{
    uint8_t *grid;
    uint64_t *packed;
    CHK(hipMalloc(&grid, FIELD * NF));
    CHK(hipMalloc(&packed, 2ull * NF * ROWS * 8));
    CHK(hipMemset(grid, 1, FIELD * NF));
    const uint32_t N = 2 * NF * ROWS;   // both x faces: 2 Mi elements
    // every launch below covers exactly [0, N) (or the copy range) with per_wg | N
    const int it = 20;
    for (uint32_t per : {1024u, 2048u, 4096u, 8192u}) {
        uint32_t wg = N / per;
        if (wg * per != N) { printf("bad split\n"); return 1; }
        float t0 = timeit([&] { hipLaunchKernelGGL((gather_x<PLAIN, 8, 2>), dim3(wg), dim3(256), 0, 0, grid, packed, per); }, it);
        float t1 = timeit([&] { hipLaunchKernelGGL((gather_x<NT, 8, 2>), dim3(wg), dim3(256), 0, 0, grid, packed, per); }, it);
        float t2 = timeit([&] { hipLaunchKernelGGL((gather_x<SC1, 8, 2>), dim3(wg), dim3(256), 0, 0, grid, packed, per); }, it);
        float t3 = timeit([&] { hipLaunchKernelGGL((gather_x<SC0SC1, 8, 2>), dim3(wg), dim3(256), 0, 0, grid, packed, per); }, it);
        float t4 = timeit([&] { hipLaunchKernelGGL((gather_x<PLAIN, 4, 2>), dim3(wg), dim3(256), 0, 0, grid, packed, per); }, it);
        float t5 = timeit([&] { hipLaunchKernelGGL((gather_x<PLAIN, 16, 2>), dim3(wg), dim3(256), 0, 0, grid, packed, per); }, it);
        float s0 = timeit([&] { hipLaunchKernelGGL((scatter_x<8, 2>), dim3(wg), dim3(256), 0, 0, grid, packed, per, 0); }, it);
        float s1 = timeit([&] { hipLaunchKernelGGL((scatter_x<8, 2>), dim3(wg), dim3(256), 0, 0, grid, packed, per, 1); }, it);
        printf("per_wg %5u wgs %6u | gather us: plain %.1f nt %.1f sc1 %.1f sys %.1f K4 %.1f K16 %.1f | scatter us: plain %.1f nt %.1f | Gelem/s plain %.1f\n",
               per, wg, t0, t1, t2, t3, t4, t5, s0, s1, N / t0 / 1e3);
    }
    // streaming copy calibration, 512 MiB and 32 MiB
    for (size_t bytes : {512ull << 20, 32ull << 20}) {
        uint32_t n = uint32_t(bytes / 16);
        if ((1ull << 30) + bytes > FIELD * NF) { printf("bad copy size\n"); return 1; }
        for (uint32_t per : {4096u, 16384u}) {
            if ((n / per) * per != n) { printf("bad split\n"); return 1; }
            float t = timeit([&] { hipLaunchKernelGGL((stream_copy<4>), dim3(n / per), dim3(256), 0, 0, (const u32x4 *) grid, (u32x4 *) (grid + (1ull << 30)), per); }, it);
            printf("copy %4zu MiB per_wg %5u: %.1f us  %.0f GB/s (r+w)\n", bytes >> 20, per * 16, t, 2.0 * bytes / t / 1e3);
        }
    }
    return 0;
}
