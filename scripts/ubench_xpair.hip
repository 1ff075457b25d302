// ubench_xpair.hip -- the floor of the halo's x faces without the engine (round 3).
// Both x faces of 16 fields of a 256^3 double grid: 2 Mi 8-byte elements, one per 128-byte
// line (x- at byte 0, x+ at byte 2040 of every 2 KiB row), gathered into a contiguous stream
// and scattered back to the SAME lines, as bench.py's pack + unpack step does.  Bare kernels
// (K elements per thread in flight, the engine's unroll) timed with events:
//   gather-only and scatter-only loops, the gather+scatter pair loop (the bench step), and the
//   pair with a 1 GiB read between operations (the cold-clean protocol).
// Store variants of the scatter: plain, write-through (sc1), non-temporal.  Not the product.
#include <hip/hip_runtime.h>

#include <algorithm>
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

typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr uint32_t ROWS = 16u * 65536u;   // 16 fields x 256 planes x 256 rows
constexpr uint32_t NE = 2 * ROWS;         // both x faces

// element e of the packed stream (field-major, then face, then row, like the halo struct)
__device__ __forceinline__ size_t user_off(uint32_t e)
{
    const uint32_t f = e >> 17, side = (e >> 16) & 1, row = (f << 16) | (e & 0xFFFF);
    return size_t(row) * 2048 + side * 2040;
}

template <int K>
__global__ __launch_bounds__(256) void gather(const uint8_t *__restrict__ user, u32x2 *__restrict__ packed)
{
    const uint32_t base = blockIdx.x * 256 * K + threadIdx.x;
    u32x2 v[K];
#pragma unroll
    for (int k = 0; k < K; ++k)
        v[k] = __builtin_nontemporal_load(reinterpret_cast<const u32x2 *>(user + user_off(base + k * 256)));
#pragma unroll
    for (int k = 0; k < K; ++k) packed[base + k * 256] = v[k];
}

template <int K, int MODE>
__global__ __launch_bounds__(256) void scatter(uint8_t *__restrict__ user, const u32x2 *__restrict__ packed)
{
    const uint32_t base = blockIdx.x * 256 * K + threadIdx.x;
    u32x2 v[K];
#pragma unroll
    for (int k = 0; k < K; ++k) v[k] = packed[base + k * 256];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        u32x2 *p = reinterpret_cast<u32x2 *>(user + user_off(base + k * 256));
        if constexpr (MODE == 0) *p = v[k];
        else if constexpr (MODE == 1) asm volatile("global_store_dwordx2 %0, %1, off sc1" ::"v"(p), "v"(v[k]) : "memory");
        else __builtin_nontemporal_store(v[k], p);
    }
}

__global__ __launch_bounds__(256) void flush_read(const u32x4 *__restrict__ a, u32x4 *__restrict__ sink, size_t nv)
{
    u32x4 acc = {0, 0, 0, 0};
    for (size_t i = size_t(blockIdx.x) * 256 + threadIdx.x; i < nv; i += size_t(gridDim.x) * 256) acc ^= a[i];
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) sink[threadIdx.x] = acc;
}

static float med(std::vector<float> v)
{
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

int main()
{
    uint8_t *U;
    u32x2 *P;
    u32x4 *F, *SINK;
    const size_t FV = (1ull << 30) / 16;
    CHK(hipMalloc(&U, size_t(ROWS) * 2048));
    CHK(hipMalloc(&P, size_t(NE) * 8));
    CHK(hipMalloc(&F, FV * 16));
    CHK(hipMalloc(&SINK, 4096));
    CHK(hipMemset(U, 1, size_t(ROWS) * 2048));
    CHK(hipMemset(F, 2, FV * 16));
    constexpr int K = 8;
    const dim3 grid(NE / (256 * K)), blk(256);
    const int reps = 30, n = reps + 3;
    std::vector<hipEvent_t> ev(4 * n);
    for (auto &h : ev) CHK(hipEventCreate(&h));
    printf("x faces of 16 fields: %u lines gathered + scattered (2 Mi), K = %d\n", NE, K);
    auto run = [&](auto scat, const char *name) {
        std::vector<float> g1, s1, gp, sp, gf, sf;
        for (int mode = 0; mode < 4; ++mode) {
            // every repetition enqueued before any wait: the events see device time only
            for (int i = 0; i < n; ++i) {
                const bool flush = mode == 3;
                hipEvent_t *q = &ev[4 * i];
                if (flush) hipLaunchKernelGGL(flush_read, dim3(4096), blk, 0, 0, F, SINK, FV);
                CHK(hipEventRecord(q[0]));
                if (mode != 1) hipLaunchKernelGGL((gather<K>), grid, blk, 0, 0, U, P);
                CHK(hipEventRecord(q[1]));
                if (flush) hipLaunchKernelGGL(flush_read, dim3(4096), blk, 0, 0, F, SINK, FV);
                CHK(hipEventRecord(q[2]));
                if (mode != 0) scat();
                CHK(hipEventRecord(q[3]));
            }
            CHK(hipDeviceSynchronize());
            for (int i = 3; i < n; ++i) {
                hipEvent_t *q = &ev[4 * i];
                float a, b;
                CHK(hipEventElapsedTime(&a, q[0], q[1]));
                CHK(hipEventElapsedTime(&b, q[2], q[3]));
                if (mode == 0) g1.push_back(a * 1e3f);
                if (mode == 1) s1.push_back(b * 1e3f);
                if (mode == 2) { gp.push_back(a * 1e3f); sp.push_back(b * 1e3f); }
                if (mode == 3) { gf.push_back(a * 1e3f); sf.push_back(b * 1e3f); }
            }
        }
        printf("scatter %-13s | gather-only %6.1f us (%4.1f G lines/s) | scatter-only %6.1f us | pair: gather %6.1f "
               "scatter %6.1f step %6.1f us | cold-clean: gather %6.1f scatter %6.1f us\n",
               name, med(g1), NE / med(g1) / 1e3, med(s1), med(gp), med(sp), med(gp) + med(sp), med(gf), med(sf));
    };
    run([&] { hipLaunchKernelGGL((scatter<K, 0>), grid, blk, 0, 0, U, P); }, "plain");
    run([&] { hipLaunchKernelGGL((scatter<K, 1>), grid, blk, 0, 0, U, P); }, "sc1");
    run([&] { hipLaunchKernelGGL((scatter<K, 2>), grid, blk, 0, 0, U, P); }, "nontemporal");
    return 0;
}
