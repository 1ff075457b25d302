// ubench_xpol.hip -- round 3: the halo's x faces (2 Mi lines, one 8-byte element per 128-byte
// line) gathered with each load cache policy, then scattered back with non-temporal stores (the
// engine's unpack policy), in the engine's face-major order.  With non-temporal gathers the
// scatter's partial writes go to DRAM as read-modify-writes; with plain gathers they merge in the
// Infinity Cache, but the gather itself is slower.  Is there a policy with both?
//   P0 plain, P1 nt, P2 sc1, P3 nt sc1, P4 nt sc0 sc1, P5 sc0 sc1
// Inline-asm loads (vector loads, explicit vmcnt wait).  Not the product.
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

template <int ORDER>
__device__ __forceinline__ size_t user_off(uint32_t e)
{
    uint32_t f, side, r;   // field, face, row within the field (16 bits)
    if (ORDER == 0) { f = e >> 17; side = (e >> 16) & 1; r = e & 0xFFFF; }
    else if (ORDER == 1) { f = e >> 17; side = e & 1; r = (e >> 1) & 0xFFFF; }
    else if (ORDER == 2) { f = e >> 17; side = (e >> 5) & 1; r = ((e >> 6) << 5 | (e & 31)) & 0xFFFF; }
    else if (ORDER == 3) { f = e & 15; side = (e >> 4) & 1; r = e >> 5; }
    else { f = e >> 17; side = (e >> 16) & 1; r = __brev(e & 0xFFFF) >> 16; }
    return size_t((f << 16) | r) * 2048 + side * 2040;
}

template <int POL>
__device__ __forceinline__ u32x2 ldx(const void *p)
{
    u32x2 v;
    if constexpr (POL == 0) asm volatile("global_load_dwordx2 %0, %1, off" : "=v"(v) : "v"(p) : "memory");
    else if constexpr (POL == 1) asm volatile("global_load_dwordx2 %0, %1, off nt" : "=v"(v) : "v"(p) : "memory");
    else if constexpr (POL == 2) asm volatile("global_load_dwordx2 %0, %1, off sc1" : "=v"(v) : "v"(p) : "memory");
    else if constexpr (POL == 3) asm volatile("global_load_dwordx2 %0, %1, off sc1 nt" : "=v"(v) : "v"(p) : "memory");
    else if constexpr (POL == 4) asm volatile("global_load_dwordx2 %0, %1, off sc0 sc1 nt" : "=v"(v) : "v"(p) : "memory");
    else asm volatile("global_load_dwordx2 %0, %1, off sc0 sc1" : "=v"(v) : "v"(p) : "memory");
    return v;
}

template <int K, int POL>
__global__ __launch_bounds__(256) void gather(const uint8_t *__restrict__ user, u32x2 *__restrict__ packed)
{
    const uint32_t base = blockIdx.x * 256 * K + threadIdx.x;
    u32x2 v[K];
#pragma unroll
    for (int k = 0; k < K; ++k)
        v[k] = ldx<POL>(user + user_off<0>(base + k * 256));
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int k = 0; k < K; ++k) packed[base + k * 256] = v[k];
}

template <int K, int ORDER>
__global__ __launch_bounds__(256) void scatter(uint8_t *__restrict__ user, const u32x2 *__restrict__ packed)
{
    const uint32_t base = blockIdx.x * 256 * K + threadIdx.x;
    u32x2 v[K];
#pragma unroll
    for (int k = 0; k < K; ++k) v[k] = packed[base + k * 256];
#pragma unroll
    for (int k = 0; k < K; ++k)
        __builtin_nontemporal_store(v[k], reinterpret_cast<u32x2 *>(user + user_off<ORDER>(base + k * 256)));
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
    u32x2 *P_;
    u32x4 *F, *SINK;
    const size_t FV = (1ull << 30) / 16;
    CHK(hipMalloc(&U, size_t(ROWS) * 2048));
    CHK(hipMalloc(&P_, size_t(NE) * 8));
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
    auto run = [&](auto gath, auto scat, const char *name) {
        std::vector<float> g1, s1, gp, sp, gf, sf;
        for (int mode = 0; mode < 4; ++mode) {
            // every repetition enqueued before any wait: the events see device time only
            for (int i = 0; i < n; ++i) {
                const bool flush = mode == 3;
                hipEvent_t *q = &ev[4 * i];
                if (flush) hipLaunchKernelGGL(flush_read, dim3(4096), blk, 0, 0, F, SINK, FV);
                CHK(hipEventRecord(q[0]));
                if (mode != 1) gath();
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
        printf("gather %-10s | gather-only %6.1f us (%4.1f G lines/s) | scatter-only %6.1f us | pair: gather %6.1f "
               "scatter %6.1f step %6.1f us | cold-clean: gather %6.1f scatter %6.1f us\n",
               name, med(g1), NE / med(g1) / 1e3, med(s1), med(gp), med(sp), med(gp) + med(sp), med(gf), med(sf));
    };
#define POLV(P, NAME)                                                                                   \
    run([&] { hipLaunchKernelGGL((gather<K, P>), grid, blk, 0, 0, U, P_); },                            \
        [&] { hipLaunchKernelGGL((scatter<K, 0>), grid, blk, 0, 0, U, P_); }, NAME);
    for (int round = 0; round < 2; ++round) {
        POLV(0, "plain") POLV(1, "nt") POLV(2, "sc1") POLV(3, "sc1 nt") POLV(4, "sc0 sc1 nt") POLV(5, "sc0 sc1")
    }
    return 0;
}
