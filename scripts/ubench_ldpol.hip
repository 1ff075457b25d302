// ubench_ldpol.hip -- round 3: does the cache-coherence scope of a load change what an isolated
// 8-byte gather costs?  The halo's x faces read one 8-byte element per 128-byte line (2 Mi lines
// at a 2 KiB stride); with default loads the L2 fetches the whole line (profiles/
// r2_ubench_gran.log).  Here the same gather with relaxed atomic loads at each memory scope
// (gfx950 encodes the scope in the instruction's sc0 / sc1 bits: wavefront none, workgroup sc0,
// agent sc1, system sc0 sc1) and with the non-temporal hint, timed with events; run under
// rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum to see the request size the L2 sends
// to memory.  Stores are not varied (the unpack's partial-line writes are settled at the memory
// side).  Not the product.
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

constexpr uint32_t NE = 2u << 20;   // lines
constexpr int K = 8;

template <int POL>
__device__ __forceinline__ uint64_t ld(const uint64_t *p)
{
    if constexpr (POL == 0) return *p;
    else if constexpr (POL == 1) return __builtin_nontemporal_load(p);
    else if constexpr (POL == 2) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    else if constexpr (POL == 3) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

template <int POL>
__global__ __launch_bounds__(256) void gather(const uint8_t *__restrict__ user, uint64_t *__restrict__ packed)
{
    const uint32_t base = blockIdx.x * 256 * K + threadIdx.x;
    uint64_t v[K];
#pragma unroll
    for (int k = 0; k < K; ++k)
        v[k] = ld<POL>(reinterpret_cast<const uint64_t *>(user + size_t(base + k * 256) * 2048));
#pragma unroll
    for (int k = 0; k < K; ++k) packed[base + k * 256] = v[k];
}

template <typename F>
float timeit(F f, int iters)
{
    std::vector<float> t;
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    for (int i = 0; i < iters + 2; ++i) {
        CHK(hipEventRecord(a));
        f();
        CHK(hipEventRecord(b));
        CHK(hipEventSynchronize(b));
        float ms;
        CHK(hipEventElapsedTime(&ms, a, b));
        if (i >= 2) t.push_back(ms * 1000.f);
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
}

int main(int argc, char **argv)
{
    const int iters = argc > 1 ? atoi(argv[1]) : 10;
    uint8_t *U;
    uint64_t *P;
    CHK(hipMalloc(&U, size_t(NE) * 2048));
    CHK(hipMalloc(&P, size_t(NE) * 8));
    CHK(hipMemset(U, 1, size_t(NE) * 2048));
    const dim3 grid(NE / (256 * K)), blk(256);
    const char *names[] = {"plain", "non-temporal", "workgroup (sc0)", "agent (sc1)", "system (sc0 sc1)"};
    float t[5];
    for (int round = 0; round < 2; ++round) {
        t[0] = timeit([&] { hipLaunchKernelGGL(gather<0>, grid, blk, 0, 0, U, P); }, iters);
        t[1] = timeit([&] { hipLaunchKernelGGL(gather<1>, grid, blk, 0, 0, U, P); }, iters);
        t[2] = timeit([&] { hipLaunchKernelGGL(gather<2>, grid, blk, 0, 0, U, P); }, iters);
        t[3] = timeit([&] { hipLaunchKernelGGL(gather<3>, grid, blk, 0, 0, U, P); }, iters);
        t[4] = timeit([&] { hipLaunchKernelGGL(gather<4>, grid, blk, 0, 0, U, P); }, iters);
        for (int i = 0; i < 5; ++i)
            printf("8-byte gather of 2 Mi lines, %-17s: %6.1f us (%4.1f G lines/s)\n", names[i], t[i], NE / t[i] / 1e3);
    }
    return 0;
}
