// ubench6.hip -- x-face gather under every load cache policy of gfx950 (sc0 / sc1 / nt
// bits), to see whether any of them changes the memory-side request size or rate
// (tuning evidence, not product).  Both x faces of 16 fields of a 256^3 double grid:
// 2 Mi 8-byte loads at a 2 KiB stride; kernels are named per policy for rocprofv3 --pmc.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

constexpr size_t FIELD = 256ull * 256 * 256 * 8;
constexpr int NF = 16;
constexpr uint32_t ROWS = 65536;
constexpr uint32_t N = 2u * NF * ROWS;
constexpr int K = 8;

__device__ __forceinline__ size_t xaddr(uint32_t e)
{
    const uint32_t row = e % ROWS, r = e / ROWS, field = r % NF, face = r / NF;
    return size_t(field) * FIELD + size_t(row) * 2048 + (face ? 2040 : 0);
}

#define XG(NAME, ASM)                                                                          \
    __global__ __launch_bounds__(256) void NAME(const uint8_t *__restrict__ g, uint64_t *__restrict__ out) \
    {                                                                                          \
        const uint32_t base = blockIdx.x * 2048u;                                              \
        for (uint32_t e0 = base + threadIdx.x; e0 < base + 2048u; e0 += 256 * K) {             \
            uint64_t v[K];                                                                     \
            _Pragma("unroll") for (int k = 0; k < K; ++k)                                      \
                asm volatile(ASM : "=v"(v[k]) : "v"(g + xaddr(e0 + k * 256)) : "memory");      \
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");                                   \
            _Pragma("unroll") for (int k = 0; k < K; ++k) out[e0 + k * 256] = v[k];            \
        }                                                                                      \
    }

XG(xg_default, "global_load_dwordx2 %0, %1, off")
XG(xg_sc0, "global_load_dwordx2 %0, %1, off sc0")
XG(xg_sc1, "global_load_dwordx2 %0, %1, off sc1")
XG(xg_sc0sc1, "global_load_dwordx2 %0, %1, off sc0 sc1")
XG(xg_nt, "global_load_dwordx2 %0, %1, off nt")
XG(xg_sc0sc1nt, "global_load_dwordx2 %0, %1, off sc0 sc1 nt")
XG(xg_sc1nt, "global_load_dwordx2 %0, %1, off sc1 nt")

template <typename F> float timeit(F f, int it)
{
    hipEvent_t a, b; CHK(hipEventCreate(&a)); CHK(hipEventCreate(&b));
    f(); CHK(hipDeviceSynchronize());
    CHK(hipEventRecord(a)); for (int i = 0; i < it; ++i) f(); CHK(hipEventRecord(b));
    CHK(hipEventSynchronize(b)); float ms; CHK(hipEventElapsedTime(&ms, a, b)); return ms * 1000.f / it;
}

int main(int argc, char **argv)
{
    const int it = argc > 1 ? atoi(argv[1]) : 10;
    uint8_t *g; uint64_t *p;
    CHK(hipMalloc(&g, FIELD * NF)); CHK(hipMalloc(&p, size_t(N) * 8));
    CHK(hipMemset(g, 1, FIELD * NF));
    const dim3 grid(N / 2048), blk(256);
    struct { const char *name; void (*k)(const uint8_t *, uint64_t *); } ks[] = {
        {"default", xg_default}, {"sc0", xg_sc0}, {"sc1", xg_sc1}, {"sc0 sc1", xg_sc0sc1},
        {"nt", xg_nt}, {"sc0 sc1 nt", xg_sc0sc1nt}, {"sc1 nt", xg_sc1nt}};
    for (auto &k : ks) {
        float t = timeit([&] { hipLaunchKernelGGL(k.k, grid, blk, 0, 0, g, p); }, it);
        printf("gather %-12s %7.1f us  %5.1f G elem/s\n", k.name, t, N / t / 1e3);
    }
    return 0;
}
