// ubench4.hip -- memory-REQUEST accounting for the x-face pattern on gfx950 (tuning
// evidence, not product).  Kernels are named so a rocprofv3 --pmc pass can attribute
// TCC_EA0_RDREQ / TCC_BUBBLE / TCC_EA0_WRREQ per access form:
//   xg_*   : gather both x faces of NF 256^3 double fields (8 B at 2 KiB stride)
//   xs_*   : scatter into the same elements (plain / line-prefetched / nt)
//   copy16 : 16 B-per-lane streaming copy (calibration: 128 B requests?)
//   read16 : 16 B-per-lane streaming read-only (the read roofline)
// Usage: ubench4 [iters]   (prints us per launch and G elements or GB/s)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

constexpr size_t FIELD = 256ull * 256 * 256 * 8;   // 128 MiB
constexpr int NF = 16;                              // 2 GiB: the bench's working set
constexpr uint32_t ROWS = 65536;
constexpr uint32_t N = 2u * NF * ROWS;              // 2 Mi x-face elements
constexpr int K = 8;

__device__ __forceinline__ size_t xaddr(uint32_t e)
{
    const uint32_t row = e % ROWS, r = e / ROWS, field = r % NF, face = r / NF;
    return size_t(field) * FIELD + size_t(row) * 2048 + (face ? 2040 : 0);
}

__global__ __launch_bounds__(256) void xg_plain(const uint8_t *__restrict__ g, uint64_t *__restrict__ out)
{
    const uint32_t base = blockIdx.x * 2048u;
    for (uint32_t e0 = base + threadIdx.x; e0 < base + 2048u; e0 += 256 * K) {
        uint64_t v[K];
#pragma unroll
        for (int k = 0; k < K; ++k) v[k] = *reinterpret_cast<const uint64_t *>(g + xaddr(e0 + k * 256));
#pragma unroll
        for (int k = 0; k < K; ++k) out[e0 + k * 256] = v[k];
    }
}

// 4-byte halves: does a narrower access change the request size?
__global__ __launch_bounds__(256) void xg_dword(const uint8_t *__restrict__ g, uint32_t *__restrict__ out)
{
    const uint32_t base = blockIdx.x * 4096u;
    for (uint32_t e0 = base + threadIdx.x; e0 < base + 4096u; e0 += 256 * K) {
        uint32_t v[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint32_t e = e0 + k * 256;
            v[k] = *reinterpret_cast<const uint32_t *>(g + xaddr(e >> 1) + (e & 1) * 4);
        }
#pragma unroll
        for (int k = 0; k < K; ++k) out[e0 + k * 256] = v[k];
    }
}

template <int MODE>   // 0 plain, 1 nt store, 2 load-the-line-then-store, 3 sc1 (agent) store
__global__ __launch_bounds__(256) void xs(uint8_t *__restrict__ g, const uint64_t *__restrict__ in)
{
    const uint32_t base = blockIdx.x * 2048u;
    for (uint32_t e0 = base + threadIdx.x; e0 < base + 2048u; e0 += 256 * K) {
        uint64_t v[K];
#pragma unroll
        for (int k = 0; k < K; ++k) v[k] = in[e0 + k * 256];
        if (MODE == 2) {
            uint64_t old[K];
#pragma unroll
            for (int k = 0; k < K; ++k) old[k] = *reinterpret_cast<volatile const uint64_t *>(g + xaddr(e0 + k * 256));
#pragma unroll
            for (int k = 0; k < K; ++k) asm volatile("" ::"v"(old[k]));
        }
#pragma unroll
        for (int k = 0; k < K; ++k) {
            uint64_t *p = reinterpret_cast<uint64_t *>(g + xaddr(e0 + k * 256));
            if (MODE == 1) __builtin_nontemporal_store(v[k], p);
            else if (MODE == 3) __hip_atomic_store(p, v[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            else *p = v[k];
        }
    }
}

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void copy16(const u32x4 *__restrict__ a, u32x4 *__restrict__ b)
{
    const uint32_t base = blockIdx.x * 4096u;
    for (uint32_t r = 0; r < 4096u; r += 1024u) {
        u32x4 v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = a[base + r + k * 256 + threadIdx.x];
#pragma unroll
        for (int k = 0; k < 4; ++k) b[base + r + k * 256 + threadIdx.x] = v[k];
    }
}

__global__ __launch_bounds__(256) void read16(const u32x4 *__restrict__ a, unsigned *__restrict__ sink)
{
    const uint32_t base = blockIdx.x * 4096u;
    u32x4 acc = {0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < 16; ++k) acc ^= a[base + k * 256 + threadIdx.x];
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) sink[0] = 1;
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
    const int it = argc > 1 ? atoi(argv[1]) : 10;
    static_assert(N % 2048 == 0, "grid split");
    uint8_t *g, *c;
    uint64_t *p;
    unsigned *sink;
    const size_t CB = 512ull << 20;   // copy / read size
    CHK(hipMalloc(&g, FIELD * NF)); CHK(hipMalloc(&p, size_t(N) * 8));
    CHK(hipMalloc(&c, 2 * CB)); CHK(hipMalloc(&sink, 4));
    CHK(hipMemset(g, 1, FIELD * NF)); CHK(hipMemset(p, 2, size_t(N) * 8)); CHK(hipMemset(c, 3, 2 * CB));
    const dim3 blk(256);
    float t;
    t = timeit([&] { hipLaunchKernelGGL(xg_plain, dim3(N / 2048), blk, 0, 0, g, p); }, it);
    printf("xg_plain     %7.1f us  %5.1f G elem/s\n", t, N / t / 1e3);
    t = timeit([&] { hipLaunchKernelGGL(xg_dword, dim3(2 * N / 4096), blk, 0, 0, g, (uint32_t *) p); }, it);
    printf("xg_dword     %7.1f us  %5.1f G dword/s (2 per element)\n", t, 2.0 * N / t / 1e3);
    t = timeit([&] { hipLaunchKernelGGL((xs<0>), dim3(N / 2048), blk, 0, 0, g, p); }, it);
    printf("xs_plain     %7.1f us  %5.1f G elem/s\n", t, N / t / 1e3);
    t = timeit([&] { hipLaunchKernelGGL((xs<1>), dim3(N / 2048), blk, 0, 0, g, p); }, it);
    printf("xs_nt        %7.1f us  %5.1f G elem/s\n", t, N / t / 1e3);
    t = timeit([&] { hipLaunchKernelGGL((xs<2>), dim3(N / 2048), blk, 0, 0, g, p); }, it);
    printf("xs_prefetch  %7.1f us  %5.1f G elem/s\n", t, N / t / 1e3);
    t = timeit([&] { hipLaunchKernelGGL((xs<3>), dim3(N / 2048), blk, 0, 0, g, p); }, it);
    printf("xs_sc1       %7.1f us  %5.1f G elem/s\n", t, N / t / 1e3);
    // pair loop: gather then scatter the same elements (the bench's pack+unpack order)
    t = timeit([&] {
        hipLaunchKernelGGL(xg_plain, dim3(N / 2048), blk, 0, 0, g, p);
        hipLaunchKernelGGL((xs<0>), dim3(N / 2048), blk, 0, 0, g, p);
    }, it);
    printf("pair plain   %7.1f us  (gather+scatter)\n", t);
    t = timeit([&] {
        hipLaunchKernelGGL(xg_plain, dim3(N / 2048), blk, 0, 0, g, p);
        hipLaunchKernelGGL((xs<2>), dim3(N / 2048), blk, 0, 0, g, p);
    }, it);
    printf("pair prefetch%7.1f us  (gather+scatter)\n", t);
    const uint32_t n16 = uint32_t(CB / 16);
    t = timeit([&] { hipLaunchKernelGGL(copy16, dim3(n16 / 4096), blk, 0, 0, (const u32x4 *) c, (u32x4 *) (c + CB)); }, it);
    printf("copy16       %7.1f us  %6.0f GB/s r+w\n", t, 2.0 * CB / t / 1e3);
    t = timeit([&] { hipLaunchKernelGGL(read16, dim3(n16 / 4096), blk, 0, 0, (const u32x4 *) c, sink); }, it);
    printf("read16       %7.1f us  %6.0f GB/s read\n", t, 1.0 * CB / t / 1e3);
    CHK(hipDeviceSynchronize());
    return 0;
}
