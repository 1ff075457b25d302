// ubench7.hip -- one-element-per-line strided gather rate vs the span the gathers cover
// (tuning evidence for DESIGN.md §10: cfg3's dim-2 face gathers run slower than cfg2's
// x faces with the same request count).  2 Mi elements of E bytes at a fixed stride, the
// packed side coalesced, K = 8 loads in flight per lane and non-temporal user loads, as in
// the engine's sparse affine path.  Spans 1-8 GiB; element at offset 0 or at the last E
// bytes of its stride (cfg3's dim-2 face sits at byte 2044 of every 2 KiB row).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

constexpr uint32_t N = 2u << 20;       // elements
constexpr uint32_t PER_WG = 2048;      // one unrolled pass of 256 lanes x K
constexpr int K = 8;

template <typename T>
__global__ __launch_bounds__(256) void gat(const uint8_t *__restrict__ in, T *__restrict__ out, uint64_t stride,
                                           uint64_t off)
{
    const uint32_t base = blockIdx.x * PER_WG;
    T v[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const uint32_t e = base + threadIdx.x + k * 256;
        v[k] = __builtin_nontemporal_load(reinterpret_cast<const T *>(in + uint64_t(e) * stride + off));
    }
#pragma unroll
    for (int k = 0; k < K; ++k) out[base + threadIdx.x + k * 256] = v[k];
}

// read-only sweep of 1 GiB: evicts the gathered lines from the Infinity Cache without
// leaving dirty lines behind
__global__ __launch_bounds__(256) void sweep(const uint4 *__restrict__ p, size_t n, uint32_t *sink)
{
    uint32_t acc = 0;
    for (size_t i = size_t(blockIdx.x) * 256 + threadIdx.x; i < n; i += size_t(gridDim.x) * 256)
        acc ^= p[i].x ^ p[i].w;
    if (acc == 0x9E3779B9u) sink[0] = acc;
}

// per launch: the sweep first, so that no gathered line is still cached
template <typename F> float timeit(F f, int it, void *flush)
{
    hipEvent_t a, b; CHK(hipEventCreate(&a)); CHK(hipEventCreate(&b));
    float tot = 0;
    for (int i = 0; i < it; ++i) {
        hipLaunchKernelGGL(sweep, dim3(4096), dim3(256), 0, 0, (const uint4 *) flush, (size_t(1) << 30) / 16,
                           (uint32_t *) flush);
        CHK(hipEventRecord(a)); f(); CHK(hipEventRecord(b));
        CHK(hipEventSynchronize(b)); float ms; CHK(hipEventElapsedTime(&ms, a, b)); tot += ms;
    }
    return tot * 1000.f / it;
}

int main(int argc, char **argv)
{
    const int it = argc > 1 ? atoi(argv[1]) : 20;
    const uint64_t max_stride = 4096;
    uint8_t *a; void *b, *fl;
    CHK(hipMalloc(&a, size_t(N) * max_stride)); CHK(hipMalloc(&b, size_t(N) * 8));
    CHK(hipMalloc(&fl, size_t(1) << 30)); CHK(hipMemset(fl, 3, size_t(1) << 30));
    CHK(hipMemset(a, 1, size_t(N) * max_stride));
    const dim3 grid(N / PER_WG), blk(256);
    for (uint64_t stride : {512ull, 1024ull, 2048ull, 4096ull}) {
        for (int last = 0; last < 2; ++last) {
            const float t4 = timeit([&] { hipLaunchKernelGGL((gat<uint32_t>), grid, blk, 0, 0, a,
                                                             (uint32_t *) b, stride, last ? stride - 4 : 0); }, it, fl);
            const float t8 = timeit([&] { hipLaunchKernelGGL((gat<uint64_t>), grid, blk, 0, 0, a,
                                                             (uint64_t *) b, stride, last ? stride - 8 : 0); }, it, fl);
            printf("stride %5llu B span %5llu MiB %s | 4 B: %6.1f us %5.1f G/s | 8 B: %6.1f us %5.1f G/s\n",
                   (unsigned long long) stride, (unsigned long long) (stride * N >> 20),
                   last ? "end " : "head", t4, N / t4 / 1e3, t8, N / t8 / 1e3);
        }
    }
    return 0;
}
