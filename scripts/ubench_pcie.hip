// ubench_pcie.hip -- how fast can a kernel move bytes to and from pinned host memory over
// PCIe, against the DMA engines (round 2, the e2e "hostdirect" path): 48 MiB, the cfg2
// packed stream.  Rows:
//   dma   : hipMemcpyAsync D2H / H2D
//   kern  : a copy kernel, G workgroups x 256 lanes x 16 B, plain or non-temporal host stores
//   split : a kernel moves the first part while the DMA engine moves the rest, two streams
// for host memory from hipHostMalloc default flags (what torch pin_memory hands out) and
// hipHostMallocNonCoherent.  Not part of the product.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CHK(x)                                                                          \
    do {                                                                                \
        hipError_t e = (x);                                                             \
        if (e != hipSuccess) {                                                          \
            printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);             \
            exit(1);                                                                    \
        }                                                                               \
    } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr size_t BYTES = 48u << 20;

template <bool NT>
__global__ __launch_bounds__(256) void kcopy(const u32x4 *__restrict__ s, u32x4 *__restrict__ d, size_t n)
{
    for (size_t i = size_t(blockIdx.x) * 256 + threadIdx.x; i < n; i += size_t(gridDim.x) * 256) {
        const u32x4 v = s[i];
        if constexpr (NT)
            __builtin_nontemporal_store(v, d + i);
        else
            d[i] = v;
    }
}

// narrow lanes: W-byte stores per lane (the pack of 8-B / 4-B gathers writes the packed stream so)
template <typename T>
__global__ __launch_bounds__(256) void kcopy_w(const T *__restrict__ s, T *__restrict__ d, size_t n)
{
    for (size_t i = size_t(blockIdx.x) * 256 + threadIdx.x; i < n; i += size_t(gridDim.x) * 256)
        d[i] = s[i];
}

// one workgroup owns a contiguous chunk (the convertor's task layout)
__global__ __launch_bounds__(256) void kcopy_chunked(const u32x4 *__restrict__ s, u32x4 *__restrict__ d,
                                                     size_t n, size_t per)
{
    const size_t b = size_t(blockIdx.x) * per, e = b + per < n ? b + per : n;
    for (size_t i = b + threadIdx.x; i < e; i += 256)
        d[i] = s[i];
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
    CHK(hipDeviceSynchronize());
    float ms;
    CHK(hipEventElapsedTime(&ms, a, b));
    return ms * 1000.f / iters;
}

static double gbs(float us) { return BYTES / (us * 1e3); }

int main(int argc, char **argv)
{
    const int iters = argc > 1 ? atoi(argv[1]) : 10;
    const size_t n = BYTES / 16;
    void *dbuf;
    CHK(hipMalloc(&dbuf, BYTES));
    CHK(hipMemset(dbuf, 3, BYTES));
    hipStream_t s2;
    CHK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    const unsigned flags[2] = {hipHostMallocDefault, hipHostMallocNonCoherent};
    const char *fname[2] = {"default", "noncoherent"};
    for (int fi = 0; fi < (argc > 2 ? 2 : 1); ++fi) {
        void *h;
        CHK(hipHostMalloc(&h, BYTES, flags[fi]));
        memset(h, 1, BYTES);
        const u32x4 *D = (const u32x4 *) dbuf;
        u32x4 *H = (u32x4 *) h;
        printf("[%s host memory]\n", fname[fi]);
        const float td = timeit([&] { CHK(hipMemcpyAsync(h, dbuf, BYTES, hipMemcpyDeviceToHost, 0)); }, iters);
        const float th = timeit([&] { CHK(hipMemcpyAsync(dbuf, h, BYTES, hipMemcpyHostToDevice, 0)); }, iters);
        printf("  dma D2H %.1f us %.2f GB/s | H2D %.1f us %.2f GB/s\n", td, gbs(td), th, gbs(th));
        for (int g : {64, 128, 256, 512, 1024, 2048, 8192}) {
            const float kw = timeit([&] { hipLaunchKernelGGL(kcopy<false>, dim3(g), dim3(256), 0, 0, D, H, n); }, iters);
            const float kn = timeit([&] { hipLaunchKernelGGL(kcopy<true>, dim3(g), dim3(256), 0, 0, D, H, n); }, iters);
            const float kr = timeit([&] { hipLaunchKernelGGL(kcopy<false>, dim3(g), dim3(256), 0, 0, (const u32x4 *) H,
                                                             (u32x4 *) dbuf, n); }, iters);
            printf("  kern G=%5d  write %.1f us %.2f GB/s | nt write %.1f us %.2f GB/s | read %.1f us %.2f GB/s\n", g, kw,
                   gbs(kw), kn, gbs(kn), kr, gbs(kr));
        }
        for (int g : {256, 1024, 4096}) {
            const float k8 = timeit([&] { hipLaunchKernelGGL(kcopy_w<uint64_t>, dim3(g), dim3(256), 0, 0,
                                                             (const uint64_t *) dbuf, (uint64_t *) h, BYTES / 8); }, iters);
            const float k4 = timeit([&] { hipLaunchKernelGGL(kcopy_w<uint32_t>, dim3(g), dim3(256), 0, 0,
                                                             (const uint32_t *) dbuf, (uint32_t *) h, BYTES / 4); }, iters);
            printf("  kern G=%5d  8-B lanes write %.1f us %.2f GB/s | 4-B lanes write %.1f us %.2f GB/s\n", g, k8, gbs(k8),
                   k4, gbs(k4));
        }
        for (size_t per : {size_t(4096), size_t(16384), size_t(65536)}) {   // 16-B units per workgroup
            const unsigned g = unsigned((n + per - 1) / per);
            const float kc = timeit([&] { hipLaunchKernelGGL(kcopy_chunked, dim3(g), dim3(256), 0, 0, D, H, n, per); }, iters);
            printf("  kern chunked %zu KiB per workgroup (%u wgs) write %.1f us %.2f GB/s\n", per * 16 / 1024, g, kc, gbs(kc));
        }
        for (int pct : {25, 50, 75}) {
            const size_t nk = n * pct / 100, off = nk * 16;
            const float tw = timeit([&] {
                hipLaunchKernelGGL(kcopy<false>, dim3(1024), dim3(256), 0, 0, D, H, nk);
                CHK(hipMemcpyAsync((char *) h + off, (char *) dbuf + off, BYTES - off, hipMemcpyDeviceToHost, s2));
                CHK(hipStreamSynchronize(s2));
            }, iters);
            const float tr = timeit([&] {
                hipLaunchKernelGGL(kcopy<false>, dim3(1024), dim3(256), 0, 0, (const u32x4 *) H, (u32x4 *) dbuf, nk);
                CHK(hipMemcpyAsync((char *) dbuf + off, (char *) h + off, BYTES - off, hipMemcpyHostToDevice, s2));
                CHK(hipStreamSynchronize(s2));
            }, iters);
            printf("  split kernel %d%% + dma: write %.1f us %.2f GB/s | read %.1f us %.2f GB/s\n", pct, tw, gbs(tw), tr,
                   gbs(tr));
        }
        CHK(hipHostFree(h));
    }
    return 0;
}
