// ubench_gran.hip -- what an isolated narrow gather costs at the memory side on gfx950
// (round 2): is the x-face read (8 bytes every 2 KiB) fetched as a 64-byte or a 128-byte
// request?  Three kernels touch the same 2 Mi lines of a 4 GiB buffer (one per 2 KiB):
//   g8   : one 8-byte load per line           (the x-face gather)
//   l64  : 64 bytes per line (4 lanes x 16 B)
//   l128 : 128 bytes per line (8 lanes x 16 B)
// Their times and, under rocprofv3 --pmc, TCC_EA0_RDREQ / _RDREQ_32B / FETCH_SIZE per
// kernel say which granularity the single gather pays for.  Not part of the product.
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
constexpr uint32_t LINES = 2u << 20;     // 2 Mi lines
constexpr size_t STRIDE = 2048;          // one line per 2 KiB (the x-face stride)

// BYTES per line: 8 (one lane), 64 (4 lanes x 16 B) or 128 (8 lanes x 16 B)
template <int BYTES>
__global__ __launch_bounds__(256) void touch(const uint8_t *__restrict__ g, u32x4 *__restrict__ out)
{
    constexpr int LPL = BYTES >= 16 ? BYTES / 16 : 1;   // lanes per line
    const uint32_t gid = blockIdx.x * 256u + threadIdx.x;
    const uint32_t line = gid / LPL, sub = gid % LPL;
    if (line >= LINES)
        return;
    const uint8_t *p = g + size_t(line) * STRIDE;
    u32x4 v;
    if constexpr (BYTES == 8) {
        const uint64_t x = __builtin_nontemporal_load(reinterpret_cast<const uint64_t *>(p));
        v = u32x4{uint32_t(x), uint32_t(x >> 32), 0u, 0u};
    } else {
        v = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(p) + sub);
    }
    if ((v.x ^ v.y ^ v.z ^ v.w) == 0x9e3779b9u)   // never true: keeps the loads alive
        out[gid] = v;
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
    uint8_t *g;
    u32x4 *out;
    const size_t bytes = size_t(LINES) * STRIDE;   // 4 GiB
    CHK(hipMalloc(&g, bytes));
    CHK(hipMalloc(&out, size_t(LINES) * 8 * sizeof(u32x4)));
    CHK(hipMemset(g, 1, bytes));
    const uint32_t b8 = LINES / 256, b64 = LINES * 4 / 256, b128 = LINES * 8 / 256;
    const float t8 = timeit([&] { hipLaunchKernelGGL(touch<8>, dim3(b8), dim3(256), 0, 0, g, out); }, iters);
    const float t64 = timeit([&] { hipLaunchKernelGGL(touch<64>, dim3(b64), dim3(256), 0, 0, g, out); }, iters);
    const float t128 = timeit([&] { hipLaunchKernelGGL(touch<128>, dim3(b128), dim3(256), 0, 0, g, out); }, iters);
    printf("2 Mi lines at a 2 KiB stride: 8 B each %.1f us (%.1f G lines/s) | 64 B each %.1f us (%.1f) | "
           "128 B each %.1f us (%.1f)\n",
           t8, LINES / t8 / 1e3, t64, LINES / t64 / 1e3, t128, LINES / t128 / 1e3);
    return 0;
}
