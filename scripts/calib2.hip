// calib2.hip -- the halo's x-face pair (gather, then partial-line scatter on the SAME lines) under
// different load cache policies.  Round 5 question: the unpack's partial writes merge in the
// Infinity Cache when the lines the pack read are still there (a 1 Mi-line face: 26 us per
// unpack; the 16-field halo's 2 Mi lines = 256 MiB of 128-B lines, the whole cache: 78 us).  Do
// loads that fetch less than a 128-B line (uncached sc0/sc1 reads may go out as 32-B requests,
// TCC_EA0_RD_UNCACHED_32B) shrink the cache footprint so the pair merges at 2 Mi lines?  Not part
// of the product.
//
// Per (L, load policy, store policy): flush (1 GiB plain read), gather of one 8-B element per line
// at a 2 KiB pitch (timed), scatter of one 8-B element per line into the same lines (timed).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHK(x)                                                                          \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);       \
            std::exit(1);                                                               \
        }                                                                               \
    } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr size_t PITCH = 2048;

__global__ __launch_bounds__(256) void flush(const u32x4 *__restrict__ p, size_t n, uint32_t *sink)
{
    uint32_t acc = 0;
    for (size_t i = size_t(blockIdx.x) * 256 + threadIdx.x; i < n; i += size_t(gridDim.x) * 256) {
        const u32x4 v = p[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x9E3779B9u)
        sink[threadIdx.x] = acc;
}

// LP: 0 plain, 1 nt, 2 sc1, 3 sc0 sc1, 4 nt sc0 sc1
template <int LP>
__device__ __forceinline__ uint64_t load8(const uint8_t *p)
{
    uint64_t v;
    if constexpr (LP == 0) {
        v = *reinterpret_cast<const uint64_t *>(p);
    } else if constexpr (LP == 1) {
        v = __builtin_nontemporal_load(reinterpret_cast<const uint64_t *>(p));
    } else if constexpr (LP == 2) {
        asm volatile("global_load_dwordx2 %0, %1, off sc1\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
    } else if constexpr (LP == 3) {
        asm volatile("global_load_dwordx2 %0, %1, off sc0 sc1\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
    } else {
        asm volatile("global_load_dwordx2 %0, %1, off sc0 sc1 nt\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
    }
    return v;
}

template <int LP>
__global__ __launch_bounds__(256) void gather(const uint8_t *__restrict__ big, uint64_t *__restrict__ out, size_t L)
{
    const size_t t = size_t(blockIdx.x) * 256 + threadIdx.x;
    if (t < L)
        out[t] = load8<LP>(big + t * PITCH);
}

// SP: 0 plain, 1 nt
template <int SP>
__global__ __launch_bounds__(256) void scatter(uint8_t *__restrict__ big, const uint64_t *__restrict__ in, size_t L)
{
    const size_t t = size_t(blockIdx.x) * 256 + threadIdx.x;
    if (t >= L)
        return;
    uint64_t *q = reinterpret_cast<uint64_t *>(big + t * PITCH);
    if (SP)
        __builtin_nontemporal_store(in[t] + 1, q);
    else
        *q = in[t] + 1;
}

template <int LP>
void launch_gather(const uint8_t *big, uint64_t *out, size_t L)
{
    hipLaunchKernelGGL(gather<LP>, dim3(uint32_t((L + 255) / 256)), dim3(256), 0, nullptr, big, out, L);
}

int main(int argc, char **argv)
{
    const int reps = argc > 1 ? std::atoi(argv[1]) : 5;
    const size_t Lmax = size_t(4) << 20;
    uint8_t *big = nullptr;
    uint64_t *compact = nullptr;
    u32x4 *fl = nullptr;
    uint32_t *sink = nullptr;
    const size_t nflush = (size_t(1) << 30) / 16;
    CHK(hipMalloc(&big, Lmax * PITCH));
    CHK(hipMalloc(&compact, Lmax * 8));
    CHK(hipMalloc(&fl, nflush * 16));
    CHK(hipMalloc(&sink, 1024));
    CHK(hipMemset(big, 1, Lmax * PITCH));
    CHK(hipMemset(fl, 2, nflush * 16));
    CHK(hipDeviceSynchronize());
    hipEvent_t e0, e1, e2;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    CHK(hipEventCreate(&e2));
    const char *lname[5] = {"plain", "nt", "sc1", "sc0sc1", "nt_sc0sc1"};
    for (size_t L : {size_t(1) << 20, size_t(2) << 20, size_t(3) << 20, size_t(4) << 20})
        for (int lp = 0; lp < 5; ++lp)
            for (int sp = 0; sp < 2; ++sp) {
                float g = 0, s = 0;
                for (int r = 0; r < reps; ++r) {
                    hipLaunchKernelGGL(flush, dim3(4096), dim3(256), 0, nullptr, fl, nflush, sink);
                    CHK(hipEventRecord(e0, nullptr));
                    switch (lp) {
                    case 0: launch_gather<0>(big, compact, L); break;
                    case 1: launch_gather<1>(big, compact, L); break;
                    case 2: launch_gather<2>(big, compact, L); break;
                    case 3: launch_gather<3>(big, compact, L); break;
                    default: launch_gather<4>(big, compact, L); break;
                    }
                    CHK(hipEventRecord(e1, nullptr));
                    if (sp)
                        hipLaunchKernelGGL(scatter<1>, dim3(uint32_t((L + 255) / 256)), dim3(256), 0, nullptr, big,
                                           compact, L);
                    else
                        hipLaunchKernelGGL(scatter<0>, dim3(uint32_t((L + 255) / 256)), dim3(256), 0, nullptr, big,
                                           compact, L);
                    CHK(hipEventRecord(e2, nullptr));
                    CHK(hipEventSynchronize(e2));
                    float a = 0, b = 0;
                    CHK(hipEventElapsedTime(&a, e0, e1));
                    CHK(hipEventElapsedTime(&b, e1, e2));
                    g += a;
                    s += b;
                }
                std::printf("{\"lines\": %zu, \"load\": \"%s\", \"store\": \"%s\", \"gather_us\": %.2f, "
                            "\"scatter_us\": %.2f, \"gather_G_lines_s\": %.2f, \"scatter_G_lines_s\": %.2f}\n",
                            L, lname[lp], sp ? "nt" : "plain", g * 1e3 / reps, s * 1e3 / reps,
                            L / (g * 1e-3 / reps) / 1e9, L / (s * 1e-3 / reps) / 1e9);
            }
    return 0;
}
