// ubench3.hip -- cfg4 (64 Mi unique random floats out of a 1 GiB buffer) access-order
// experiments on gfx950 (tuning only, not product).  Compares the direct gather with a
// two-phase "address-ordered read, then local permutation" scheme.
//   direct : packed[i] = user[d[i]]
//   phase 1: T[slot[k]] = user[s[k]]      (s = d sorted; slot = bucket-major position)
//   phase 2: packed[i]  = T[idx[i]]       (idx local to a bucket of NB packed elements)
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

constexpr uint32_t N = 64u << 20;        // elements
constexpr uint32_t RANGE = 1u << 28;     // floats in the user buffer (1 GiB)

__global__ __launch_bounds__(256) void direct(const float *__restrict__ u, const int *__restrict__ d,
                                              float *__restrict__ p, uint32_t n)
{
    for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) p[i] = u[d[i]];
}

__global__ __launch_bounds__(256) void phase1(const float *__restrict__ u, const int *__restrict__ s,
                                              const int *__restrict__ slot, float *__restrict__ T, uint32_t n)
{
    for (uint32_t k = blockIdx.x * 256 + threadIdx.x; k < n; k += gridDim.x * 256) T[slot[k]] = u[s[k]];
}

__global__ __launch_bounds__(256) void phase1_sorted_only(const float *__restrict__ u, const int *__restrict__ s,
                                                          float *__restrict__ T, uint32_t n)
{
    for (uint32_t k = blockIdx.x * 256 + threadIdx.x; k < n; k += gridDim.x * 256) T[k] = u[s[k]];
}

__global__ __launch_bounds__(256) void phase2(const float *__restrict__ T, const int *__restrict__ idx,
                                              float *__restrict__ p, uint32_t n)
{
    for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) p[i] = T[idx[i]];
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
    const uint32_t NB_LOG = argc > 1 ? uint32_t(atoi(argv[1])) : 22;   // bucket = 2^NB_LOG packed elems
    std::vector<int> d(N);
    uint64_t x = 0x5EED;
    for (uint32_t i = 0; i < N; ++i) { d[i] = int(x); x = (1664525ull * x + 1013904223ull) % RANGE; }
    // address order via the inverse map (d is a set of unique values)
    std::vector<int> inv(RANGE, -1);
    for (uint32_t i = 0; i < N; ++i) inv[uint32_t(d[i])] = int(i);
    std::vector<int> s, pidx;
    s.reserve(N); pidx.reserve(N);
    for (uint32_t v = 0; v < RANGE; ++v) if (inv[v] >= 0) { s.push_back(int(v)); pidx.push_back(inv[v]); }
    std::vector<int>().swap(inv);
    // bucket-major slots: bucket b = packed index >> NB_LOG; inside a bucket, address order
    const uint32_t NBK = N >> NB_LOG;
    std::vector<uint32_t> fill(NBK, 0);
    std::vector<int> slot(N), idx(N);
    for (uint32_t k = 0; k < N; ++k) {
        uint32_t b = uint32_t(pidx[k]) >> NB_LOG;
        uint32_t sl = (b << NB_LOG) + fill[b]++;
        slot[k] = int(sl);
        idx[uint32_t(pidx[k])] = int(sl);
    }
    float *u, *p, *T; int *dd, *ds, *dslot, *didx;
    CHK(hipMalloc(&u, size_t(RANGE) * 4)); CHK(hipMalloc(&p, size_t(N) * 4)); CHK(hipMalloc(&T, size_t(N) * 4));
    CHK(hipMalloc(&dd, size_t(N) * 4)); CHK(hipMalloc(&ds, size_t(N) * 4));
    CHK(hipMalloc(&dslot, size_t(N) * 4)); CHK(hipMalloc(&didx, size_t(N) * 4));
    CHK(hipMemcpy(dd, d.data(), size_t(N) * 4, hipMemcpyHostToDevice));
    CHK(hipMemcpy(ds, s.data(), size_t(N) * 4, hipMemcpyHostToDevice));
    CHK(hipMemcpy(dslot, slot.data(), size_t(N) * 4, hipMemcpyHostToDevice));
    CHK(hipMemcpy(didx, idx.data(), size_t(N) * 4, hipMemcpyHostToDevice));
    {
        std::vector<float> h(RANGE);
        for (uint32_t i = 0; i < RANGE; ++i) h[i] = float(i);
        CHK(hipMemcpy(u, h.data(), size_t(RANGE) * 4, hipMemcpyHostToDevice));
    }
    const dim3 grid(4096), blk(256);
    float t0 = timeit([&] { hipLaunchKernelGGL(direct, grid, blk, 0, 0, u, dd, p, N); }, 5);
    std::vector<float> ref(N), got(N);
    CHK(hipMemcpy(ref.data(), p, size_t(N) * 4, hipMemcpyDeviceToHost));
    float t1 = timeit([&] { hipLaunchKernelGGL(phase1, grid, blk, 0, 0, u, ds, dslot, T, N); }, 5);
    float t1s = timeit([&] { hipLaunchKernelGGL(phase1_sorted_only, grid, blk, 0, 0, u, ds, T, N); }, 5);
    hipLaunchKernelGGL(phase1, grid, blk, 0, 0, u, ds, dslot, T, N);
    float t2 = timeit([&] { hipLaunchKernelGGL(phase2, grid, blk, 0, 0, T, didx, p, N); }, 5);
    float t12 = timeit([&] {
        hipLaunchKernelGGL(phase1, grid, blk, 0, 0, u, ds, dslot, T, N);
        hipLaunchKernelGGL(phase2, grid, blk, 0, 0, T, didx, p, N);
    }, 5);
    CHK(hipMemcpy(got.data(), p, size_t(N) * 4, hipMemcpyDeviceToHost));
    size_t bad = 0;
    for (uint32_t i = 0; i < N; ++i) bad += ref[i] != got[i];
    printf("bucket 2^%u elems (%u buckets): direct %.1f us | phase1 %.1f us (sorted-only %.1f) | phase2 %.1f us | 1+2 %.1f us | mismatches %zu\n",
           NB_LOG, NBK, t0, t1, t1s, t2, t12, bad);
    return 0;
}
