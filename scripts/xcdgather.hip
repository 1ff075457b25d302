// xcdgather.hip -- can an index-list gather run out of the XCD L2s?  Round 5 question for cfg4
// (64 Mi unique random 4-byte elements of a 1 GiB buffer): the address-ordered engine moves every
// element twice (pass 1 into address-ordered runs, pass 2 through an LDS permutation).  If the
// elements of each small address RANGE are gathered by workgroups of ONE XCD while that range
// sits in its L2, the source lines come from HBM once and every further element of the line is an
// L2 hit: one pass in the packed order per range.  This measures the rate of that gather (and of
// the mirror scatter) against range size and XCD placement.  Not part of the product.
//
// Elements: one random 4-byte slot of every 16 bytes (64 Mi, unique), grouped by range (RB bytes
// of source: RB / 16 elements), shuffled inside the range (the packed order is random).  A
// range's elements are contiguous in the list; out / in is the list-ordered stream.
//   xcd    range r on XCD r % 8 (blockIdx b: XCD b % 8, the b / 8-th chunk of that XCD's ranges)
//   flat   chunk b of the list on block b (every XCD works in every range at once)
//   random the list fully shuffled (no ranges: the direct gather)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <random>
#include <vector>

#define CHK(x)                                                                          \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);       \
            std::exit(1);                                                               \
        }                                                                               \
    } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr uint32_t NT = 256, PER = 8, CHUNK = NT * PER;
constexpr size_t SRC = size_t(1) << 30, NE = SRC / 16;

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

// list position of the block's chunk: XCD mode keeps each XCD on its own ranges
template <bool XCD>
__device__ __forceinline__ size_t chunk_base(uint32_t b, uint32_t per_range)
{
    if (!XCD)
        return size_t(b) * CHUNK;
    const uint32_t x = b & 7u, w = b >> 3;
    const size_t j = size_t(w) * CHUNK;              // position in XCD x's sequence of ranges
    const size_t k = j / per_range;                  // its k-th range: range x + 8k
    return (size_t(x) + 8 * k) * per_range + j % per_range;
}

template <bool XCD>
__global__ __launch_bounds__(NT) void gather(const float *__restrict__ src, const uint32_t *__restrict__ list,
                                             float *__restrict__ out, uint32_t per_range)
{
    const size_t base = chunk_base<XCD>(blockIdx.x, per_range) + threadIdx.x;
    uint32_t a[PER];
    float v[PER];
#pragma unroll
    for (int q = 0; q < PER; ++q)
        a[q] = __builtin_nontemporal_load(list + base + q * NT);
#pragma unroll
    for (int q = 0; q < PER; ++q)
        v[q] = src[a[q]];
#pragma unroll
    for (int q = 0; q < PER; ++q)
        __builtin_nontemporal_store(v[q], out + base + q * NT);
}

template <bool XCD>
__global__ __launch_bounds__(NT) void scatter(float *__restrict__ dst, const uint32_t *__restrict__ list,
                                              const float *__restrict__ in, uint32_t per_range)
{
    const size_t base = chunk_base<XCD>(blockIdx.x, per_range) + threadIdx.x;
    uint32_t a[PER];
    float v[PER];
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        a[q] = __builtin_nontemporal_load(list + base + q * NT);
        v[q] = __builtin_nontemporal_load(in + base + q * NT);
    }
#pragma unroll
    for (int q = 0; q < PER; ++q)
        dst[a[q]] = v[q];
}

int main(int argc, char **argv)
{
    const int reps = argc > 1 ? std::atoi(argv[1]) : 3;
    float *src = nullptr, *stream = nullptr;
    uint32_t *list = nullptr, *sink = nullptr;
    u32x4 *fl = nullptr;
    const size_t nflush = (size_t(1) << 30) / 16;
    CHK(hipMalloc(&src, SRC));
    CHK(hipMalloc(&stream, NE * 4));
    CHK(hipMalloc(&list, NE * 4));
    CHK(hipMalloc(&fl, nflush * 16));
    CHK(hipMalloc(&sink, 1024));
    CHK(hipMemset(src, 1, SRC));
    CHK(hipMemset(stream, 3, NE * 4));
    CHK(hipMemset(fl, 2, nflush * 16));
    std::mt19937_64 rng(12345);
    std::vector<uint32_t> h(NE);
    for (size_t i = 0; i < NE; ++i)
        h[i] = uint32_t(i * 4 + (rng() & 3));   // one 4-byte slot of every 16 bytes, address order
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    auto time = [&](auto launch) {
        std::vector<float> t;
        for (int r = 0; r < reps; ++r) {
            hipLaunchKernelGGL(flush, dim3(4096), dim3(256), 0, nullptr, fl, nflush, sink);
            CHK(hipEventRecord(e0, nullptr));
            launch();
            CHK(hipEventRecord(e1, nullptr));
            CHK(hipEventSynchronize(e1));
            float ms = 0;
            CHK(hipEventElapsedTime(&ms, e0, e1));
            t.push_back(ms * 1e3f);
        }
        std::sort(t.begin(), t.end());
        return t[t.size() / 2];
    };
    const dim3 grid(uint32_t(NE / CHUNK)), blk(NT);
    for (uint32_t rb_kib : {512u, 1024u, 2048u, 4096u, 0u}) {
        // rb_kib 0: fully random order
        std::vector<uint32_t> l = h;
        uint32_t per_range = 0;
        if (rb_kib) {
            per_range = rb_kib * 1024 / 16;
            for (size_t r = 0; r < NE / per_range; ++r)
                std::shuffle(l.begin() + r * per_range, l.begin() + (r + 1) * per_range, rng);
        } else {
            std::shuffle(l.begin(), l.end(), rng);
        }
        CHK(hipMemcpy(list, l.data(), NE * 4, hipMemcpyHostToDevice));
        const uint32_t pr = per_range ? per_range : uint32_t(CHUNK);
        const float gx = time([&] { hipLaunchKernelGGL(gather<true>, grid, blk, 0, nullptr, src, list, stream, pr); });
        const float gf = time([&] { hipLaunchKernelGGL(gather<false>, grid, blk, 0, nullptr, src, list, stream, pr); });
        const float sx = time([&] { hipLaunchKernelGGL(scatter<true>, grid, blk, 0, nullptr, src, list, stream, pr); });
        const float sf = time([&] { hipLaunchKernelGGL(scatter<false>, grid, blk, 0, nullptr, src, list, stream, pr); });
        std::printf("{\"range_kib\": %u, \"elements\": %zu, \"gather_xcd_us\": %.1f, \"gather_flat_us\": %.1f, "
                    "\"scatter_xcd_us\": %.1f, \"scatter_flat_us\": %.1f}\n",
                    rb_kib, NE, gx, gf, sx, sf);
        std::fflush(stdout);
    }
    return 0;
}
