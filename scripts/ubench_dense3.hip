// ubench_dense3.hip -- round 3: why the engine's line-dense pack (one task = a few 4 KiB
// chunks, 1183-1197 us on BASELINE config 5) trails the bare one-chunk-per-workgroup kernel
// (1082 us, scripts/ubench_dense2.hip).  Shapes of config 5: 128 Mi records of 20 bytes at a
// 32-byte stride (4 GiB user span, 2.5 GiB packed).  Not part of the product.
//   B   one 4 KiB chunk (128 records) per workgroup, 1 Mi workgroups (ubench_dense2's best)
//   P   persistent: G workgroups, workgroup b takes chunks b, b + G, b + 2G, ... (at any time
//       the grid works on a contiguous window of G chunks), single buffer
//   Q   P with the next chunk's loads in flight while the current one is written out
//   T   contiguous runs: workgroup b takes chunks [b*n, (b+1)*n) with Q's prefetch (the engine's
//       multi-chunk task)
// Every variant is checked against B's packed bytes.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CHK(x)                                                                          \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);            \
            exit(1);                                                                    \
        }                                                                               \
    } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr uint64_t NREC = 128ull << 20;
constexpr uint32_t REC = 20, STRIDE = 32, WPR = REC / 4, R = 128;
constexpr uint32_t NCH = uint32_t(NREC / R);            // 1 Mi chunks
constexpr uint32_t NO = R * REC / 16;                    // 160 packed vectors per chunk

__device__ __forceinline__ void emit(const uint32_t *lds, u32x4 *dst)
{
    for (uint32_t c = threadIdx.x; c < NO; c += 256) {
        uint32_t d[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint32_t q = 4 * c + uint32_t(i), r = q / WPR, w = q - r * WPR;
            d[i] = lds[r * (STRIDE / 4) + w];
        }
        dst[c] = u32x4{d[0], d[1], d[2], d[3]};
    }
}

__global__ __launch_bounds__(256) void pack_b(const u32x4 *__restrict__ user, u32x4 *__restrict__ packed)
{
    __shared__ u32x4 buf[256];
    const uint64_t ch = blockIdx.x;
    buf[threadIdx.x] = __builtin_nontemporal_load(user + ch * 256 + threadIdx.x);
    __syncthreads();
    emit(reinterpret_cast<const uint32_t *>(buf), packed + ch * NO);
}

template <bool PREFETCH, bool NT>
__global__ __launch_bounds__(256) void pack_p(const u32x4 *__restrict__ user, u32x4 *__restrict__ packed)
{
    __shared__ u32x4 buf[256];
    uint32_t ch = blockIdx.x;
    u32x4 v = NT ? __builtin_nontemporal_load(user + uint64_t(ch) * 256 + threadIdx.x) : user[uint64_t(ch) * 256 + threadIdx.x];
    for (; ch < NCH; ch += gridDim.x) {
        if (!PREFETCH && ch != blockIdx.x)
            v = NT ? __builtin_nontemporal_load(user + uint64_t(ch) * 256 + threadIdx.x) : user[uint64_t(ch) * 256 + threadIdx.x];
        __syncthreads();
        buf[threadIdx.x] = v;
        __syncthreads();
        const uint32_t nx = ch + gridDim.x;
        if (PREFETCH && nx < NCH)
            v = NT ? __builtin_nontemporal_load(user + uint64_t(nx) * 256 + threadIdx.x) : user[uint64_t(nx) * 256 + threadIdx.x];
        emit(reinterpret_cast<const uint32_t *>(buf), packed + uint64_t(ch) * NO);
    }
}

// two chunks in flight per workgroup (loads of ch + G and ch + 2G while ch is written)
__global__ __launch_bounds__(256) void pack_p2(const u32x4 *__restrict__ user, u32x4 *__restrict__ packed)
{
    __shared__ u32x4 buf[256];
    const uint32_t G = gridDim.x;
    uint32_t ch = blockIdx.x;
    u32x4 v0 = __builtin_nontemporal_load(user + uint64_t(ch) * 256 + threadIdx.x);
    u32x4 v1 = ch + G < NCH ? __builtin_nontemporal_load(user + uint64_t(ch + G) * 256 + threadIdx.x) : v0;
    for (; ch < NCH; ch += G) {
        __syncthreads();
        buf[threadIdx.x] = v0;
        __syncthreads();
        v0 = v1;
        if (ch + 2 * G < NCH)
            v1 = __builtin_nontemporal_load(user + uint64_t(ch + 2 * G) * 256 + threadIdx.x);
        emit(reinterpret_cast<const uint32_t *>(buf), packed + uint64_t(ch) * NO);
    }
}

__global__ __launch_bounds__(256) void pack_t(const u32x4 *__restrict__ user, u32x4 *__restrict__ packed, uint32_t n)
{
    __shared__ u32x4 buf[256];
    uint32_t ch = blockIdx.x * n;
    const uint32_t end = ch + n;
    u32x4 v = __builtin_nontemporal_load(user + uint64_t(ch) * 256 + threadIdx.x);
    for (; ch < end; ++ch) {
        __syncthreads();
        buf[threadIdx.x] = v;
        __syncthreads();
        if (ch + 1 < end)
            v = __builtin_nontemporal_load(user + uint64_t(ch + 1) * 256 + threadIdx.x);
        emit(reinterpret_cast<const uint32_t *>(buf), packed + uint64_t(ch) * NO);
    }
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
    int ncu = 0;
    CHK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    const uint64_t ubytes = NREC * STRIDE, pbytes = NREC * REC;
    void *u, *p, *ref;
    CHK(hipMalloc(&u, ubytes));
    CHK(hipMalloc(&p, pbytes));
    CHK(hipMalloc(&ref, pbytes));
    {
        std::vector<uint32_t> h(ubytes / 4);
        uint32_t x = 12345;
        for (auto &w : h) { x = x * 1664525u + 1013904223u; w = x; }
        CHK(hipMemcpy(u, h.data(), ubytes, hipMemcpyHostToDevice));
    }
    const u32x4 *uu = (const u32x4 *) u;
    u32x4 *pp = (u32x4 *) p;
    hipLaunchKernelGGL(pack_b, dim3(NCH), dim3(256), 0, 0, uu, (u32x4 *) ref);
    CHK(hipDeviceSynchronize());
    std::vector<char> hr(pbytes), hp(pbytes);
    CHK(hipMemcpy(hr.data(), ref, pbytes, hipMemcpyDeviceToHost));
    auto check = [&](const char *nm) {
        CHK(hipDeviceSynchronize());
        CHK(hipMemcpy(hp.data(), p, pbytes, hipMemcpyDeviceToHost));
        if (memcmp(hp.data(), hr.data(), pbytes) != 0) printf("  MISMATCH in %s\n", nm);
        CHK(hipMemset(p, 0, pbytes));
    };
    auto gbs = [&](float us) { return (ubytes + pbytes) / (us * 1e3); };
    printf("config-5 pack, %d CUs, %u chunks of %u records (4 KiB), %d iterations per figure\n", ncu, NCH, R, iters);
    for (int round = 0; round < 2; ++round) {
        float t = timeit([&] { hipLaunchKernelGGL(pack_b, dim3(NCH), dim3(256), 0, 0, uu, pp); }, iters);
        printf("B  one chunk per workgroup              : %7.1f us (%4.0f GB/s)\n", t, gbs(t));
        for (int per : {4, 8, 16}) {
            const uint32_t G = uint32_t(ncu * per);
            t = timeit([&] { hipLaunchKernelGGL((pack_p<false, true>), dim3(G), dim3(256), 0, 0, uu, pp); }, iters);
            if (!round) check("P");
            printf("P  persistent G=%5u, single buffer    : %7.1f us (%4.0f GB/s)\n", G, t, gbs(t));
            t = timeit([&] { hipLaunchKernelGGL((pack_p<true, true>), dim3(G), dim3(256), 0, 0, uu, pp); }, iters);
            if (!round) check("Q");
            printf("Q  persistent G=%5u, prefetch 1       : %7.1f us (%4.0f GB/s)\n", G, t, gbs(t));
            t = timeit([&] { hipLaunchKernelGGL((pack_p<true, false>), dim3(G), dim3(256), 0, 0, uu, pp); }, iters);
            if (!round) check("Qt");
            printf("Qt persistent G=%5u, prefetch, plain ld: %7.1f us (%4.0f GB/s)\n", G, t, gbs(t));
            t = timeit([&] { hipLaunchKernelGGL(pack_p2, dim3(G), dim3(256), 0, 0, uu, pp); }, iters);
            if (!round) check("Q2");
            printf("Q2 persistent G=%5u, prefetch 2       : %7.1f us (%4.0f GB/s)\n", G, t, gbs(t));
        }
        for (uint32_t n : {2u, 8u}) {
            t = timeit([&] { hipLaunchKernelGGL(pack_t, dim3(NCH / n), dim3(256), 0, 0, uu, pp, n); }, iters);
            if (!round) check("T");
            printf("T  %u contiguous chunks per workgroup    : %7.1f us (%4.0f GB/s)\n", n, t, gbs(t));
        }
    }
    return 0;
}
