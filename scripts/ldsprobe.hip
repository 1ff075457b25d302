// ldsprobe.hip -- where can an argument-free kernel find which launch record it serves?
//   1. the hardware register HW_REG_LDS_ALLOC (s_getreg: no memory access) for dynamic LDS sizes
//      0 .. 16 KiB: the raw value each size gives, so a launch can carry a small index in its LDS size;
//   2. device time per back-to-back launch (256 workgroups, 2000 launches between one event pair)
//      of an empty kernel, one that reads its dispatch packet (the packet lives in the host-memory
//      AQL queue), one that reads HW_REG_LDS_ALLOC, and one launched with 4 KiB of dynamic LDS.
// Not part of the library.
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>

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

// HW_REG_LDS_ALLOC = hardware register 6; the whole 32 bits (size field 31 = 32 bits - 1)
constexpr int kLdsAlloc = (31 << 11) | (0 << 6) | 6;

__global__ void k_reg(uint32_t *out)
{
    if (threadIdx.x == 0 && blockIdx.x == 0)
        out[0] = __builtin_amdgcn_s_getreg(kLdsAlloc);
}

__global__ void k_empty() {}

__device__ uint32_t g_sink;

__global__ void k_packet()
{
    using CPacket = const __attribute__((address_space(4))) hsa_kernel_dispatch_packet_t;
    CPacket *pk = (CPacket *) __builtin_amdgcn_dispatch_ptr();
    if (pk->group_segment_size == 12345u && threadIdx.x == 0)
        g_sink = 1;
}

__global__ void k_getreg()
{
    if (__builtin_amdgcn_s_getreg(kLdsAlloc) == 12345u && threadIdx.x == 0)
        g_sink = 1;
}

int main()
{
    uint32_t *d;
    CHK(hipMalloc(&d, 4));
    for (uint32_t lds = 0; lds <= 16384; lds += 128) {
        CHK(hipMemset(d, 0xFF, 4));
        hipLaunchKernelGGL(k_reg, dim3(1), dim3(64), lds, nullptr, d);
        uint32_t h = 0;
        CHK(hipMemcpy(&h, d, 4, hipMemcpyDeviceToHost));
        std::printf("{\"dyn_lds\": %u, \"lds_alloc_reg\": %u, \"hex\": \"0x%08x\"}\n", lds, h, h);
    }
    hipStream_t s;
    CHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    const int n = 2000;
    auto timeit = [&](const char *what, auto launch) {
        for (int i = 0; i < 50; ++i)
            launch();
        CHK(hipStreamSynchronize(s));
        CHK(hipEventRecord(a, s));
        for (int i = 0; i < n; ++i)
            launch();
        CHK(hipEventRecord(b, s));
        CHK(hipStreamSynchronize(s));
        float ms = 0;
        CHK(hipEventElapsedTime(&ms, a, b));
        std::printf("{\"what\": \"%s\", \"device_us_per_launch\": %.3f}\n", what, ms * 1e3 / n);
    };
    const dim3 g(256), blk(256);
    timeit("empty kernel, 256 workgroups", [&] { hipLaunchKernelGGL(k_empty, g, blk, 0, s); });
    timeit("reads its dispatch packet, 256 workgroups", [&] { hipLaunchKernelGGL(k_packet, g, blk, 0, s); });
    timeit("reads HW_REG_LDS_ALLOC, 256 workgroups", [&] { hipLaunchKernelGGL(k_getreg, g, blk, 0, s); });
    timeit("reads HW_REG_LDS_ALLOC, 4 KiB dynamic LDS, 256 workgroups",
           [&] { hipLaunchKernelGGL(k_getreg, g, blk, 4096, s); });
    timeit("empty kernel, 4 KiB dynamic LDS, 256 workgroups", [&] { hipLaunchKernelGGL(k_empty, g, blk, 4096, s); });
    return 0;
}
