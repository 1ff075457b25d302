// synccost.cpp -- how fast can the host learn that a small kernel finished?  HIP's own completion
// (hipStreamSynchronize: 9.5 us round trip for an empty kernel, profiles/r5_hostcost_sync.jsonl)
// against a flag the kernel itself stores to pinned host memory at its end (system scope) while
// the host spins on it.  Not part of the product: the question is whether a synchronous MPI_Pack
// could return earlier than the stream's completion signal.
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
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

__global__ void empty_kernel() {}

// one workgroup: after its work (none) thread 0 publishes `seq` to the host flag
__global__ void flag_kernel(volatile uint32_t *flag, uint32_t seq)
{
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence_system();
        __hip_atomic_store(const_cast<uint32_t *>(flag), seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

using clk = std::chrono::steady_clock;

int main(int argc, char **argv)
{
    const int iters = argc > 1 ? std::atoi(argv[1]) : 2000;
    hipStream_t s;
    CHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    uint32_t *flag = nullptr;
    CHK(hipHostMalloc(&flag, 64, hipHostMallocMapped | hipHostMallocCoherent));
    *flag = 0;
    auto wall = [&](auto op) {
        for (int i = 0; i < 20; ++i)
            op(i);
        const auto t0 = clk::now();
        for (int i = 0; i < iters; ++i)
            op(i + 20);
        return std::chrono::duration<double, std::micro>(clk::now() - t0).count() / iters;
    };
    double w = wall([&](int) {
        hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s);
        CHK(hipStreamSynchronize(s));
    });
    std::printf("{\"what\": \"empty kernel + hipStreamSynchronize\", \"call_us\": %.3f}\n", w);
    uint32_t seq = 0;
    w = wall([&](int) {
        ++seq;
        hipLaunchKernelGGL(flag_kernel, dim3(1), dim3(64), 0, s, (volatile uint32_t *) flag, seq);
        while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != seq) {
        }
    });
    std::printf("{\"what\": \"flag kernel + host spin on pinned flag\", \"call_us\": %.3f}\n", w);
    CHK(hipStreamSynchronize(s));
    w = wall([&](int) {
        ++seq;
        hipLaunchKernelGGL(flag_kernel, dim3(1), dim3(64), 0, s, (volatile uint32_t *) flag, seq);
        while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != seq) {
        }
        CHK(hipStreamSynchronize(s));
    });
    std::printf("{\"what\": \"flag kernel + spin + hipStreamSynchronize\", \"call_us\": %.3f}\n", w);
    CHK(hipHostFree(flag));
    return 0;
}
