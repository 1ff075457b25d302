// hostcost.cpp -- the engine's host cost per call from C (no Python): what a PML or the opal
// bridge pays per pack / unpack of a small message, next to a bare kernel launch and a
// hipMemcpyAsync of the same bytes.  Per operation: host microseconds to enqueue (the calls
// return without waiting: asynchronous convertors on one stream) and device microseconds per
// operation (one event pair around the whole loop).  Not part of the product.
//
//   ./scripts/hostcost [iters]     (built by: hipcc --offload-arch=gfx950 -O2 -Iinclude
//                                   scripts/hostcost.cpp -Lompi_amd -lddt_hip -Wl,-rpath,...)
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <sys/uio.h>

#include "ddt_hip.h"

#define CHK(x)                                                                          \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);       \
            std::exit(1);                                                               \
        }                                                                               \
    } while (0)
#define DCHK(x)                                                                         \
    do {                                                                                \
        int r_ = (x);                                                                   \
        if (r_ < 0) {                                                                   \
            std::printf("ddt error %d (%s) at %d\n", r_, ddt_last_error(), __LINE__);   \
            std::exit(1);                                                               \
        }                                                                               \
    } while (0)

__global__ void empty_kernel() {}
// the move kernel's argument shape (items pointer, count, two bases, task count: 36 bytes)
__global__ void empty_kernel_args(const void *p, uint32_t n, uint64_t a, uint64_t b, uint32_t t)
{
    if (n == 0xFFFFFFFFu && t == 7u)
        *reinterpret_cast<uint64_t *>(const_cast<void *>(p)) = a + b;
}

// a 512 KiB copy with its pointers in kernel arguments, and the same with the pointers in a
// device-global record (no kernel arguments at all: no gridDim / blockDim, which would add
// hidden arguments): 32 workgroups x 256 threads x 4 x 16 B
typedef unsigned int u32x4v __attribute__((ext_vector_type(4)));
struct SlotRec { const u32x4v *src; u32x4v *dst; };
__device__ SlotRec g_slot[4];
__global__ __launch_bounds__(256) void copy_args(const u32x4v *__restrict__ src, u32x4v *__restrict__ dst)
{
    const uint32_t t = blockIdx.x * 1024 + threadIdx.x;
    u32x4v v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k)
        v[k] = src[t + k * 256];
#pragma unroll
    for (int k = 0; k < 4; ++k)
        dst[t + k * 256] = v[k];
}
template <int K>
__global__ __launch_bounds__(256) void copy_slot()
{
    const SlotRec r = g_slot[K];
    const uint32_t t = blockIdx.x * 1024 + threadIdx.x;
    u32x4v v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k)
        v[k] = r.src[t + k * 256];
#pragma unroll
    for (int k = 0; k < 4; ++k)
        r.dst[t + k * 256] = v[k];
}

using clk = std::chrono::steady_clock;

struct Res { double host_us, dev_us; };

template <typename F>
Res run(hipStream_t s, int iters, F op)
{
    for (int i = 0; i < 20; ++i)
        op();
    CHK(hipStreamSynchronize(s));
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    CHK(hipEventRecord(a, s));
    const auto t0 = clk::now();
    for (int i = 0; i < iters; ++i)
        op();
    const auto t1 = clk::now();
    CHK(hipEventRecord(b, s));
    CHK(hipEventSynchronize(b));
    float ms = 0;
    CHK(hipEventElapsedTime(&ms, a, b));
    CHK(hipEventDestroy(a));
    CHK(hipEventDestroy(b));
    return {std::chrono::duration<double, std::micro>(t1 - t0).count() / iters, ms * 1e3 / iters};
}

int main(int argc, char **argv)
{
    const int iters = argc > 1 ? std::atoi(argv[1]) : 2000;
    const size_t n = 256, e = 8, field = n * n * n * e;
    uint8_t *user = nullptr, *packed = nullptr, *copy = nullptr;
    CHK(hipMalloc(&user, field));
    CHK(hipMalloc(&packed, 1 << 20));
    CHK(hipMalloc(&copy, 1 << 20));
    CHK(hipMemset(user, 1, field));
    hipStream_t s;
    CHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    const ddt_datatype_t *dbl = ddt_predefined(16);
    // the halo's faces of one 256^3 double field (bench.face_recipes)
    ddt_datatype_t *xf = nullptr, *yf = nullptr, *zf = nullptr;
    DCHK(ddt_type_create_vector(n * n, 1, ptrdiff_t(n), dbl, &xf));
    DCHK(ddt_type_create_vector(n, n, ptrdiff_t(n * n), dbl, &yf));
    DCHK(ddt_type_create_contiguous(n * n, dbl, &zf));
    for (ddt_datatype_t *t : {xf, yf, zf})
        DCHK(ddt_type_commit(t));
    ddt_convertor_t *cv = ddt_convertor_create();
    DCHK(ddt_convertor_set_stream(cv, s, 1));

    const size_t face = n * n * e;   // 512 KiB packed per face
    std::printf("{\"what\": \"empty kernel\", \"bytes\": 0, ");
    Res r = run(s, iters, [&] { hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s); });
    std::printf("\"host_us\": %.3f, \"device_us\": %.3f}\n", r.host_us, r.dev_us);
    std::printf("{\"what\": \"empty kernel, 36 B of arguments\", \"bytes\": 0, ");
    r = run(s, iters, [&] { hipLaunchKernelGGL(empty_kernel_args, dim3(1), dim3(64), 0, s, (const void *) packed, 1u, 2ull, 3ull, 4u); });
    std::printf("\"host_us\": %.3f, \"device_us\": %.3f}\n", r.host_us, r.dev_us);
    std::printf("{\"what\": \"empty kernel, 36 B of arguments, 32 x 256 threads\", \"bytes\": 0, ");
    r = run(s, iters, [&] { hipLaunchKernelGGL(empty_kernel_args, dim3(32), dim3(256), 0, s, (const void *) packed, 1u, 2ull, 3ull, 4u); });
    std::printf("\"host_us\": %.3f, \"device_us\": %.3f}\n", r.host_us, r.dev_us);
    std::printf("{\"what\": \"512 KiB copy kernel, pointers in arguments\", \"bytes\": %zu, ", face);
    r = run(s, iters, [&] { hipLaunchKernelGGL(copy_args, dim3(32), dim3(256), 0, s, (const u32x4v *) packed, (u32x4v *) copy); });
    std::printf("\"host_us\": %.3f, \"device_us\": %.3f}\n", r.host_us, r.dev_us);
    {
        SlotRec h{(const u32x4v *) packed, (u32x4v *) copy};
        CHK(hipMemcpyToSymbol(HIP_SYMBOL(g_slot), &h, sizeof(h)));
    }
    std::printf("{\"what\": \"512 KiB copy kernel, pointers in a device record (no arguments)\", \"bytes\": %zu, ", face);
    r = run(s, iters, [&] { hipLaunchKernelGGL(copy_slot<0>, dim3(32), dim3(256), 0, s); });
    std::printf("\"host_us\": %.3f, \"device_us\": %.3f}\n", r.host_us, r.dev_us);
    std::printf("{\"what\": \"hipMemcpyAsync D2D\", \"bytes\": %zu, ", face);
    r = run(s, iters, [&] { CHK(hipMemcpyAsync(copy, packed, face, hipMemcpyDeviceToDevice, s)); });
    std::printf("\"host_us\": %.3f, \"device_us\": %.3f}\n", r.host_us, r.dev_us);

    // the runtime calls a pack makes besides its launch
    {
        hipPointerAttribute_t a;
        r = run(s, iters, [&] { (void) hipPointerGetAttributes(&a, packed); });
        std::printf("{\"what\": \"hipPointerGetAttributes\", \"host_us\": %.3f}\n", r.host_us);
        hipStreamCaptureStatus cs;
        r = run(s, iters, [&] { (void) hipStreamIsCapturing(s, &cs); });
        std::printf("{\"what\": \"hipStreamIsCapturing\", \"host_us\": %.3f}\n", r.host_us);
        int d;
        r = run(s, iters, [&] { (void) hipGetDevice(&d); });
        std::printf("{\"what\": \"hipGetDevice\", \"host_us\": %.3f}\n", r.host_us);
    }
    const char *names[3] = {"x", "y", "z"};
    ddt_datatype_t *faces[3] = {xf, yf, zf};
    for (int f = 0; f < 3; ++f) {
        for (int dir = 0; dir < 2; ++dir) {
            auto op = [&] {
                struct iovec iov = {packed, face};
                uint32_t cnt = 1;
                size_t md = face;
                if (dir == 0) {
                    DCHK(ddt_convertor_prepare_for_send(cv, faces[f], 1, user));
                    DCHK(ddt_convertor_pack(cv, &iov, &cnt, &md));
                } else {
                    DCHK(ddt_convertor_prepare_for_recv(cv, faces[f], 1, user));
                    DCHK(ddt_convertor_unpack(cv, &iov, &cnt, &md));
                }
            };
            r = run(s, iters, op);
            std::printf("{\"what\": \"engine %s %s face, 1 field\", \"bytes\": %zu, \"host_us\": %.3f, "
                        "\"device_us\": %.3f}\n", dir ? "unpack" : "pack", names[f], face, r.host_us, r.dev_us);
        }
        // the prepare alone (a PML prepares once per message, then packs fragments)
        r = run(s, iters, [&] { DCHK(ddt_convertor_prepare_for_send(cv, faces[f], 1, user)); });
        std::printf("{\"what\": \"engine prepare_for_send %s face\", \"bytes\": 0, \"host_us\": %.3f}\n",
                    names[f], r.host_us);
    }
    // synchronous calls (MPI_Pack semantics: the data is in place on return): an empty kernel
    // then a wait, by hipStreamSynchronize, by hipEventSynchronize, by polling hipEventQuery;
    // then the engine's own synchronous MPI_Pack of the y face
    {
        hipEvent_t ev;
        CHK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        auto wall = [&](auto op) {
            for (int i = 0; i < 20; ++i)
                op();
            const auto t0 = clk::now();
            for (int i = 0; i < iters; ++i)
                op();
            return std::chrono::duration<double, std::micro>(clk::now() - t0).count() / iters;
        };
        double w = wall([&] {
            hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s);
            CHK(hipStreamSynchronize(s));
        });
        std::printf("{\"what\": \"empty kernel + hipStreamSynchronize\", \"call_us\": %.3f}\n", w);
        w = wall([&] {
            hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s);
            CHK(hipEventRecord(ev, s));
            CHK(hipEventSynchronize(ev));
        });
        std::printf("{\"what\": \"empty kernel + event record + hipEventSynchronize\", \"call_us\": %.3f}\n", w);
        w = wall([&] {
            hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s);
            CHK(hipEventRecord(ev, s));
            while (hipEventQuery(ev) == hipErrorNotReady) {
            }
        });
        std::printf("{\"what\": \"empty kernel + event record + hipEventQuery poll\", \"call_us\": %.3f}\n", w);
        for (int f = 0; f < 3; ++f) {
            size_t pos = 0;
            w = wall([&] {
                pos = 0;
                DCHK(ddt_pack(user, 1, faces[f], packed, face, &pos));
            });
            std::printf("{\"what\": \"engine MPI_Pack (synchronous) %s face\", \"bytes\": %zu, \"call_us\": %.3f}\n",
                        names[f], face, w);
        }
        CHK(hipEventDestroy(ev));
    }
    // the same with descriptors always in the kernel arguments (ddt_tune "ptr" 0)
    ddt_tune("ptr", 0);
    for (int f = 1; f < 2; ++f) {
        r = run(s, iters, [&] {
            struct iovec iov = {packed, face};
            uint32_t cnt = 1;
            size_t md = face;
            DCHK(ddt_convertor_prepare_for_send(cv, faces[f], 1, user));
            DCHK(ddt_convertor_pack(cv, &iov, &cnt, &md));
        });
        std::printf("{\"what\": \"engine pack %s face, inline descriptors\", \"host_us\": %.3f, \"device_us\": %.3f}\n",
                    names[f], r.host_us, r.dev_us);
    }
    ddt_tune("ptr", 1);
    ddt_convertor_destroy(cv);
    for (ddt_datatype_t *t : {xf, yf, zf})
        ddt_type_destroy(&t);
    return 0;
}
