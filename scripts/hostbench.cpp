// hostbench.cpp -- host-side cost of one convertor pack call through the C ABI (what a PML
// pays per fragment), measured without Python: prepare + pack of a small x-face window,
// asynchronous on one stream, so the loop measures enqueue cost only.  Also the
// synchronous MPI_Pack-style call (ddt_pack) end to end.
//   hipcc -O2 -I include scripts/hostbench.cpp -L ompi_amd -lddt_hip -o scripts/hostbench
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "ddt_hip.h"

#define CHK(x) do { int _r = (x); if (_r < 0) { printf("%s failed %d: %s\n", #x, _r, ddt_last_error()); exit(1); } } while (0)
#define HCHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s\n", hipGetErrorString(e)); exit(1); } } while (0)

__global__ void nullptr_kernel() {}
struct Arg528 { unsigned char b[528]; };
__global__ void arg_kernel(Arg528 a) { if (a.b[0] == 255 && threadIdx.x == 999) a.b[1] = 0; }

static double now_us()
{
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main()
{
    const int n = 64;   // 64^3 double field: x face = vector(4096, 1, 64)
    ddt_datatype_t *x = nullptr;
    CHK(ddt_type_create_vector(size_t(n) * n, 1, n, ddt_predefined(DDT_FLOAT8), &x));
    CHK(ddt_type_commit(x));
    size_t fs = 0;
    CHK(ddt_type_size(x, &fs));
    void *user = nullptr, *packed = nullptr;
    HCHK(hipMalloc(&user, size_t(n) * n * n * 8));
    HCHK(hipMalloc(&packed, fs));
    hipStream_t s;
    HCHK(hipStreamCreate(&s));
    ddt_convertor_t *c = ddt_convertor_create();
    CHK(ddt_convertor_set_stream(c, s, 1));
    const int iters = 2000;
    std::vector<double> t;
    for (int rep = 0; rep < 5; ++rep) {
        HCHK(hipStreamSynchronize(s));
        double t0 = now_us();
        for (int i = 0; i < iters; ++i) {
            CHK(ddt_convertor_prepare_for_send(c, x, 1, user));
            struct iovec iov{packed, fs};
            uint32_t cnt = 1;
            size_t md = 0;
            CHK(ddt_convertor_pack(c, &iov, &cnt, &md));
        }
        double t1 = now_us();
        HCHK(hipStreamSynchronize(s));
        double t2 = now_us();
        t.push_back((t1 - t0) / iters);
        if (rep == 4)
            printf("async enqueue: %.2f us/call (host), %.2f us/call incl. drain\n", (t1 - t0) / iters,
                   (t2 - t0) / iters);
    }
    std::sort(t.begin(), t.end());
    printf("async enqueue median %.2f us/call\n", t[t.size() / 2]);
    for (long ptr : {0L, 1L}) {   // reused descriptor set: kernel-argument block vs pointer
        CHK(ddt_tune("ptr", ptr));
        CHK(ddt_convertor_prepare_for_send(c, x, 1, user));
        HCHK(hipStreamSynchronize(s));
        std::vector<double> r;
        for (int rep = 0; rep < 5; ++rep) {
            double t0 = now_us();
            for (int i = 0; i < iters; ++i) {
                size_t pos = 0;
                CHK(ddt_convertor_set_position(c, &pos));
                struct iovec iov{packed, fs};
                uint32_t cnt = 1;
                size_t md = 0;
                CHK(ddt_convertor_pack(c, &iov, &cnt, &md));
            }
            r.push_back((now_us() - t0) / iters);
            HCHK(hipStreamSynchronize(s));
        }
        std::sort(r.begin(), r.end());
        printf("repeated pack, descriptors %s: median %.2f us/call (host)\n",
               ptr ? "by pointer" : "as kernel arguments", r[r.size() / 2]);
    }
    {   // the same pack with the convertor prepared once (set_position(0) per call)
        CHK(ddt_convertor_prepare_for_send(c, x, 1, user));
        HCHK(hipStreamSynchronize(s));
        double t0 = now_us();
        for (int i = 0; i < iters; ++i) {
            size_t pos = 0;
            CHK(ddt_convertor_set_position(c, &pos));
            struct iovec iov{packed, fs};
            uint32_t cnt = 1;
            size_t md = 0;
            CHK(ddt_convertor_pack(c, &iov, &cnt, &md));
        }
        double t1 = now_us();
        HCHK(hipStreamSynchronize(s));
        printf("async pack without prepare: %.2f us/call (host)\n", (t1 - t0) / iters);
        t0 = now_us();
        for (int i = 0; i < iters; ++i)
            CHK(ddt_convertor_prepare_for_send(c, x, 1, user));
        printf("prepare_for_send alone: %.3f us/call\n", (now_us() - t0) / iters);
    }
    std::vector<double> w;
    for (int i = 0; i < 500; ++i) {
        size_t pos = 0;
        double t0 = now_us();
        CHK(ddt_pack(user, 1, x, packed, fs, &pos));
        w.push_back(now_us() - t0);
    }
    std::sort(w.begin(), w.end());
    printf("synchronous ddt_pack (MPI_Pack) of %zu bytes: median %.2f us, p10 %.2f us\n", fs,
           w[w.size() / 2], w[w.size() / 10]);
    {
        hipPointerAttribute_t a;
        const int m = 20000;
        double t0 = now_us();
        for (int i = 0; i < m; ++i)
            HCHK(hipPointerGetAttributes(&a, static_cast<char *>(user) + (i & 1023)));
        printf("hipPointerGetAttributes: %.3f us/call\n", (now_us() - t0) / m);
        t0 = now_us();
        for (int i = 0; i < m; ++i)
            hipLaunchKernelGGL(nullptr_kernel, dim3(1), dim3(64), 0, s);
        double t1 = now_us();
        HCHK(hipStreamSynchronize(s));
        printf("empty kernel launch: %.3f us/call (host enqueue), %.3f us incl. drain\n", (t1 - t0) / m,
               (now_us() - t0) / m);
        Arg528 arg{};
        t0 = now_us();
        for (int i = 0; i < m; ++i)
            hipLaunchKernelGGL(arg_kernel, dim3(32), dim3(256), 0, s, arg);
        t1 = now_us();
        HCHK(hipStreamSynchronize(s));
        printf("launch with a 528-byte argument: %.3f us/call (host enqueue)\n", (t1 - t0) / m);
    }
    ddt_convertor_destroy(c);
    ddt_type_destroy(&x);
    return 0;
}
