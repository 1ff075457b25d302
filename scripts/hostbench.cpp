// hostbench.cpp -- host-side cost of one convertor pack call through the C ABI (what a PML
// pays per fragment), measured without Python: prepare + pack of a small x-face window,
// asynchronous on one stream, so the loop measures enqueue cost only.  Also the
// synchronous MPI_Pack-style call (ddt_pack) end to end.
//   hipcc -O2 --offload-arch=gfx950 -I include scripts/hostbench.cpp -L ompi_amd -lddt_hip -Wl,-rpath,'$ORIGIN/../ompi_amd' \
//     -o scripts/hostbench
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "ddt_hip.h"
#include "opal_hip_bridge.h"

#define CHK(x) do { int _r = (x); if (_r < 0) { printf("%s failed %d: %s\n", #x, _r, ddt_last_error()); exit(1); } } while (0)
#define HCHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s\n", hipGetErrorString(e)); exit(1); } } while (0)

__global__ void nullptr_kernel() {}
struct Arg528 { unsigned char b[528]; };
// the move kernel's argument list (items, nitems, ubase, pbase, ntasks), empty body
__global__ __launch_bounds__(256) void args36_kernel(const void *items, uint32_t n, uint64_t u, uint64_t p,
                                                     uint32_t t)
{
    if (items == nullptr && n == 12345u && threadIdx.x == 999) ((uint64_t *) p)[u + t] = 0;
}
__global__ void arg_kernel(Arg528 a) { if (a.b[0] == 255 && threadIdx.x == 999) a.b[1] = 0; }

static double now_us()
{
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main()
{
    setvbuf(stdout, nullptr, _IOLBF, 0);
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
    {   // round 2: the bare HIP floor of a synchronous call -- one empty kernel and a blocking
        // wait (polling hipStreamQuery instead measured slower: 18.7 against 10.4 us)
        for (int mode = 0; mode < 2; ++mode) {
            std::vector<double> w;
            for (int i = 0; i < 500; ++i) {
                double t0 = now_us();
                hipLaunchKernelGGL(nullptr_kernel, dim3(1), dim3(64), 0, nullptr);
                if (mode == 0)
                    HCHK(hipStreamSynchronize(nullptr));
                else
                    while (hipStreamQuery(nullptr) == hipErrorNotReady) {}
                w.push_back(now_us() - t0);
            }
            std::sort(w.begin(), w.end());
            printf("empty kernel + %s: median %.2f us\n", mode ? "hipStreamQuery poll" : "hipStreamSynchronize",
                   w[w.size() / 2]);
        }
    }
    {
        hipPointerAttribute_t a;
        const int m = 20000;
        double t0 = now_us();
        for (int i = 0; i < m; ++i)
            HCHK(hipPointerGetAttributes(&a, static_cast<char *>(user) + (i & 1023)));
        printf("hipPointerGetAttributes: %.3f us/call\n", (now_us() - t0) / m);
        int d = 0;
        t0 = now_us();
        for (int i = 0; i < m; ++i)
            HCHK(hipGetDevice(&d));
        printf("hipGetDevice: %.3f us/call\n", (now_us() - t0) / m);
        hipStreamCaptureStatus cs;
        t0 = now_us();
        for (int i = 0; i < m; ++i)
            HCHK(hipStreamIsCapturing(s, &cs));
        printf("hipStreamIsCapturing: %.3f us/call\n", (now_us() - t0) / m);
        t0 = now_us();
        for (int i = 0; i < m; ++i)
            (void) hipGetLastError();
        printf("hipGetLastError: %.3f us/call\n", (now_us() - t0) / m);
        t0 = now_us();
        for (int i = 0; i < m; ++i)
            hipLaunchKernelGGL(nullptr_kernel, dim3(1), dim3(64), 0, s);
        double t1 = now_us();
        HCHK(hipStreamSynchronize(s));
        printf("empty kernel launch: %.3f us/call (host enqueue), %.3f us incl. drain\n", (t1 - t0) / m,
               (now_us() - t0) / m);
        t0 = now_us();
        for (int i = 0; i < m; ++i)
            hipLaunchKernelGGL(args36_kernel, dim3(8), dim3(256), 0, s, packed, 1u, 0ull, 0ull, 8u);
        t1 = now_us();
        HCHK(hipStreamSynchronize(s));
        printf("launch with the move kernel's 36-byte argument list: %.3f us/call (host enqueue)\n",
               (t1 - t0) / m);
        Arg528 arg{};
        t0 = now_us();
        for (int i = 0; i < m; ++i)
            hipLaunchKernelGGL(arg_kernel, dim3(32), dim3(256), 0, s, arg);
        t1 = now_us();
        HCHK(hipStreamSynchronize(s));
        printf("launch with a 528-byte argument: %.3f us/call (host enqueue)\n", (t1 - t0) / m);
    }
    {   // round 2: the opal bridge per fragment, as a PML drives it -- one asynchronous
        // opal_convertor_t prepared once, fAdvance called per 8 KiB fragment in order
        dt_elem_desc_t desc[2];
        memset(desc, 0, sizeof(desc));
        desc[0].elem.common.flags = OPAL_DATATYPE_FLAG_DATA | OPAL_DATATYPE_FLAG_CONTIGUOUS;
        desc[0].elem.common.type = 16;   // FLOAT8
        desc[0].elem.count = uint32_t(n) * n;
        desc[0].elem.blocklen = 1;
        desc[0].elem.extent = n * 8;
        desc[1].end_loop.common.type = OPAL_DATATYPE_END_LOOP;
        desc[1].end_loop.size = uint32_t(fs);
        opal_datatype_t dt;
        memset(&dt, 0, sizeof(dt));
        dt.super.obj_reference_count = 1;
        dt.flags = OPAL_DATATYPE_FLAG_COMMITTED | OPAL_DATATYPE_FLAG_DATA;
        dt.size = fs;
        dt.ub = dt.true_ub = ptrdiff_t(n * n - 1) * n * 8 + 8;
        dt.desc.length = dt.opt_desc.length = 2;
        dt.desc.used = dt.opt_desc.used = 1;
        dt.desc.desc = dt.opt_desc.desc = desc;
        opal_accelerator_stream_t ost;
        memset(&ost, 0, sizeof(ost));
        ost.stream = s;
        const size_t frag = 8192;
        std::vector<double> r;
        for (int rep = 0; rep < 5; ++rep) {
            opal_convertor_t oc;
            memset(&oc, 0, sizeof(oc));
            oc.super.obj_reference_count = 1;
            oc.pStack = oc.static_stack;
            oc.stack_size = DT_STATIC_STACK_SIZE;
            oc.flags = CONVERTOR_SEND | CONVERTOR_ACCELERATOR | CONVERTOR_ACCELERATOR_ASYNC | CONVERTOR_HOMOGENEOUS
                       | (CONVERTOR_DATATYPE_MASK & dt.flags);
            oc.local_size = oc.remote_size = fs;
            oc.pBaseBuf = static_cast<unsigned char *>(user);
            oc.count = 1;
            oc.pDesc = &dt;
            oc.use_desc = &dt.opt_desc;
            oc.stream = &ost;
            if (opal_hip_bridge_attach(&oc) != OPAL_SUCCESS) {
                printf("bridge attach failed\n");
                exit(1);
            }
            HCHK(hipStreamSynchronize(s));
            const double t0 = now_us();
            size_t calls = 0;
            int32_t rc = 0;
            while (rc == 0) {
                struct iovec iov{static_cast<char *>(packed) + oc.bConverted, frag};
                uint32_t cnt = 1;
                size_t md = 0;
                rc = oc.fAdvance(&oc, &iov, &cnt, &md);
                ++calls;
            }
            r.push_back((now_us() - t0) / double(calls));
            HCHK(hipStreamSynchronize(s));
        }
        std::sort(r.begin(), r.end());
        printf("opal bridge fAdvance, %zu-byte fragments in order (async): median %.2f us/call (host)\n", frag,
               r[r.size() / 2]);
        opal_hip_bridge_datatype_destruct(&dt);
    }
    ddt_convertor_destroy(c);
    ddt_type_destroy(&x);
    return 0;
}
