// probe_capture.cpp -- which HIP calls may one thread make while ANOTHER thread captures a
// stream in hipStreamCaptureModeGlobal (torch.cuda.graph's default), without an error and
// without invalidating that capture?  Round 3: grounds the engine's non-blocking datatype
// destruction (ddt_pool.cpp).  For each call: thread B begins a global-mode capture and
// enqueues a kernel, thread A makes the call, then B enqueues another kernel and ends the
// capture.  Prints A's return code and B's end-capture result.  Round 5: the same calls again
// with thread A switched to hipStreamCaptureModeRelaxed (hipThreadExchangeStreamCaptureMode),
// the mode the engine's attach-time table build runs under.  Not part of the product.
#include <hip/hip_runtime.h>

#include <condition_variable>
#include <cstdio>
#include <functional>
#include <mutex>
#include <thread>

__global__ void tick(int *p) { atomicAdd(p, 1); }

struct Gate {
    std::mutex m;
    std::condition_variable cv;
    int stage = 0;
    void set(int s)
    {
        std::lock_guard<std::mutex> g(m);
        stage = s;
        cv.notify_all();
    }
    void wait(int s)
    {
        std::unique_lock<std::mutex> g(m);
        cv.wait(g, [&] { return stage >= s; });
    }
};

int main()
{
    int *d = nullptr;
    (void) hipMalloc(&d, 4);
    hipStream_t sa, sb;
    (void) hipStreamCreateWithFlags(&sa, hipStreamNonBlocking);
    (void) hipStreamCreateWithFlags(&sb, hipStreamNonBlocking);
    hipEvent_t done;
    (void) hipEventCreateWithFlags(&done, hipEventDisableTiming);
    hipLaunchKernelGGL(tick, dim3(1), dim3(1), 0, sa, d);
    (void) hipEventRecord(done, sa);
    (void) hipStreamSynchronize(sa);
    void *pool_blk = nullptr;
    (void) hipMalloc(&pool_blk, 1 << 20);

    struct Case {
        const char *name;
        std::function<hipError_t()> call;
    };
    Case cases[] = {
        {"hipEventCreate", [] { hipEvent_t e; hipError_t r = hipEventCreateWithFlags(&e, hipEventDisableTiming); if (r == hipSuccess) (void) hipEventDestroy(e); return r; }},
        {"hipEventRecord(other stream)", [&] { hipEvent_t e; (void) hipEventCreateWithFlags(&e, hipEventDisableTiming); hipError_t r = hipEventRecord(e, sa); (void) hipEventDestroy(e); return r; }},
        {"hipEventQuery", [&] { return hipEventQuery(done); }},
        {"hipEventSynchronize", [&] { return hipEventSynchronize(done); }},
        {"hipStreamIsCapturing(other)", [&] { hipStreamCaptureStatus cs; return hipStreamIsCapturing(sa, &cs); }},
        {"hipStreamQuery(other)", [&] { return hipStreamQuery(sa); }},
        {"hipStreamSynchronize(other)", [&] { return hipStreamSynchronize(sa); }},
        {"hipMemcpyAsync H2D(other)+sync", [&] { static int h = 1; hipError_t r = hipMemcpyAsync(pool_blk, &h, 4, hipMemcpyHostToDevice, sa); if (r == hipSuccess) r = hipStreamSynchronize(sa); return r; }},
        {"kernel launch(other)", [&] { hipLaunchKernelGGL(tick, dim3(1), dim3(1), 0, sa, d); return hipGetLastError(); }},
        {"hipMalloc", [] { void *p = nullptr; hipError_t r = hipMalloc(&p, 1 << 20); if (p) (void) hipFree(p); return r; }},
        {"hipFree", [] { void *p = nullptr; (void) hipMalloc(&p, 1 << 20); return hipFree(p); }},
        {"hipDeviceSynchronize", [] { return hipDeviceSynchronize(); }},
    };
    for (int relaxed = 0; relaxed < 2; ++relaxed)
    for (Case &c : cases) {
        Gate g;
        hipError_t ra = hipSuccess, rb = hipSuccess, rl = hipSuccess;
        hipGraph_t graph = nullptr;
        std::thread b([&] {
            rb = hipStreamBeginCapture(sb, hipStreamCaptureModeGlobal);
            hipLaunchKernelGGL(tick, dim3(1), dim3(1), 0, sb, d);
            g.set(1);
            g.wait(2);
            hipLaunchKernelGGL(tick, dim3(1), dim3(1), 0, sb, d);
            rl = hipGetLastError();
            hipError_t re = hipStreamEndCapture(sb, &graph);
            if (rb == hipSuccess)
                rb = re;
        });
        std::thread a([&] {
            g.wait(1);
            hipStreamCaptureMode mode = hipStreamCaptureModeRelaxed;
            if (relaxed)
                (void) hipThreadExchangeStreamCaptureMode(&mode);
            ra = c.call();
            if (relaxed)
                (void) hipThreadExchangeStreamCaptureMode(&mode);
            (void) hipGetLastError();
            g.set(2);
        });
        a.join();
        b.join();
        printf("%s%-32s A: %-36s  B's capture: %s%s\n", relaxed ? "[A relaxed] " : "", c.name, hipGetErrorName(ra), hipGetErrorName(rb),
               rl != hipSuccess ? " (launch after the call failed)" : "");
        if (graph)
            (void) hipGraphDestroy(graph);
        (void) hipDeviceSynchronize();
        (void) hipGetLastError();
    }
    return 0;
}
