// hipthreads.hip -- HIP's own launch path under T threads (1, 2, 4, 8), each on its own stream:
// the control for scripts/bridgethreads.c.  Per T and per operation kind, host microseconds per
// call, device microseconds per operation on each stream, and the aggregate calls per second
// (all calls / the slowest thread's loop time):
//   empty   an empty kernel without arguments (what an engine slot launch costs HIP)
//   args    an empty kernel with 36 bytes of arguments (what a launch with arguments costs)
//   copy    hipMemcpyAsync of 512 KiB device to device (the bytes of one y face)
//   mix     the HIP calls one asynchronous engine call makes around its argument-free launch:
//           hipGetDevice x2, hipPointerGetAttributes x2 (user buffer, iovec), hipStreamIsCapturing,
//           then the empty kernel without arguments
//   cap / attr / dev   the empty kernel without arguments after ONE kind of those calls only:
//           hipStreamIsCapturing, hipPointerGetAttributes x2, hipGetDevice x2
// Not part of the library.
#include <hip/hip_runtime.h>

#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <time.h>

#define MAXT 8

__global__ void k_empty() {}
__global__ void k_args(const void *a, void *b, unsigned long long c, unsigned long long d, unsigned e)
{
    if (e == 0xFFFFFFFFu)
        *(int *) b = *(const int *) a + int(c + d);
}

static double now_us()
{
    timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec * 1e6 + t.tv_nsec * 1e-3;
}

struct Worker {
    int kind, iters;
    hipStream_t s;
    void *a, *b;
    hipEvent_t e0, e1;
    pthread_barrier_t *bar;
    double host_us;
    float dev_ms;
};

static void calls(Worker *w, int n)
{
    for (int i = 0; i < n; ++i) {
        if (w->kind == 0)
            hipLaunchKernelGGL(k_empty, dim3(32), dim3(256), 0, w->s);
        else if (w->kind == 1)
            hipLaunchKernelGGL(k_args, dim3(32), dim3(256), 0, w->s, (const void *) w->a, w->b, 1ull, 2ull, 3u);
        else if (w->kind == 2)
            (void) hipMemcpyAsync(w->b, w->a, 512 << 10, hipMemcpyDeviceToDevice, w->s);
        else {
            int d = 0;
            hipPointerAttribute_t pa;
            hipStreamCaptureStatus cs;
            if (w->kind == 3 || w->kind == 6)
                (void) hipGetDevice(&d);
            if (w->kind == 3 || w->kind == 5) {
                (void) hipPointerGetAttributes(&pa, w->a);
                (void) hipPointerGetAttributes(&pa, w->b);
            }
            if (w->kind == 3 || w->kind == 6)
                (void) hipGetDevice(&d);
            if (w->kind == 3 || w->kind == 4)
                (void) hipStreamIsCapturing(w->s, &cs);
            hipLaunchKernelGGL(k_empty, dim3(32), dim3(256), 0, w->s);
        }
    }
}

static void *run(void *p)
{
    Worker *w = (Worker *) p;
    (void) hipSetDevice(0);
    calls(w, 50);
    (void) hipStreamSynchronize(w->s);
    pthread_barrier_wait(w->bar);
    (void) hipEventRecord(w->e0, w->s);
    const double t0 = now_us();
    calls(w, w->iters);
    w->host_us = now_us() - t0;
    (void) hipEventRecord(w->e1, w->s);
    (void) hipStreamSynchronize(w->s);
    (void) hipEventElapsedTime(&w->dev_ms, w->e0, w->e1);
    return nullptr;
}

int main(int argc, char **argv)
{
    const int iters = argc > 1 ? atoi(argv[1]) : 4000;
    static Worker W[MAXT];
    for (int t = 0; t < MAXT; ++t) {
        if (hipStreamCreateWithFlags(&W[t].s, hipStreamNonBlocking) != hipSuccess || hipMalloc(&W[t].a, 512 << 10) != hipSuccess
            || hipMalloc(&W[t].b, 512 << 10) != hipSuccess || hipEventCreate(&W[t].e0) != hipSuccess
            || hipEventCreate(&W[t].e1) != hipSuccess)
            return 2;
    }
    const char *names[7] = {"empty kernel, no arguments", "empty kernel, 36 B of arguments", "hipMemcpyAsync 512 KiB D2D",
                            "the engine's HIP calls around an argument-free launch",
                            "hipStreamIsCapturing + argument-free launch", "hipPointerGetAttributes x2 + argument-free launch",
                            "hipGetDevice x2 + argument-free launch"};
    const int kmin = argc > 2 ? atoi(argv[2]) : 0;
    const int kmax = argc > 3 ? atoi(argv[3]) : 7;
    for (int kind = kmin; kind < kmax; ++kind) {
        double base = 0;
        for (int T : {1, 2, 4, 8}) {
            pthread_barrier_t bar;
            pthread_barrier_init(&bar, nullptr, unsigned(T));
            pthread_t th[MAXT];
            for (int t = 0; t < T; ++t) {
                W[t].kind = kind;
                W[t].iters = iters;
                W[t].bar = &bar;
                pthread_create(&th[t], nullptr, run, &W[t]);
            }
            double maxloop = 0, sumh = 0, sumd = 0, maxd = 0;
            for (int t = 0; t < T; ++t) {
                pthread_join(th[t], nullptr);
                maxloop = W[t].host_us > maxloop ? W[t].host_us : maxloop;
                sumh += W[t].host_us / iters;
                const double d = W[t].dev_ms * 1e3 / iters;
                sumd += d;
                maxd = d > maxd ? d : maxd;
            }
            pthread_barrier_destroy(&bar);
            const double rate = double(iters) * T / (maxloop * 1e-6);
            if (T == 1)
                base = rate;
            printf("{\"what\": \"HIP control: %s\", \"threads\": %d, \"calls_per_thread\": %d, \"host_us_per_call\": %.3f, "
                   "\"device_us_per_op\": {\"mean\": %.3f, \"max\": %.3f}, \"aggregate_calls_per_s\": %.0f, "
                   "\"speedup_vs_1\": %.3f}\n",
                   names[kind], T, iters, sumh / T, sumd / T, maxd, rate, rate / base);
            fflush(stdout);
        }
    }
    return 0;
}
