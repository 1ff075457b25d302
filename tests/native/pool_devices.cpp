// pool_devices.cpp -- CPU unit test of ddt_pool.cpp's cross-device settling.
//
// ddt_pool.cpp is linked against a mock of the few HIP runtime calls it makes (two fake
// devices, host memory for "device" blocks, events that never pass), so the test runs without a
// GPU.  A release on device 1 that could take no fence ("unknown") must NOT be settled by a
// device-0 allocation -- that allocation's hipDeviceSynchronize covers device 0 only -- and must
// be settled by the next device-1 allocation that has to call hipMalloc.  Test infrastructure.
#include <cstdio>
#include <cstdlib>
#include <set>
#include <vector>

#include <hip/hip_runtime.h>

#include "ddt_pool.h"

static int g_dev = 0;
static std::set<int> g_synced;
static std::set<void *> g_freed;

extern "C" {
hipError_t hipGetDevice(int *d) { *d = g_dev; return hipSuccess; }
hipError_t hipSetDevice(int d) { g_dev = d; return hipSuccess; }
hipError_t hipGetLastError(void) { return hipSuccess; }
hipError_t hipDeviceSynchronize(void) { g_synced.insert(g_dev); return hipSuccess; }
hipError_t hipMalloc(void **p, size_t n) { *p = std::malloc(n); return hipSuccess; }
hipError_t hipFree(void *p) { g_freed.insert(p); return hipSuccess; }
hipError_t hipEventQuery(hipEvent_t) { return hipErrorNotReady; }
hipError_t hipEventDestroy(hipEvent_t) { return hipSuccess; }
hipError_t hipEventCreateWithFlags(hipEvent_t *e, unsigned) { *e = (hipEvent_t) 0x1; return hipSuccess; }
hipError_t hipEventRecord(hipEvent_t, hipStream_t) { return hipSuccess; }
hipError_t hipStreamIsCapturing(hipStream_t, hipStreamCaptureStatus *s) { *s = hipStreamCaptureStatusNone; return hipSuccess; }
}

#define CHECK(c) do { if (!(c)) { std::printf("FAIL %s:%d %s\n", __FILE__, __LINE__, #c); return 1; } } while (0)

int main()
{
    int64_t st[6];
    hipSetDevice(1);
    void *b1 = ddt::pool_alloc(4096);
    CHECK(b1);
    ddt::pool_release({b1}, {}, /*unknown=*/true);   // e.g. its stream was destroyed

    hipSetDevice(0);
    void *b0 = ddt::pool_alloc(4096);                 // must not recycle device-1 memory
    CHECK(b0 && b0 != b1);
    CHECK(g_synced.count(1) == 0);
    ddt::pool_stats(st);
    CHECK(st[2] == 1);                                // b1 still waits on its settle

    // a fenced release on device 0 whose event never passes stays out of reach as well
    ddt::pool_release({b0}, {(hipEvent_t) 0x1}, false);
    void *c0 = ddt::pool_alloc(4096);
    CHECK(c0 != b0 && c0 != b1);

    hipSetDevice(1);
    void *b2 = ddt::pool_alloc(4096);                 // device 1 settles its own unknown release
    CHECK(g_synced.count(1) == 1);
    CHECK(b2 == b1);
    ddt::pool_stats(st);
    CHECK(st[2] == 1);                                // only b0 (fenced, device 0) still waits
    CHECK(g_freed.empty());
    std::printf("ok\n");
    return 0;
}
