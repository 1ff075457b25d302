// probe_hostrange.cpp -- does hipMemGetAddressRange report the allocation of pinned host
// memory (hipHostMalloc, hipHostRegister) through its device pointer?  (round 2: the
// pinned-iovec check in ddt_convertor.cpp).  Not part of the product.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

static void probe(const char *what, void *p, size_t n)
{
    hipPointerAttribute_t a;
    hipError_t e = hipPointerGetAttributes(&a, p);
    printf("%s: attr %s type %d dev %p host %p\n", what, hipGetErrorString(e), int(a.type), a.devicePointer,
           a.hostPointer);
    for (size_t off : {size_t(0), n / 2, n - 1}) {
        hipDeviceptr_t base = nullptr;
        size_t size = 0;
        e = hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)((char *) a.devicePointer + off));
        printf("  +%zu: range %s base %p size %zu (alloc %p + %zu)\n", off, hipGetErrorString(e), base, size,
               p, n);
        (void) hipGetLastError();
    }
}

int main()
{
    const size_t n = 3u << 20;
    void *h = nullptr;
    if (hipHostMalloc(&h, n, 0) != hipSuccess)
        return 1;
    probe("hipHostMalloc", h, n);
    void *r = aligned_alloc(4096, n);
    if (hipHostRegister(r, n, hipHostRegisterDefault) != hipSuccess)
        return 2;
    probe("hipHostRegister", r, n);
    void *d = nullptr;
    if (hipMalloc(&d, n) != hipSuccess)
        return 3;
    hipDeviceptr_t base = nullptr;
    size_t size = 0;
    hipError_t e = hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)((char *) d + 5));
    printf("hipMalloc: range %s base %p size %zu (alloc %p + %zu)\n", hipGetErrorString(e), base, size, d, n);
    return 0;
}
