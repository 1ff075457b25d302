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
        void *start = nullptr;
        size_t rsize = 0;
        hipError_t e1 = hipPointerGetAttribute(&start, HIP_POINTER_ATTRIBUTE_RANGE_START_ADDR,
                                               (hipDeviceptr_t)((char *) p + off));
        hipError_t e2 = hipPointerGetAttribute(&rsize, HIP_POINTER_ATTRIBUTE_RANGE_SIZE,
                                               (hipDeviceptr_t)((char *) p + off));
        printf("        attribute range: %s start %p / %s size %zu\n", hipGetErrorString(e1), start,
               hipGetErrorString(e2), rsize);
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
    // two registrations of one pageable buffer with an unregistered page gap between them
    char *g = (char *) aligned_alloc(4096, 3 * 4096 * 16);
    if (hipHostRegister(g, 4096 * 16, hipHostRegisterDefault) != hipSuccess
        || hipHostRegister(g + 4096 * 32, 4096 * 16, hipHostRegisterDefault) != hipSuccess)
        return 4;
    probe("gap: first registration", g, 4096 * 16);
    probe("gap: second registration", g + 4096 * 32, 4096 * 16);
    hipPointerAttribute_t ga;
    hipError_t ge = hipPointerGetAttributes(&ga, g + 4096 * 20);
    printf("gap page: attr %s type %d dev %p\n", hipGetErrorString(ge), int(ge == hipSuccess ? ga.type : -1),
           ge == hipSuccess ? ga.devicePointer : nullptr);
    (void) hipGetLastError();
    void *d = nullptr;
    if (hipMalloc(&d, n) != hipSuccess)
        return 3;
    hipDeviceptr_t base = nullptr;
    size_t size = 0;
    hipError_t e = hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)((char *) d + 5));
    printf("hipMalloc: range %s base %p size %zu (alloc %p + %zu)\n", hipGetErrorString(e), base, size, d, n);
    return 0;
}
