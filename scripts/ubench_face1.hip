// ubench_face1.hip -- round 3: the y and z faces of the north star (256^3 double grid, 512
// fields, one face type per launch) through the engine's descriptor kernel (ddt_move_kernel,
// slab on / off) against the by-value single-item kernel (ddt_affine1_kernel), on the items the
// plan compiler emits (scripts/face_{y,z}_item.bin, dumped with ddt_debug_items).  Loops of one
// direction, no flush.  Not part of the product.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../ompi_amd/csrc/ddt_move.hip.h"

using namespace ddt;

#define CHK(x)                                                                          \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);            \
            exit(1);                                                                    \
        }                                                                               \
    } while (0)

template <typename F>
float timeit(F f, int iters)
{
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    f();
    CHK(hipDeviceSynchronize());
    CHK(hipEventRecord(a));
    for (int i = 0; i < iters; ++i) f();
    CHK(hipEventRecord(b));
    CHK(hipEventSynchronize(b));
    float ms;
    CHK(hipEventElapsedTime(&ms, a, b));
    return ms * 1000.f / iters;
}

int main(int argc, char **argv)
{
    const int iters = argc > 1 ? atoi(argv[1]) : 10;
    const uint64_t field = 256ull * 256 * 256 * 8, fields = 512, face = 256ull * 256 * 8;
    const uint64_t ubytes = field * fields, pbytes = face * fields;
    void *u, *p, *p2;
    CHK(hipMalloc(&u, ubytes));
    CHK(hipMalloc(&p, pbytes));
    CHK(hipMalloc(&p2, pbytes));
    CHK(hipMemset(u, 0x5A, ubytes));
    Item *d_it;
    CHK(hipMalloc(&d_it, sizeof(Item)));
    std::vector<char> h1(pbytes), h2(pbytes);
    for (const char *nm : {"y", "z"}) {
        char path[256];
        snprintf(path, sizeof path, "scripts/face_%s_item.bin", nm);
        Item it{};
        FILE *f = fopen(path, "rb");
        if (!f || fread(&it, sizeof(Item), 1, f) != 1) {
            printf("cannot read %s\n", path);
            return 1;
        }
        fclose(f);
        it.user = 0;
        it.packed = 0;
        const uint64_t ub = uint64_t(uintptr_t(u)), pb = uint64_t(uintptr_t(p));
        ItemArgs a{};
        a.ubase = ub; a.pbase = pb; a.u0 = uint32_t(it.u0); a.u1 = uint32_t(it.u1);
        a.cu = uint32_t(it.units_per_task); a.nd = it.ndim; a.fdu = it.fd_upb; a.nt = it.nt;
        for (uint32_t j = 0; j < it.ndim; ++j) {
            a.cnt[j] = uint32_t(it.cnt[j]); a.fd[j] = it.fd[j]; a.ustr[j] = it.ustr[j]; a.pstr[j] = it.pstr[j];
        }
        auto gbs = [&](float us) { return 2.0 * pbytes / (us * 1e3); };
        const uint32_t nt = it.ntasks;
        // correctness: descriptor pack into p2, by-value pack into p
        CHK(hipMemcpy(d_it, &it, sizeof(Item), hipMemcpyHostToDevice));
        hipLaunchKernelGGL((ddt_move_kernel<0, false>), dim3(nt), dim3(THREADS), 0, 0, d_it, 1u, ub, uint64_t(uintptr_t(p2)), nt);
        hipLaunchKernelGGL((ddt_affine1_kernel<0, 3>), dim3(nt), dim3(THREADS), 0, 0, a);
        CHK(hipDeviceSynchronize());
        CHK(hipMemcpy(h1.data(), p, pbytes, hipMemcpyDeviceToHost));
        CHK(hipMemcpy(h2.data(), p2, pbytes, hipMemcpyDeviceToHost));
        printf("%s face: %u tasks, by-value pack %s the descriptor pack\n", nm, nt,
               memcmp(h1.data(), h2.data(), pbytes) ? "DIFFERS FROM" : "matches");
        for (int round = 0; round < 2; ++round) {
            for (uint32_t slab : {0u, SLAB_FULL}) {
                it.slab = slab;
                CHK(hipMemcpy(d_it, &it, sizeof(Item), hipMemcpyHostToDevice));
                float tp = timeit([&] { hipLaunchKernelGGL((ddt_move_kernel<0, false>), dim3(nt), dim3(THREADS), 0, 0, d_it, 1u, ub, pb, nt); }, iters);
                float tu = timeit([&] { hipLaunchKernelGGL((ddt_move_kernel<1, false>), dim3(nt), dim3(THREADS), 0, 0, d_it, 1u, ub, pb, nt); }, iters);
                printf("  descriptor, slab %-3s: pack %6.1f us (%4.0f GB/s, %.3f)  unpack %6.1f us (%4.0f GB/s, %.3f)\n",
                       slab ? "on" : "off", tp, gbs(tp), gbs(tp) / 8000, tu, gbs(tu), gbs(tu) / 8000);
            }
            for (uint32_t slab : {0u, SLAB_FULL}) {
                a.slab = slab;
                float tp = timeit([&] { hipLaunchKernelGGL((ddt_affine1_kernel<0, 3>), dim3(nt), dim3(THREADS), 0, 0, a); }, iters);
                float tu = timeit([&] { hipLaunchKernelGGL((ddt_affine1_kernel<1, 3>), dim3(nt), dim3(THREADS), 0, 0, a); }, iters);
                printf("  by value,   slab %-3s: pack %6.1f us (%4.0f GB/s, %.3f)  unpack %6.1f us (%4.0f GB/s, %.3f)\n",
                       slab ? "on" : "off", tp, gbs(tp), gbs(tp) / 8000, tu, gbs(tu), gbs(tu) / 8000);
            }
        }
    }
    return 0;
}
