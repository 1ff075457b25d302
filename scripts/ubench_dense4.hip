// ubench_dense4.hip -- round 3: where the engine's line-dense pack loses to the bare
// one-chunk-per-workgroup kernel on BASELINE config 5 (engine 1183-1197 us with two chunks per
// task, 1483 us with one; bare 1075-1082 us, scripts/ubench_dense2.hip / ubench_dense3.hip).
// Runs the ENGINE's own ddt_dense_kernel (ddt_move.hip.h) on config 5's launch descriptor
// (scripts/cfg5_item.bin, dumped with ddt_debug_items), then lean kernels that read the same
// descriptor, each adding one of the engine's costs.  Not part of the product.
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

constexpr uint64_t NREC = 128ull << 20;
constexpr uint32_t REC = 20, STRIDE = 32, WPR = REC / 4, R = 128;
constexpr uint32_t NCH = uint32_t(NREC / R);
constexpr uint32_t NO = R * REC / 16;

__global__ __launch_bounds__(256) void pack_b(const u32x4 *__restrict__ user, u32x4 *__restrict__ packed)
{
    __shared__ u32x4 buf[256];
    const uint64_t ch = blockIdx.x;
    buf[threadIdx.x] = __builtin_nontemporal_load(user + ch * 256 + threadIdx.x);
    __syncthreads();
    const uint32_t *lds = reinterpret_cast<const uint32_t *>(buf);
    u32x4 *dst = packed + ch * NO;
    for (uint32_t c = threadIdx.x; c < NO; c += 256) {
        uint32_t d[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint32_t q = 4 * c + uint32_t(i), r = q / WPR, w = q - r * WPR;
            d[i] = lds[r * (STRIDE / 4) + w];
        }
        dst[c] = u32x4{d[0], d[1], d[2], d[3]};
    }
}

// Lean: one chunk of R records per workgroup, everything from the descriptor.
//   MODE 0: runtime S / blen / R and fastdiv from the item, one-dim nest, 16-byte aligned
//           spans assumed (the bare kernel with its constants made runtime)
//   MODE 1: + the engine's locate_task (item search, slab remap when it->slab)
//   MODE 2: + the engine's generic first-record nest loop and inner-run check
template <int MODE>
__global__ __launch_bounds__(256) void pack_lean(const Item *__restrict__ items, uint32_t nitems, uint64_t ubase,
                                                 uint64_t pbase)
{
    __shared__ u32x4 buf[256];
    const Item *it = items;
    uint64_t rec0;
    if (MODE >= 1) {
        uint64_t ub, ue;
        it = locate_task(items, nitems, blockIdx.x, ub, ue);
        rec0 = ub / it->upb;
    } else {
        rec0 = uint64_t(blockIdx.x) * it->nbytes;
    }
    int64_t uo, po;
    if (MODE >= 2) {
        const uint32_t nd = it->ndim, inner = nd - 1;
        const uint32_t cin = uint32_t(it->cnt[inner]);
        if (uint32_t(rec0) % cin + uint32_t(it->nbytes) > cin)
            return;
        uo = 0;
        po = 0;
        uint32_t blk = uint32_t(rec0);
        for (int j = int(nd) - 1; j > 0; --j) {
            const uint32_t q = fastdiv(blk, it->fd[j]);
            const uint32_t idx = blk - q * uint32_t(it->cnt[j]);
            blk = q;
            uo += int64_t(idx) * it->ustr[j];
            po += int64_t(idx) * it->pstr[j];
        }
        uo += int64_t(blk) * it->ustr[0];
        po += int64_t(blk) * it->pstr[0];
    } else {
        uo = int64_t(rec0) * it->ustr[0];
        po = int64_t(rec0) * it->pstr[0];
    }
    const uint32_t S = uint32_t(it->ustr[it->ndim - 1]), blen = uint32_t(it->upb) * it->U;
    const uint32_t Rn = uint32_t(it->nbytes);
    const FastDiv fw = it->fd_nblk;
    const u32x4 *src = reinterpret_cast<const u32x4 *>(ubase + it->user + uint64_t(uo));
    const uint32_t nvec = ((Rn - 1) * S + blen + 15) / 16;
    if (threadIdx.x < nvec)
        buf[threadIdx.x] = __builtin_nontemporal_load(src + threadIdx.x);
    __syncthreads();
    const uint32_t *lds = reinterpret_cast<const uint32_t *>(buf);
    u32x4 *dst = reinterpret_cast<u32x4 *>(pbase + it->packed + uint64_t(po));
    const uint32_t no = Rn * blen / 16;
    for (uint32_t c = threadIdx.x; c < no; c += 256) {
        uint32_t w[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint32_t q = 4 * c + uint32_t(i), r = fastdiv(q, fw);
            w[i] = lds[(r * S) / 4 + (q - r * fw.d)];
        }
        dst[c] = u32x4{w[0], w[1], w[2], w[3]};
    }
}

// The engine's run_dense1 called straight from a minimal kernel (no dense_body loop, no
// locate_task): task b = units [b * upt, (b + 1) * upt)
__global__ __launch_bounds__(256) void pack_r1(const Item *__restrict__ items, uint64_t ubase, uint64_t pbase)
{
    __shared__ u32x4 buf[DENSE_LDS / 16 + 2];
    const Item *it = items;
    const uint32_t upt = uint32_t(it->units_per_task);
    const uint32_t ub = uint32_t(it->u0) + blockIdx.x * upt;
    run_dense1<0>(it, Bases{ubase, pbase}, ub, ub + upt, buf);
}

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
    const char *path = argc > 2 ? argv[2] : "scripts/cfg5_item.bin";
    Item base{};
    FILE *f = fopen(path, "rb");
    if (!f || fread(&base, sizeof(Item), 1, f) != 1) {
        printf("cannot read %s\n", path);
        return 1;
    }
    fclose(f);
    base.user = 0;
    base.packed = 0;
    const uint64_t ubytes = NREC * STRIDE, pbytes = NREC * REC;
    void *u, *p, *ref;
    Item *d_it;
    CHK(hipMalloc(&u, ubytes));
    CHK(hipMalloc(&p, pbytes));
    CHK(hipMalloc(&ref, pbytes));
    CHK(hipMalloc(&d_it, sizeof(Item)));
    {
        std::vector<uint32_t> h(ubytes / 4);
        uint32_t x = 12345;
        for (auto &w : h) { x = x * 1664525u + 1013904223u; w = x; }
        CHK(hipMemcpy(u, h.data(), ubytes, hipMemcpyHostToDevice));
    }
    hipLaunchKernelGGL(pack_b, dim3(NCH), dim3(256), 0, 0, (const u32x4 *) u, (u32x4 *) ref);
    CHK(hipDeviceSynchronize());
    std::vector<char> hr(pbytes), hp(pbytes);
    CHK(hipMemcpy(hr.data(), ref, pbytes, hipMemcpyDeviceToHost));
    auto check = [&](const char *nm) {
        CHK(hipDeviceSynchronize());
        CHK(hipMemcpy(hp.data(), p, pbytes, hipMemcpyDeviceToHost));
        if (memcmp(hp.data(), hr.data(), pbytes) != 0) printf("  MISMATCH in %s\n", nm);
        CHK(hipMemset(p, 0, pbytes));
    };
    auto gbs = [&](float us) { return (ubytes + pbytes) / (us * 1e3); };
    const uint64_t ub = uint64_t(uintptr_t(u)), pb = uint64_t(uintptr_t(p));
    auto set_item = [&](uint32_t chunks_per_task, uint32_t slab) {
        Item it = base;
        it.units_per_task = uint64_t(chunks_per_task) * R * it.upb;
        it.ntasks = uint32_t((it.u1 - it.u0 + it.units_per_task - 1) / it.units_per_task);
        it.slab = slab;
        CHK(hipMemcpy(d_it, &it, sizeof(Item), hipMemcpyHostToDevice));
        return it.ntasks;
    };
    printf("config-5 pack: engine kernel vs lean kernels, %d iterations per figure\n", iters);
    for (int round = 0; round < 2; ++round) {
        float t = timeit([&] { hipLaunchKernelGGL(pack_b, dim3(NCH), dim3(256), 0, 0, (const u32x4 *) u, (u32x4 *) p); }, iters);
        printf("B   bare, one chunk per workgroup            : %7.1f us (%4.0f GB/s)\n", t, gbs(t));
        for (uint32_t cpt : {1u, 2u}) {
            for (uint32_t slab : {0u, SLAB_FULL}) {
                const uint32_t nt = set_item(cpt, slab);
                t = timeit([&] { hipLaunchKernelGGL((ddt_dense_kernel<0, false>), dim3(nt), dim3(256), 0, 0, d_it, 1u, ub, pb, nt); }, iters);
                if (!round) check("engine");
                printf("E   engine kernel, %u chunk(s)/task, slab %-3s: %7.1f us (%4.0f GB/s)\n", cpt, slab ? "on" : "off", t, gbs(t));
            }
        }
        set_item(1, 0);
        t = timeit([&] { hipLaunchKernelGGL(pack_lean<0>, dim3(NCH), dim3(256), 0, 0, d_it, 1u, ub, pb); }, iters);
        if (!round) check("lean0");
        printf("L0  lean, runtime shape from the item        : %7.1f us (%4.0f GB/s)\n", t, gbs(t));
        t = timeit([&] { hipLaunchKernelGGL(pack_lean<1>, dim3(NCH), dim3(256), 0, 0, d_it, 1u, ub, pb); }, iters);
        if (!round) check("lean1");
        printf("L1  + locate_task                            : %7.1f us (%4.0f GB/s)\n", t, gbs(t));
        t = timeit([&] { hipLaunchKernelGGL(pack_lean<2>, dim3(NCH), dim3(256), 0, 0, d_it, 1u, ub, pb); }, iters);
        if (!round) check("lean2");
        printf("L2  + generic nest and inner-run check       : %7.1f us (%4.0f GB/s)\n", t, gbs(t));
        set_item(1, 0);
        t = timeit([&] { hipLaunchKernelGGL(pack_r1, dim3(NCH), dim3(256), 0, 0, d_it, ub, pb); }, iters);
        if (!round) check("r1");
        printf("R1  engine run_dense1 from a minimal kernel   : %7.1f us (%4.0f GB/s)\n", t, gbs(t));
        {
            ItemArgs da{};
            da.ubase = ub; da.pbase = pb; da.u0 = uint32_t(base.u0); da.u1 = uint32_t(base.u1);
            da.cu = uint32_t(R * base.upb); da.nd = base.ndim; da.fdu = base.fd_upb; da.fw = base.fd_nblk;
            da.nt = base.nt;
            for (uint32_t j = 0; j < base.ndim; ++j) {
                da.cnt[j] = uint32_t(base.cnt[j]); da.fd[j] = base.fd[j]; da.ustr[j] = base.ustr[j]; da.pstr[j] = base.pstr[j];
            }
            t = timeit([&] { hipLaunchKernelGGL(ddt_dense1_kernel<0>, dim3(NCH), dim3(256), 0, 0, da); }, iters);
            if (!round) check("dense1");
            printf("V   engine ddt_dense1_kernel (by value)      : %7.1f us (%4.0f GB/s)\n", t, gbs(t));
        }
        set_item(1, SLAB_FULL);
        t = timeit([&] { hipLaunchKernelGGL(pack_lean<2>, dim3(NCH), dim3(256), 0, 0, d_it, 1u, ub, pb); }, iters);
        if (!round) check("lean2s");
        printf("L2s + slab mapping                           : %7.1f us (%4.0f GB/s)\n", t, gbs(t));
    }
    return 0;
}
