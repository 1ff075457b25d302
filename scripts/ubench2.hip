// ubench2.hip -- x-face element ORDER experiments on gfx950 (tuning only, not product).
// Both x faces (x=0 and x=255) of NF fields of a 256^3 double grid: 2*NF*65536 8-byte
// elements at a 2 KiB stride.  The mapping lane -> element changes; traffic does not.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

constexpr size_t FIELD = 256ull * 256 * 256 * 8;
constexpr int NF = 24;                 // 3 GiB: lines touched (384 MiB) exceed the 256 MiB MALL
constexpr uint32_t ROWS = 65536;
constexpr uint32_t N = 2u * NF * ROWS;

// element index -> byte offset in the grid, per ordering
template <int ORD> __device__ __forceinline__ size_t addr_of(uint32_t e)
{
    uint32_t row, field, face;
    if (ORD == 0) {        // face-major, field, row (row fastest)  == engine today
        row = e % ROWS; uint32_t r = e / ROWS; field = r % NF; face = r / NF;
    } else if (ORD == 1) { // row-major pairs: (row, face) adjacent lanes hit one 2 KiB grid row
        face = e & 1; uint32_t r = e >> 1; row = r % ROWS; field = r / ROWS;
    } else if (ORD == 2) { // field fastest: 64 lanes span NF fields
        field = e % NF; uint32_t r = e / NF; face = r & 1; row = r >> 1;
    } else {               // row pairs: 4 consecutive rows x 2 faces per 8 lanes
        face = (e >> 2) & 1; uint32_t r = ((e >> 3) << 2) | (e & 3); row = r % ROWS; field = r / ROWS;
    }
    return size_t(field) * FIELD + size_t(row) * 2048 + (face ? 2040 : 0);
}

template <int ORD, bool NT>
__global__ __launch_bounds__(256) void gather(const uint8_t *__restrict__ g, uint64_t *__restrict__ out)
{
    constexpr int K = 8;
    const uint32_t base = blockIdx.x * 4096u;
    for (uint32_t e0 = base + threadIdx.x; e0 < base + 4096u; e0 += 256 * K) {
        uint64_t v[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint64_t *p = reinterpret_cast<const uint64_t *>(g + addr_of<ORD>(e0 + k * 256));
            v[k] = NT ? __builtin_nontemporal_load(p) : *p;
        }
#pragma unroll
        for (int k = 0; k < K; ++k) out[e0 + k * 256] = v[k];
    }
}

template <int ORD, bool NT>
__global__ __launch_bounds__(256) void scatter(uint8_t *__restrict__ g, const uint64_t *__restrict__ in)
{
    constexpr int K = 8;
    const uint32_t base = blockIdx.x * 4096u;
    for (uint32_t e0 = base + threadIdx.x; e0 < base + 4096u; e0 += 256 * K) {
        uint64_t v[K];
#pragma unroll
        for (int k = 0; k < K; ++k) v[k] = in[e0 + k * 256];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            uint64_t *p = reinterpret_cast<uint64_t *>(g + addr_of<ORD>(e0 + k * 256));
            if (NT) __builtin_nontemporal_store(v[k], p); else *p = v[k];
        }
    }
}

template <typename F> float timeit(F f, int it)
{
    hipEvent_t a, b; CHK(hipEventCreate(&a)); CHK(hipEventCreate(&b));
    f(); CHK(hipDeviceSynchronize());
    CHK(hipEventRecord(a)); for (int i = 0; i < it; ++i) f(); CHK(hipEventRecord(b));
    CHK(hipEventSynchronize(b)); float ms; CHK(hipEventElapsedTime(&ms, a, b)); return ms * 1000.f / it;
}

int main()
{
    static_assert(N % 4096 == 0, "grid split");
    uint8_t *g; uint64_t *p;
    CHK(hipMalloc(&g, FIELD * NF)); CHK(hipMalloc(&p, size_t(N) * 8));
    CHK(hipMemset(g, 1, FIELD * NF));
    const dim3 grid(N / 4096), blk(256);
    auto run = [&](const char *name, auto kg, auto ks) {
        float tg = timeit([&] { hipLaunchKernelGGL(kg, grid, blk, 0, 0, g, p); }, 10);
        float ts = timeit([&] { hipLaunchKernelGGL(ks, grid, blk, 0, 0, g, p); }, 10);
        printf("%-28s gather %6.1f us (%5.1f Gelem/s)   scatter %6.1f us (%5.1f Gelem/s)\n", name, tg, N / tg / 1e3, ts, N / ts / 1e3);
    };
    run("ord0 face,field,row  plain", gather<0, false>, scatter<0, false>);
    run("ord0 face,field,row  nt", gather<0, true>, scatter<0, true>);
    run("ord1 (row,face) pairs plain", gather<1, false>, scatter<1, false>);
    run("ord1 (row,face) pairs nt", gather<1, true>, scatter<1, true>);
    run("ord2 field fastest plain", gather<2, false>, scatter<2, false>);
    run("ord2 field fastest nt", gather<2, true>, scatter<2, true>);
    run("ord3 4rows x 2faces plain", gather<3, false>, scatter<3, false>);
    run("ord3 4rows x 2faces nt", gather<3, true>, scatter<3, true>);
    return 0;
}
