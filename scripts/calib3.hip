// calib3.hip -- the cfg2 halo's traffic at the halo's own addresses, in different orders.  Round 5
// question: the engine's unpack spends ~70 us on the x faces where scripts/calib2.hip's bare pair
// (one line per 2 KiB, right after the gather) needs 51 us.  Is the gap the halo's addresses (two
// lines per 2 KiB row, 16 fields of 128 MiB) or the y/z + packed-stream traffic between the x
// gather and the x scatter (evicting gathered lines from the Infinity Cache)?  If the order
// matters, the engine can order its tasks (x last in the pack, first in the unpack).  Not part of
// the product.
//
// Buffers: 16 fields of 256^3 doubles (2 GiB), a 48 MiB packed buffer.  Kernels: x gather (plain
// 8-B loads, one per line, non-temporal packed stores), x scatter (non-temporal packed loads;
// non-temporal or plain 8-B stores), y/z pack and unpack (16-B lanes, non-temporal both sides).
// Sequences, each after a 1 GiB plain-read flush, timed per kernel with events.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHK(x)                                                                          \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);       \
            std::exit(1);                                                               \
        }                                                                               \
    } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr size_t N = 256, F = 16, E = 8;
constexpr size_t ROW = N * E, PLANE = N * ROW, FIELD = N * PLANE;
constexpr size_t NX = F * 2 * N * N;            // x elements (2 Mi)
constexpr size_t YZ16 = F * 4 * N * N * E / 16; // y + z faces in 16-B units (2 Mi)

__global__ __launch_bounds__(256) void flush(const u32x4 *__restrict__ p, size_t n, uint32_t *sink)
{
    uint32_t acc = 0;
    for (size_t i = size_t(blockIdx.x) * 256 + threadIdx.x; i < n; i += size_t(gridDim.x) * 256) {
        const u32x4 v = p[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x9E3779B9u)
        sink[threadIdx.x] = acc;
}

// x element t: row r = t % (N*N), face s = (t / (N*N)) % 2, field f = t / (2*N*N); PAIR: the two
// faces' elements of one row adjacent (s = t % 2), so a row's two lines are touched together
template <bool PAIR = false>
__device__ __forceinline__ size_t xoff(size_t t)
{
    if (PAIR) {
        const size_t s = t & 1, r = (t >> 1) % (N * N), f = t / (2 * N * N);
        return f * FIELD + r * ROW + s * (ROW - E);
    }
    const size_t r = t % (N * N), s = (t / (N * N)) & 1, f = t / (2 * N * N);
    return f * FIELD + r * ROW + s * (ROW - E);
}

template <bool PAIR = false>
__global__ __launch_bounds__(256) void xgather(const uint8_t *__restrict__ u, uint64_t *__restrict__ p)
{
    const size_t t = size_t(blockIdx.x) * 256 + threadIdx.x;
    if (t < NX)
        __builtin_nontemporal_store(*reinterpret_cast<const uint64_t *>(u + xoff<PAIR>(t)), p + t);
}

template <bool NTS, bool PAIR = false>
__global__ __launch_bounds__(256) void xscatter(uint8_t *__restrict__ u, const uint64_t *__restrict__ p)
{
    const size_t t = size_t(blockIdx.x) * 256 + threadIdx.x;
    if (t >= NX)
        return;
    uint64_t *q = reinterpret_cast<uint64_t *>(u + xoff<PAIR>(t));
    const uint64_t v = __builtin_nontemporal_load(p + t);
    if (NTS)
        __builtin_nontemporal_store(v, q);
    else
        *q = v;
}

// y/z 16-B unit t: the first half are y rows (field f, face s, plane k: 2 KiB rows), the second
// half z planes (field f, face s: 512 KiB contiguous)
__device__ __forceinline__ size_t yzoff(size_t t)
{
    const size_t half = YZ16 / 2;
    if (t < half) {
        const size_t w = t % (ROW / 16), k = (t / (ROW / 16)) % N, s = (t / (ROW / 16 * N)) & 1,
                     f = t / (ROW / 16 * N * 2);
        return f * FIELD + k * PLANE + s * (N - 1) * ROW + w * 16;
    }
    t -= half;
    const size_t w = t % (PLANE / 16), s = (t / (PLANE / 16)) & 1, f = t / (PLANE / 16 * 2);
    return f * FIELD + s * (N - 1) * PLANE + w * 16;
}

template <int DIR>
__global__ __launch_bounds__(256) void yz(uint8_t *__restrict__ u, u32x4 *__restrict__ p)
{
    const size_t t = size_t(blockIdx.x) * 256 + threadIdx.x;
    if (t >= YZ16)
        return;
    u32x4 *q = reinterpret_cast<u32x4 *>(u + yzoff(t));
    if (DIR == 0)
        __builtin_nontemporal_store(__builtin_nontemporal_load(q), p + t);
    else
        __builtin_nontemporal_store(__builtin_nontemporal_load(p + t), q);
}

int main(int argc, char **argv)
{
    const int reps = argc > 1 ? std::atoi(argv[1]) : 5;
    uint8_t *u = nullptr, *pk = nullptr;
    u32x4 *fl = nullptr;
    uint32_t *sink = nullptr;
    const size_t nflush = (size_t(1) << 30) / 16;
    CHK(hipMalloc(&u, F * FIELD));
    CHK(hipMalloc(&pk, NX * 8 + YZ16 * 16));
    CHK(hipMalloc(&fl, nflush * 16));
    CHK(hipMalloc(&sink, 1024));
    CHK(hipMemset(u, 1, F * FIELD));
    CHK(hipMemset(fl, 2, nflush * 16));
    CHK(hipDeviceSynchronize());
    uint64_t *px = reinterpret_cast<uint64_t *>(pk);
    u32x4 *pyz = reinterpret_cast<u32x4 *>(pk + NX * 8);
    const dim3 gx(uint32_t(NX / 256)), gyz(uint32_t(YZ16 / 256)), b(256);
    hipEvent_t ev[8];
    for (auto &e : ev)
        CHK(hipEventCreate(&e));
    // op codes: 0 x gather, 1 x scatter nt, 2 x scatter plain, 3 yz pack, 4 yz unpack; 5-7 the
    // x kernels with a row's two face elements adjacent
    const char *oname[8] = {"xg", "xs_nt", "xs_plain", "yzp", "yzu", "xg_pair", "xs_nt_pair", "xs_plain_pair"};
    struct Seq { const char *name; int n; int op[4]; };
    const Seq seqs[] = {
        {"x_alone_nt", 2, {0, 1}},
        {"x_alone_plain", 2, {0, 2}},
        {"x_outer_nt", 4, {0, 3, 4, 1}},      // x gather, y/z pack, y/z unpack, x scatter
        {"x_inner_nt", 4, {3, 0, 1, 4}},      // y/z pack, x gather, x scatter, y/z unpack
        {"x_first_nt", 4, {0, 3, 1, 4}},      // x first in both passes
        {"x_pack_last_nt", 4, {3, 0, 4, 1}},  // x last in both passes
        {"x_inner_plain", 4, {3, 0, 2, 4}},
        {"x_first_plain", 4, {0, 3, 2, 4}},
        {"x_alone_nt_pair", 2, {5, 6}},
        {"x_alone_plain_pair", 2, {5, 7}},
        {"x_first_nt_pair", 4, {5, 3, 6, 4}},
    };
    for (const Seq &s : seqs) {
        float acc[4] = {0, 0, 0, 0}, tot = 0;
        for (int r = 0; r < reps; ++r) {
            hipLaunchKernelGGL(flush, dim3(4096), b, 0, nullptr, fl, nflush, sink);
            CHK(hipEventRecord(ev[0], nullptr));
            for (int i = 0; i < s.n; ++i) {
                switch (s.op[i]) {
                case 0: hipLaunchKernelGGL(xgather<false>, gx, b, 0, nullptr, u, px); break;
                case 1: hipLaunchKernelGGL(xscatter<true>, gx, b, 0, nullptr, u, px); break;
                case 2: hipLaunchKernelGGL(xscatter<false>, gx, b, 0, nullptr, u, px); break;
                case 3: hipLaunchKernelGGL(yz<0>, gyz, b, 0, nullptr, u, pyz); break;
                case 5: hipLaunchKernelGGL(xgather<true>, gx, b, 0, nullptr, u, px); break;
                case 6: hipLaunchKernelGGL((xscatter<true, true>), gx, b, 0, nullptr, u, px); break;
                case 7: hipLaunchKernelGGL((xscatter<false, true>), gx, b, 0, nullptr, u, px); break;
                default: hipLaunchKernelGGL(yz<1>, gyz, b, 0, nullptr, u, pyz); break;
                }
                CHK(hipEventRecord(ev[i + 1], nullptr));
            }
            CHK(hipEventSynchronize(ev[s.n]));
            for (int i = 0; i < s.n; ++i) {
                float ms = 0;
                CHK(hipEventElapsedTime(&ms, ev[i], ev[i + 1]));
                acc[i] += ms;
            }
            float ms = 0;
            CHK(hipEventElapsedTime(&ms, ev[0], ev[s.n]));
            tot += ms;
        }
        std::printf("{\"seq\": \"%s\", \"total_us\": %.2f", s.name, tot * 1e3 / reps);
        for (int i = 0; i < s.n; ++i)
            std::printf(", \"%d_%s_us\": %.2f", i, oname[s.op[i]], acc[i] * 1e3 / reps);
        std::printf("}\n");
    }
    return 0;
}
