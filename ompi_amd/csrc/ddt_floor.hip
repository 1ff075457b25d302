// ddt_floor.hip -- bare gfx950 kernels that price a workload's parts (measurement only, not the
// product; bench.py loads libddt_floor.so beside the engine to report `floor_us`).
//
// A derived-datatype move is made of a few access primitives, each with its own ceiling on this
// chip:
//   element gather   one 4- or 8-byte element per user-side position (the halo's x faces: one
//                    element per 128-byte line, bound by the memory side's line rate);
//   element scatter  the reverse with non-temporal stores (a partial-line write each);
//   block copy       runs of >= 16 bytes (y rows, z planes) at the streaming rate;
//   records          short records at a pitch within each line (config 5), through LDS;
//   listed elements  4-byte elements in address order from an index list (config 4).
// Each kernel here does only its primitive, with the shape passed by value and the positions
// decomposed by shifts -- no descriptors, no task search, no window logic.  The engine is
// compared with the sum of the parts measured in the same run, on the same buffers, in the same
// pack-then-unpack order and with the same cache policies (plain gathers, non-temporal scatters,
// non-temporal streaming loads).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <vector>

namespace {

typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// position p (element or block index) -> user offset: p = ((i2 << l1) | i1) << l0 | i0
struct Shape {
    int64_t s0, s1, s2, base;
    uint32_t l0, l1;
    uint64_t n;   // positions
};

__device__ __forceinline__ int64_t user_off(const Shape &sh, uint64_t p)
{
    const uint64_t i0 = p & ((uint64_t(1) << sh.l0) - 1);
    const uint64_t i1 = (p >> sh.l0) & ((uint64_t(1) << sh.l1) - 1);
    const uint64_t i2 = p >> (sh.l0 + sh.l1);
    return sh.base + int64_t(i0) * sh.s0 + int64_t(i1) * sh.s1 + int64_t(i2) * sh.s2;
}

template <int E> struct Vec;
template <> struct Vec<4> { typedef unsigned int T; };
template <> struct Vec<8> { typedef u32x2 T; };

constexpr int K = 8;   // elements in flight per lane

template <int E>
__global__ __launch_bounds__(256) void gather(const uint8_t *__restrict__ user, uint8_t *__restrict__ packed,
                                              Shape sh)
{
    typedef typename Vec<E>::T T;
    const uint64_t p0 = uint64_t(blockIdx.x) * 256 * K + threadIdx.x;
    T v[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const uint64_t p = p0 + uint64_t(k) * 256;
        if (p < sh.n)
            v[k] = *reinterpret_cast<const T *>(user + user_off(sh, p));
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const uint64_t p = p0 + uint64_t(k) * 256;
        if (p < sh.n)
            reinterpret_cast<T *>(packed)[p] = v[k];
    }
}

template <int E>
__global__ __launch_bounds__(256) void scatter(uint8_t *__restrict__ user, const uint8_t *__restrict__ packed,
                                               Shape sh)
{
    typedef typename Vec<E>::T T;
    const uint64_t p0 = uint64_t(blockIdx.x) * 256 * K + threadIdx.x;
    T v[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const uint64_t p = p0 + uint64_t(k) * 256;
        if (p < sh.n)
            v[k] = reinterpret_cast<const T *>(packed)[p];
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const uint64_t p = p0 + uint64_t(k) * 256;
        if (p < sh.n)
            __builtin_nontemporal_store(v[k], reinterpret_cast<T *>(user + user_off(sh, p)));
    }
}

// blocks of (1 << lw) 16-byte units; a workgroup moves 16 KiB (4 units per lane in flight)
template <int DIR>
__global__ __launch_bounds__(256) void copy_blocks(uint8_t *__restrict__ user, uint8_t *__restrict__ packed,
                                                   Shape sh, uint32_t lw)
{
    const uint64_t units = sh.n << lw;
    const uint64_t u0 = uint64_t(blockIdx.x) * 1024 + threadIdx.x;
    u32x4 v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint64_t u = u0 + uint64_t(k) * 256;
        if (u >= units)
            continue;
        const int64_t uo = user_off(sh, u >> lw) + int64_t(u & ((uint64_t(1) << lw) - 1)) * 16;
        v[k] = DIR == 0 ? __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(user + uo))
                        : __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(packed) + u);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint64_t u = u0 + uint64_t(k) * 256;
        if (u >= units)
            continue;
        const int64_t uo = user_off(sh, u >> lw) + int64_t(u & ((uint64_t(1) << lw) - 1)) * 16;
        if (DIR == 0)
            reinterpret_cast<u32x4 *>(packed)[u] = v[k];
        else
            *reinterpret_cast<u32x4 *>(user + uo) = v[k];
    }
}

// Records of REC bytes at a STRIDE-byte pitch (BASELINE config 5: 20 of every 32 bytes), one 4 KiB
// user-span chunk per workgroup through LDS -- the bare kernels of r3 (scripts/ubench_dense4.hip
// pack_b, ubench_dense5.hip unpack U0): whole 16-byte loads of the span, packed stores built from
// LDS; the unpack stores each record with plain dwordx4 + dword stores.
template <uint32_t REC, uint32_t STRIDE>
__global__ __launch_bounds__(256) void records_pack(const uint8_t *__restrict__ user, uint8_t *__restrict__ packed,
                                                    uint64_t nrec)
{
    constexpr uint32_t R = 4096 / STRIDE, WPR = REC / 4, NO = R * REC / 16;
    __shared__ u32x4 buf[256];
    const uint64_t ch = blockIdx.x;
    const u32x4 *src = reinterpret_cast<const u32x4 *>(user) + ch * 256;
    if (ch * R + (threadIdx.x * 16u) / STRIDE < nrec)
        buf[threadIdx.x] = __builtin_nontemporal_load(src + threadIdx.x);
    __syncthreads();
    const uint32_t *lds = reinterpret_cast<const uint32_t *>(buf);
    u32x4 *dst = reinterpret_cast<u32x4 *>(packed) + ch * NO;
    const uint64_t left = (nrec - ch * R) * REC / 16;
    for (uint32_t c = threadIdx.x; c < NO && c < left; c += 256) {
        uint32_t d[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint32_t q = 4 * c + uint32_t(i), r = q / WPR, w = q - r * WPR;
            d[i] = lds[r * (STRIDE / 4) + w];
        }
        dst[c] = u32x4{d[0], d[1], d[2], d[3]};
    }
}

template <uint32_t REC, uint32_t STRIDE>
__global__ __launch_bounds__(256) void records_unpack(uint8_t *__restrict__ user, const uint8_t *__restrict__ packed,
                                                      uint64_t nrec)
{
    constexpr uint32_t R = 4096 / STRIDE, WPR = REC / 4, NV = R * REC / 16;
    __shared__ uint32_t lds[R * WPR];
    const uint64_t r0 = uint64_t(blockIdx.x) * R;
    const u32x4 *src = reinterpret_cast<const u32x4 *>(packed) + r0 * REC / 16;
    const uint64_t left = (nrec - r0) * REC / 16;
    for (uint32_t i = threadIdx.x; i < NV && i < left; i += 256)
        *reinterpret_cast<u32x4 *>(&lds[4 * i]) = __builtin_nontemporal_load(src + i);
    __syncthreads();
    for (uint32_t r = threadIdx.x; r < R && r0 + r < nrec; r += 256) {
        const uint32_t *l = &lds[r * WPR];
        uint32_t *d = reinterpret_cast<uint32_t *>(user + (r0 + r) * STRIDE);
        *reinterpret_cast<u32x4 *>(d) = u32x4{l[0], l[1], l[2], l[3]};
#pragma unroll
        for (uint32_t w = 4; w < WPR; ++w)
            d[w] = l[w];
    }
}

// 4-byte elements at an ascending element-index list (BASELINE config 4 in address order): the
// gather reads every touched line once, in address order, and writes a compact stream; the
// scatter is the masked partial-line write of every element (r2's ubench_masked "mask").
template <int DIR>
__global__ __launch_bounds__(256) void listed(uint8_t *__restrict__ user, uint8_t *__restrict__ packed,
                                              const uint32_t *__restrict__ idx, uint64_t n, int64_t base)
{
    const uint64_t p0 = uint64_t(blockIdx.x) * 256 * K + threadIdx.x;
    uint32_t j[K], v[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const uint64_t p = p0 + uint64_t(k) * 256;
        j[k] = p < n ? idx[p] : 0;
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const uint64_t p = p0 + uint64_t(k) * 256;
        if (p < n)
            v[k] = DIR == 0 ? *reinterpret_cast<const uint32_t *>(user + base + int64_t(j[k]) * 4)
                            : reinterpret_cast<const uint32_t *>(packed)[p];
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const uint64_t p = p0 + uint64_t(k) * 256;
        if (p >= n)
            continue;
        if (DIR == 0)
            reinterpret_cast<uint32_t *>(packed)[p] = v[k];
        else
            *reinterpret_cast<uint32_t *>(user + base + int64_t(j[k]) * 4) = v[k];
    }
}

}  // namespace

extern "C" {

// One part of a workload: kind 0 element gather/scatter (esize 4 or 8), kind 1 block copy
// (blen = 16 << lw bytes), kind 2 records (esize bytes at an s0-byte pitch: 20 at 32 only),
// kind 3 4-byte elements at the ascending element-index list `list` (n = count, not a power of
// two).  Kinds 0-2: positions n = 1 << (l0 + l1 + l2); user offset base + i0*s0 + i1*s1 + i2*s2.
// Packed bytes land at packed + poff.  `ubuf` / `pbuf` (device addresses, 0 = the run's buffers)
// redirect a part to scratch buffers: a pass of the engine over its own scratch (config 4's
// address-ordered U stream) that moves no user or packed bytes.
struct ddt_floor_part {
    int32_t kind, esize;
    uint32_t l0, l1, l2, lw;
    int64_t s0, s1, s2, base, poff;
    uint64_t list, count, ubuf, pbuf;
};

static void launch_part(void *user, void *packed, const ddt_floor_part &q, int dir, hipStream_t stream)
{
    Shape sh{q.s0, q.s1, q.s2, q.base, q.l0, q.l1, uint64_t(1) << (q.l0 + q.l1 + q.l2)};
    uint8_t *u = q.ubuf ? reinterpret_cast<uint8_t *>(q.ubuf) : static_cast<uint8_t *>(user);
    uint8_t *p = (q.pbuf ? reinterpret_cast<uint8_t *>(q.pbuf) : static_cast<uint8_t *>(packed)) + q.poff;
    if (q.kind == 2) {
        if (q.esize != 20 || q.s0 != 32)
            return;   // the one record shape measured (config 5)
        const uint64_t R = 4096 / 32;
        const dim3 grid(uint32_t((sh.n + R - 1) / R));
        if (dir)
            hipLaunchKernelGGL((records_unpack<20, 32>), grid, dim3(256), 0, stream, u + q.base, p, sh.n);
        else
            hipLaunchKernelGGL((records_pack<20, 32>), grid, dim3(256), 0, stream, u + q.base, p, sh.n);
        return;
    }
    if (q.kind == 3) {
        const dim3 grid(uint32_t((q.count + 256 * K - 1) / (256 * K)));
        const uint32_t *ix = reinterpret_cast<const uint32_t *>(q.list);
        if (dir)
            hipLaunchKernelGGL(listed<1>, grid, dim3(256), 0, stream, u, p, ix, q.count, q.base);
        else
            hipLaunchKernelGGL(listed<0>, grid, dim3(256), 0, stream, u, p, ix, q.count, q.base);
        return;
    }
    if (q.kind == 0) {
        const dim3 grid(uint32_t((sh.n + 256 * K - 1) / (256 * K)));
        if (q.esize == 4 && dir)
            hipLaunchKernelGGL(scatter<4>, grid, dim3(256), 0, stream, u, p, sh);
        else if (q.esize == 4)
            hipLaunchKernelGGL(gather<4>, grid, dim3(256), 0, stream, u, p, sh);
        else if (dir)
            hipLaunchKernelGGL(scatter<8>, grid, dim3(256), 0, stream, u, p, sh);
        else
            hipLaunchKernelGGL(gather<8>, grid, dim3(256), 0, stream, u, p, sh);
    } else {
        const dim3 grid(uint32_t(((sh.n << q.lw) + 1023) / 1024));
        if (dir)
            hipLaunchKernelGGL(copy_blocks<1>, grid, dim3(256), 0, stream, u, p, sh, q.lw);
        else
            hipLaunchKernelGGL(copy_blocks<0>, grid, dim3(256), 0, stream, u, p, sh, q.lw);
    }
}

// One launch of one part on `stream` (dir 0 pack, 1 unpack), for a caller that brackets it with
// its own events and cache flushes (bench.py's per-face protocol).  Returns a HIP error code.
int ddt_floor_launch(void *user, void *packed, const struct ddt_floor_part *part, int dir, void *stream)
{
    launch_part(user, packed, *part, dir, static_cast<hipStream_t>(stream));
    return int(hipGetLastError());
}

// Times `reps` rounds of the workload's pack (every part in order) then its unpack, each part
// bracketed by events on the null stream; out[2*i] / out[2*i+1] = median pack / unpack
// microseconds of part i.  Returns 0, or a HIP error code.
int ddt_floor_run(void *user, void *packed, const struct ddt_floor_part *parts, int nparts, int reps,
                  float *out)
{
    std::vector<hipEvent_t> ev(size_t(nparts) * 4 * size_t(reps + 2));
    for (auto &e : ev)
        if (hipEventCreate(&e) != hipSuccess)
            return int(hipGetLastError());
    auto launch = [&](const ddt_floor_part &q, int dir) { launch_part(user, packed, q, dir, nullptr); };
    const int rounds = reps + 2;   // two warm rounds
    for (int r = 0; r < rounds; ++r)
        for (int dir = 0; dir < 2; ++dir)
            for (int i = 0; i < nparts; ++i) {
                hipEvent_t *e = &ev[((size_t(r) * 2 + dir) * nparts + i) * 2];
                (void) hipEventRecord(e[0], nullptr);
                launch(parts[i], dir);
                (void) hipEventRecord(e[1], nullptr);
            }
    hipError_t err = hipDeviceSynchronize();
    if (err == hipSuccess) {
        for (int dir = 0; dir < 2; ++dir)
            for (int i = 0; i < nparts; ++i) {
                std::vector<float> t;
                for (int r = 2; r < rounds; ++r) {
                    hipEvent_t *e = &ev[((size_t(r) * 2 + dir) * nparts + i) * 2];
                    float ms = 0;
                    (void) hipEventElapsedTime(&ms, e[0], e[1]);
                    t.push_back(ms * 1e3f);
                }
                std::sort(t.begin(), t.end());
                out[2 * i + dir] = t[t.size() / 2];
            }
    }
    for (auto &e : ev)
        (void) hipEventDestroy(e);
    return int(err);
}

}  // extern "C"
