// ddt_sorted.hip -- address-ordered two-pass engine for large small-block index lists
// (MPI_Type_indexed / create_indexed_block / hindexed whose blocks are a few elements of
// 4, 8 or 16 bytes; BASELINE config 4: 64 Mi random floats out of a 1 GiB buffer).
//
// The direct list kernel (ddt_move.hip.h, run_list_uni) issues one memory request per
// element: a random 4-byte gather over a span far beyond the Infinity Cache runs at the
// memory-side request ceiling (~44 G requests/s, profiles/r1_ubench4_requests.log), and a
// random 4-byte scatter is a read-modify-write of a 32-byte sector (~27 G/s).  Here the
// user side is visited in ADDRESS order instead, so each 128-byte line is fetched (or
// written) once, and the permutation back to type-map order runs through LDS:
//
//   pack   pass 1 (one workgroup per chunk of CH address-ordered elements):
//            lds[SL[j]] = user[A[j]]        A = sorted element offsets, SL = LDS slot
//            U[ubase(c,k) + q] = lds[off(c,k) + q]   runs grouped by destination bucket
//          pass 2 (one workgroup per bucket of RG packed elements):
//            lds[upos[s]] = U[s];  packed[k*RG + t] = lds[t]
//   unpack is the same two passes reversed.
//
// The pack keeps U chunk-major by default (round 6, ddt_tune slayout): pass 1 streams its whole
// chunk image to U[c * (CH + skew)] and pass 2 reads the bucket's runs in place inside the images
// (k_pack1c / k_pack2c), so the pack's scattered accesses are reads; the unpack keeps the
// bucket-major U below (mirrored, its pass 2' would write the runs scattered).
//
// Bucket-major U: the (chunk, bucket) runs end to end (round 5; they were padded to whole
// 64-byte segments before: 43 % of U was padding at cfg4).  Neighbouring chunks' runs share
// segments, so pass 1 deals its chunks to the XCDs in contiguous slabs and both halves of a
// shared segment meet in one L2.  CH = RG = 128 KiB / element size, so the LDS image of a
// chunk or a bucket is 128 KiB (gfx950: 160 KiB per CU).  The plan (A, SL, run tables,
// upos) is built once on the device from the list's displacements: a bitmap of the
// touched elements gives each element its address rank by popcount, and a repeated element
// makes the list ineligible (the direct kernel then keeps type-map order).
//
// This replaces, for such lists, the per-block cbmemcpy loop of
// opal_pack_accelerator_simple / opal_unpack_accelerator_simple
// (opal_datatype_pack_accelerator.c:161-295, opal_datatype_unpack_accelerator.c:210-368),
// whose committed description for config 4 is 32 M DATA entries.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <stdexcept>
#include <string>

#include "ddt_sorted.h"
#include "ddt_pool.h"

namespace ddt {

namespace {

typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
template <int E> struct Elem;
template <> struct Elem<4> { using T = uint32_t; };
template <> struct Elem<8> { using T = u32x2; };
template <> struct Elem<16> { using T = u32x4; };

constexpr int PT = 1024;               // threads per pass workgroup (16 wave64)
constexpr int BT = 256;                // threads per build workgroup
constexpr uint32_t LDS_BYTES = 128u << 10;
// SEGB bytes of a run move per lane group (SEG lanes, SortedList::segb).  U runs are unpadded
// by default (ddt_tune("sseg") 1, round 5: cfg4 1399 -> 1362 us per step) or padded to whole
// SEGB segments (sseg 32 / 64 / 128): 64 B (round 1; 32 B: less padding, but cfg4 1461 -> 1512
// us) or 128 B (round 2: half the memory requests of the scattered run writes and reads, more
// padding).
constexpr uint32_t SEG_DEFAULT = 64;
constexpr uint16_t PAD = 0xFFFF;       // upos of a padding slot

// Access policy bits of one run (SortedList::run, ddt_tune("spol")):
constexpr uint32_t POL_USER_WT = 1;    // unpack 1': user-side stores written through L2 (sc1)
constexpr uint32_t POL_STREAM_NTS = 2; // stores of U and of the packed side non-temporal
constexpr uint32_t POL_STREAM_NTL = 4; // loads of A, SL, U, upos and the packed side non-temporal
constexpr uint32_t POL_USER_NTL = 8;   // pack 1: user-side loads non-temporal
// timing-only bits (wrong results; scripts/ab.py phase breakdowns): skip the user-side phase
// of pass 1 / 1' (the address-ordered gather or scatter), or its run phase (emit or load runs)
constexpr uint32_t POL_SKIP_USER = 16;
constexpr uint32_t POL_SKIP_RUNS = 32;
// set by run() for a plan built with sseg = 1 (the default): U runs end to end, no padding slots
constexpr uint32_t POL_UNPADDED = 64;
// pass 1 / 1': chunks dealt to the XCDs in contiguous slabs (workgroups are dealt round-robin
// over the 8 XCDs), so the runs of neighbouring chunks -- adjacent in U -- are written into one L2
constexpr uint32_t POL_XCD_SLAB = 128;
// pass 2 / 2' of 4-byte elements move four U slots per lane (one 16-byte U load or store, one
// 8-byte upos load; round 6) and the packed side as 16-byte words when it is 16-byte aligned
constexpr uint32_t POL_VEC2 = 256;
// timing only (wrong results): LDS writes of the permutations go to conflict-free addresses
// (pass 1: the element's own index, pass 2: its U slot), to price the bank conflicts
constexpr uint32_t POL_NOCONF = 512;
// chunk-major U for the pack (1024) / the unpack (2048) (r6): pass 1 / 1' stream the chunk image
// to / from U[c * CH ..], pass 2 / 2' move the bucket's runs from / to their places in the images;
// the scattered accesses are then the pack's reads and the unpack's writes of pass 2 / 2'
constexpr uint32_t POL_CMAJ_PACK = 1024;
constexpr uint32_t POL_CMAJ_UNPACK = 2048;
// pass 2 / 2' of a chunk-major direction: buckets dealt to the XCDs in slabs (neighbouring
// buckets' runs share lines in every chunk image; set by run(), r6 A/B: pack 546 -> 519 us,
// chunk-major unpack 920 -> 871 us)
constexpr uint32_t POL_P2_SLAB = 4096;
// bits 16..23: pass 1 / 1' start stagger (round 6 A/B): the first wave of workgroups (one per CU)
// sleeps ((blockIdx / 8) % 4) x this many s_sleep(127) periods, so the CUs' gather and emission
// phases do not run in lockstep
constexpr uint32_t POL_STAGGER_SHIFT = 16;

__device__ __forceinline__ void stagger(uint32_t pol)
{
    const uint32_t units = (pol >> POL_STAGGER_SHIFT) & 0xFFu;
    if (!units || blockIdx.x >= 256u)
        return;
    const uint32_t n = ((blockIdx.x >> 3) & 3u) * units;
    for (uint32_t i = 0; i < n; ++i)
        __builtin_amdgcn_s_sleep(127);
}

__device__ __forceinline__ uint32_t chunk_of(uint32_t b, uint32_t n, uint32_t pol)
{
    if (!(pol & POL_XCD_SLAB))
        return b;
    const uint32_t x = b & 7u, i = b >> 3, per = n >> 3, rem = n & 7u;
    return x * per + (x < rem ? x : rem) + i;   // a bijection on [0, n)
}

template <typename T> __device__ __forceinline__ T ldp(const T *p, bool nt)
{
    return nt ? __builtin_nontemporal_load(p) : *p;
}
template <typename T> __device__ __forceinline__ void stp(T *p, T v, bool nt)
{
    if (nt)
        __builtin_nontemporal_store(v, p);
    else
        *p = v;
}
__device__ __forceinline__ void st_sc1(uint32_t *p, uint32_t v)
{
    asm volatile("global_store_dword %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ void st_sc1(u32x2 *p, u32x2 v)
{
    asm volatile("global_store_dwordx2 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ void st_sc1(u32x4 *p, u32x4 v)
{
    asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
}

// Sorted element offsets as the pass kernels read them: 16-bit offsets within 64-element
// groups plus one 32-bit base per group when every group spans < 64 Ki elements (the
// build checks; 2.06 bytes per element instead of 4), else the plain 32-bit array.
struct AddrList {
    const uint32_t *A;
    const uint16_t *A16;
    const uint32_t *Abase;
};
__device__ __forceinline__ uint32_t addr_at(const AddrList &L, uint32_t j, bool nt)
{
    return L.A16 ? L.Abase[j >> 6] + uint32_t(ldp(&L.A16[j], nt)) : ldp(&L.A[j], nt);
}

#define HK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess)                                                                   \
            throw std::runtime_error(std::string("sorted list: ") + #x + ": " + hipGetErrorString(e_)); \
    } while (0)

// ------------------------------------------------------------------ plan build kernels
__global__ __launch_bounds__(BT) void k_bitmap(const int32_t *__restrict__ disp, uint32_t n, uint32_t shift,
                                               uint32_t *__restrict__ bm, uint32_t *__restrict__ dup)
{
    for (uint32_t i = blockIdx.x * BT + threadIdx.x; i < n; i += gridDim.x * BT) {
        const uint32_t a = uint32_t(disp[i]) >> shift;
        const uint32_t bit = 1u << (a & 31);
        const uint32_t old = atomicOr(&bm[a >> 5], bit);
        if (old & bit)
            atomicOr(dup, 1u);
    }
}

__global__ __launch_bounds__(BT) void k_popc(const uint32_t *__restrict__ bm, uint32_t w, uint32_t *__restrict__ pc)
{
    for (uint32_t i = blockIdx.x * BT + threadIdx.x; i < w; i += gridDim.x * BT)
        pc[i] = __popc(bm[i]);
}

__device__ __forceinline__ uint32_t rank_of(uint32_t a, const uint32_t *bm, const uint32_t *wpre)
{
    const uint32_t w = a >> 5, below = (1u << (a & 31)) - 1u;
    return wpre[w] + __popc(bm[w] & below);
}

// A[j] = a; count (chunk, bucket) and remember each block's rank inside its run
__global__ __launch_bounds__(BT) void k_rank(const int32_t *__restrict__ disp, uint32_t n, uint32_t shift,
                                             const uint32_t *__restrict__ bm, const uint32_t *__restrict__ wpre,
                                             uint32_t ch, uint32_t rg, uint32_t nb, uint32_t *__restrict__ A,
                                             uint32_t *__restrict__ cnt, uint16_t *__restrict__ rr)
{
    for (uint32_t i = blockIdx.x * BT + threadIdx.x; i < n; i += gridDim.x * BT) {
        const uint32_t a = uint32_t(disp[i]) >> shift;
        const uint32_t j = rank_of(a, bm, wpre);
        A[j] = a;
        const uint32_t c = j / ch, k = i / rg;
        rr[i] = uint16_t(atomicAdd(&cnt[size_t(c) * nb + k], 1u));
    }
}

// 16-bit form of A: offsets inside groups of 64 consecutive sorted elements; *maxspan gets
// the largest group span (the form is used only if it is < 64 Ki)
__global__ __launch_bounds__(BT) void k_compress(const uint32_t *__restrict__ A, uint32_t n,
                                                 uint16_t *__restrict__ A16, uint32_t *__restrict__ Abase,
                                                 uint32_t *__restrict__ maxspan)
{
    for (uint32_t j = blockIdx.x * BT + threadIdx.x; j < n; j += gridDim.x * BT) {
        const uint32_t g0 = j & ~63u, base = A[g0];
        const uint32_t d = A[j] - base;
        A16[j] = uint16_t(d);
        if (j == g0)
            Abase[j >> 6] = base;
        if (d > 0xFFFFu)
            atomicMax(maxspan, d);
    }
}

// per chunk: off(c,k) = exclusive prefix over k of cnt(c,k); padded counts transposed to
// bucket-major for the U layout scan
__global__ __launch_bounds__(BT) void k_chunk_tables(const uint32_t *__restrict__ cnt, uint32_t nc, uint32_t nb,
                                                     uint32_t seg, uint16_t *__restrict__ off16,
                                                     uint32_t *__restrict__ padT)
{
    __shared__ uint32_t part[BT];
    const uint32_t c = blockIdx.x;
    const uint32_t per = (nb + BT - 1) / BT;
    const uint32_t k0 = threadIdx.x * per, k1 = min(nb, k0 + per);
    uint32_t s = 0;
    for (uint32_t k = k0; k < k1; ++k)
        s += cnt[size_t(c) * nb + k];
    part[threadIdx.x] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t acc = 0;
        for (int t = 0; t < BT; ++t) {
            const uint32_t v = part[t];
            part[t] = acc;
            acc += v;
        }
    }
    __syncthreads();
    uint32_t o = part[threadIdx.x];
    for (uint32_t k = k0; k < k1; ++k) {
        const uint32_t v = cnt[size_t(c) * nb + k];
        off16[size_t(c) * nb + k] = uint16_t(o);
        padT[size_t(k) * nc + c] = (v + seg - 1) / seg * seg;
        o += v;
    }
}

// chunk-major copy of the bucket-major run bases, and the first slot of every bucket
__global__ __launch_bounds__(BT) void k_run_bases(const uint32_t *__restrict__ ubT, uint32_t nc, uint32_t nb,
                                                  uint32_t total, uint32_t skew, uint32_t *__restrict__ ub,
                                                  uint32_t *__restrict__ bstart)
{
    const size_t n = size_t(nc) * nb;
    for (size_t x = size_t(blockIdx.x) * BT + threadIdx.x; x < n; x += size_t(gridDim.x) * BT) {
        const uint32_t k = uint32_t(x / nc), c = uint32_t(x % nc);
        ub[size_t(c) * nb + k] = ubT[x] + k * skew;
        if (c == 0)
            bstart[k] = ubT[x] + k * skew;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0)
        bstart[nb] = total + nb * skew;
}

// bucket-major run tables of the chunk-major layout
__global__ __launch_bounds__(BT) void k_cmaj_tables(const uint16_t *__restrict__ off16, const uint32_t *__restrict__ ubT,
                                                    uint32_t nc, uint32_t nb, uint32_t cst, uint32_t *__restrict__ physT,
                                                    uint16_t *__restrict__ vrelT)
{
    const size_t n = size_t(nc) * nb;
    for (size_t x = size_t(blockIdx.x) * BT + threadIdx.x; x < n; x += size_t(gridDim.x) * BT) {
        const uint32_t k = uint32_t(x / nc), c = uint32_t(x % nc);
        physT[x] = c * cst + off16[size_t(c) * nb + k];
        vrelT[x] = uint16_t(ubT[x] - ubT[size_t(k) * nc]);
    }
}

__global__ __launch_bounds__(BT) void k_assign(const int32_t *__restrict__ disp, uint32_t n, uint32_t shift,
                                               const uint32_t *__restrict__ bm, const uint32_t *__restrict__ wpre,
                                               uint32_t ch, uint32_t rg, uint32_t nb, const uint16_t *__restrict__ rr,
                                               const uint16_t *__restrict__ off16, const uint32_t *__restrict__ ub,
                                               uint16_t *__restrict__ SL, uint16_t *__restrict__ upos)
{
    for (uint32_t i = blockIdx.x * BT + threadIdx.x; i < n; i += gridDim.x * BT) {
        const uint32_t a = uint32_t(disp[i]) >> shift;
        const uint32_t j = rank_of(a, bm, wpre);
        const uint32_t c = j / ch, k = i / rg;
        const size_t ck = size_t(c) * nb + k;
        SL[j] = uint16_t(off16[ck] + rr[i]);
        upos[ub[ck] + rr[i]] = uint16_t(i - k * rg);
    }
}

// ------------------------------------------------------------------ pass kernels
// The (chunk, bucket) run tables of a chunk are staged in LDS first (coalesced; off has a
// sentinel = the chunk's element count, so cnt(k) = off(k+1) - off(k)): the run loops then
// wait on no global load for their addresses.  MAXNB = 2*CH/SEG = 4096 for every element
// size (the sorted_plan size rule), so chunk image + tables = 155 KiB of the 160.
constexpr uint32_t MAXNB = 4096;

template <int NT>
__device__ __forceinline__ void stage_tables(const uint16_t *__restrict__ off16, const uint32_t *__restrict__ ub,
                                             uint32_t c, uint32_t nb, uint32_t m, uint16_t *toff, uint32_t *tub)
{
    for (uint32_t k = threadIdx.x; k < nb; k += NT) {
        toff[k] = off16[size_t(c) * nb + k];
        tub[k] = ub[size_t(c) * nb + k];
    }
    if (threadIdx.x == 0)
        toff[nb] = uint16_t(m);   // m <= CH <= 32 Ki
}

// pack pass 1, second phase: the chunk image's runs out to U, bucket by bucket
template <int E, int SEGB, int NT>
__device__ __forceinline__ void emit_runs(const typename Elem<E>::T *lds, const uint16_t *toff, const uint32_t *tub,
                                          uint8_t *__restrict__ U, uint32_t nb, bool nts, bool unpadded)
{
    using T = typename Elem<E>::T;
    constexpr uint32_t SEG = SEGB / E;
    T *dst = reinterpret_cast<T *>(U);
    const uint32_t sub = threadIdx.x / SEG, lane = threadIdx.x % SEG;
    for (uint32_t k = sub; k < nb; k += NT / SEG) {
        const uint32_t o = toff[k], cn = toff[k + 1] - o;
        const uint32_t b = tub[k], pn = unpadded ? cn : (cn + SEG - 1) / SEG * SEG;
        for (uint32_t q = lane; q < pn; q += SEG)
            stp(&dst[b + q], lds[o + q], nts);   // padding slots carry a neighbour's bytes: whole segments
    }
}

// pack pass 1: gather the chunk in address order into LDS, emit its runs bucket by bucket.
// CDIV = 2 (round 4, ddt_tune("schunk", 2)): half-size chunks (64 KiB images, buckets stay
// 128 KiB) in 512-thread workgroups, two per CU, so one chunk's gather overlaps another's run
// emission; needs nb <= MAXNB / 2.
template <int E, int SEGB, int K, int CDIV>
__global__ __launch_bounds__(PT / CDIV) void k_pack1(const uint8_t *__restrict__ user, const AddrList al,
                                                     const uint16_t *__restrict__ SL, const uint16_t *__restrict__ off16,
                                                     const uint32_t *__restrict__ ub, uint8_t *__restrict__ U, uint32_t n,
                                                     uint32_t nb, uint32_t pol)
{
    using T = typename Elem<E>::T;
    constexpr uint32_t NT = PT / CDIV;
    constexpr uint32_t CH = LDS_BYTES / E / CDIV, SEG = SEGB / E;
    const bool ntl = pol & POL_STREAM_NTL, nts = pol & POL_STREAM_NTS, ntu = pol & POL_USER_NTL;
    __shared__ T lds[CH + SEG];
    __shared__ uint16_t toff[MAXNB / CDIV + 1];
    __shared__ uint32_t tub[MAXNB / CDIV];
    stagger(pol);
    const uint32_t c = chunk_of(blockIdx.x, gridDim.x, pol), j0 = c * CH;
    const uint32_t m = min(CH, n - j0);
    stage_tables<NT>(off16, ub, c, nb, m, toff, tub);
    const T *src = reinterpret_cast<const T *>(user);
    const bool noconf = pol & POL_NOCONF;
    // K elements per thread in flight: each is a dependent pair (offset, then the user
    // element), so K sets how many of the chunk's CH / PT per thread share one latency
    const uint32_t mg = (pol & POL_SKIP_USER) ? 0u : m;
    for (uint32_t t0 = threadIdx.x; t0 < mg; t0 += NT * K) {
        T v[K];
        uint32_t s[K];
#pragma unroll
        for (int q = 0; q < K; ++q) {
            const uint32_t t = t0 + q * NT;
            if (t < m) {
                s[q] = ldp(&SL[j0 + t], ntl);
                v[q] = ldp(&src[addr_at(al, j0 + t, ntl)], ntu);
            }
        }
#pragma unroll
        for (int q = 0; q < K; ++q)
            if (t0 + q * NT < m)
                lds[noconf ? t0 + q * NT : s[q]] = v[q];
    }
    __syncthreads();
    emit_runs<E, SEGB, NT>(lds, toff, tub, U, (pol & POL_SKIP_RUNS) ? 0u : nb, nts, pol & POL_UNPADDED);
}

// pack pass 2: the bucket's runs scatter into LDS by destination, then stream out
template <int E, int K>
__global__ __launch_bounds__(PT) void k_pack2(const uint8_t *__restrict__ U, const uint16_t *__restrict__ upos,
                                              const uint32_t *__restrict__ bstart, uint8_t *__restrict__ packed,
                                              uint32_t n, uint32_t pol, uint32_t skew)
{
    using T = typename Elem<E>::T;
    constexpr uint32_t RG = LDS_BYTES / E;
    const bool ntl = pol & POL_STREAM_NTL, nts = pol & POL_STREAM_NTS;
    __shared__ T lds[RG];
    const uint32_t k = blockIdx.x;
    const uint32_t s0 = bstart[k], s1 = bstart[k + 1] - skew;
    const T *src = reinterpret_cast<const T *>(U);
    
    for (uint32_t x0 = s0 + threadIdx.x; x0 < s1; x0 += PT * K) {
        T v[K];
        uint32_t p[K];
#pragma unroll
        for (int q = 0; q < K; ++q) {
            const uint32_t x = x0 + q * PT;
            p[q] = PAD;
            if (x < s1) {
                p[q] = ldp(&upos[x], ntl);
                v[q] = ldp(&src[x], ntl);
            }
        }
#pragma unroll
        for (int q = 0; q < K; ++q)
            if (p[q] != PAD)
                lds[p[q]] = v[q];
    }
    __syncthreads();
    const uint32_t m = min(RG, n - k * RG);
    T *dst = reinterpret_cast<T *>(packed) + size_t(k) * RG;
    for (uint32_t t = threadIdx.x; t < m; t += PT)
        stp(&dst[t], lds[t], nts);
}

// unpack pass 2': the bucket's packed elements into LDS, then out to U in run order
template <int E, int K>
__global__ __launch_bounds__(PT) void k_unpack2(const uint8_t *__restrict__ packed, const uint16_t *__restrict__ upos,
                                                const uint32_t *__restrict__ bstart, uint8_t *__restrict__ U,
                                                uint32_t n, uint32_t pol, uint32_t skew)
{
    using T = typename Elem<E>::T;
    constexpr uint32_t RG = LDS_BYTES / E;
    const bool ntl = pol & POL_STREAM_NTL, nts = pol & POL_STREAM_NTS;
    __shared__ T lds[RG];
    const uint32_t k = blockIdx.x;
    const uint32_t m = min(RG, n - k * RG);
    const T *src = reinterpret_cast<const T *>(packed) + size_t(k) * RG;
    
    for (uint32_t t0 = threadIdx.x; t0 < m; t0 += PT * K) {
        T v[K];
#pragma unroll
        for (int q = 0; q < K; ++q)
            if (t0 + q * PT < m)
                v[q] = ldp(&src[t0 + q * PT], ntl);
#pragma unroll
        for (int q = 0; q < K; ++q)
            if (t0 + q * PT < m)
                lds[t0 + q * PT] = v[q];
    }
    __syncthreads();
    const uint32_t s0 = bstart[k], s1 = bstart[k + 1] - skew;
    T *dst = reinterpret_cast<T *>(U);
    for (uint32_t x0 = s0 + threadIdx.x; x0 < s1; x0 += PT * K) {
        uint32_t p[K];
#pragma unroll
        for (int q = 0; q < K; ++q)
            p[q] = x0 + q * PT < s1 ? uint32_t(ldp(&upos[x0 + q * PT], ntl)) : uint32_t(PAD);
#pragma unroll
        for (int q = 0; q < K; ++q) {
            if (x0 + q * PT < s1) {
                T v{};
                if (p[q] != PAD)
                    v = lds[p[q]];
                stp(&dst[x0 + q * PT], v, nts);   // padding slots written too: whole segments
            }
        }
    }
}


// pass 2 / 2' of 4-byte elements, four U slots per lane (POL_VEC2, round 6).  U and upos are
// read (or U written) as aligned quads of slots covering the bucket's [s0, s1); a quad shared
// with a neighbouring bucket is read whole and used in part, and written element by element.
// Allocation slack (dalloc: +16 bytes) covers the last quad's overrun.
typedef unsigned short u16x4 __attribute__((ext_vector_type(4)));

template <int K>
__global__ __launch_bounds__(PT) void k_pack2v(const uint8_t *__restrict__ U, const uint16_t *__restrict__ upos,
                                               const uint32_t *__restrict__ bstart, uint8_t *__restrict__ packed,
                                               uint32_t n, uint32_t pol, uint32_t skew)
{
    constexpr uint32_t RG = LDS_BYTES / 4;
    const bool ntl = pol & POL_STREAM_NTL, nts = pol & POL_STREAM_NTS, noconf = pol & POL_NOCONF;
    __shared__ uint32_t lds[RG];
    const uint32_t k = blockIdx.x;
    const uint32_t s0 = bstart[k], s1 = bstart[k + 1] - skew;
    const u32x4 *src = reinterpret_cast<const u32x4 *>(U);
    const u16x4 *up = reinterpret_cast<const u16x4 *>(upos);
    const uint32_t q0 = s0 >> 2, q1 = (s1 + 3) >> 2;
    for (uint32_t x0 = q0 + threadIdx.x; x0 < q1; x0 += PT * K) {
        u32x4 v[K];
        u16x4 p[K];
#pragma unroll
        for (int q = 0; q < K; ++q) {
            const uint32_t x = x0 + q * PT;
            if (x < q1) {
                p[q] = ldp(&up[x], ntl);
                v[q] = ldp(&src[x], ntl);
            }
        }
#pragma unroll
        for (int q = 0; q < K; ++q) {
            const uint32_t x = x0 + q * PT;
            if (x >= q1)
                continue;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const uint32_t slot = 4 * x + e;
                if (slot >= s0 && slot < s1 && p[q][e] != PAD)
                    lds[noconf ? (slot - s0) & (RG - 1) : p[q][e]] = v[q][e];
            }
        }
    }
    __syncthreads();
    const uint32_t m = min(RG, n - k * RG);
    uint8_t *dst8 = packed + size_t(k) * RG * 4;
    if ((reinterpret_cast<uintptr_t>(dst8) & 15) == 0) {
        u32x4 *dst = reinterpret_cast<u32x4 *>(dst8);
        const u32x4 *l4 = reinterpret_cast<const u32x4 *>(lds);
        for (uint32_t t = threadIdx.x; t < m / 4; t += PT)
            stp(&dst[t], l4[t], nts);
        for (uint32_t t = (m & ~3u) + threadIdx.x; t < m; t += PT)
            reinterpret_cast<uint32_t *>(dst8)[t] = lds[t];
    } else {
        uint32_t *dst = reinterpret_cast<uint32_t *>(dst8);
        for (uint32_t t = threadIdx.x; t < m; t += PT)
            stp(&dst[t], lds[t], nts);
    }
}

template <int K>
__global__ __launch_bounds__(PT) void k_unpack2v(const uint8_t *__restrict__ packed, const uint16_t *__restrict__ upos,
                                                 const uint32_t *__restrict__ bstart, uint8_t *__restrict__ U,
                                                 uint32_t n, uint32_t pol, uint32_t skew)
{
    constexpr uint32_t RG = LDS_BYTES / 4;
    const bool ntl = pol & POL_STREAM_NTL, nts = pol & POL_STREAM_NTS;
    __shared__ uint32_t lds[RG];
    const uint32_t k = blockIdx.x;
    const uint32_t m = min(RG, n - k * RG);
    const uint8_t *src8 = packed + size_t(k) * RG * 4;
    if ((reinterpret_cast<uintptr_t>(src8) & 15) == 0) {
        const u32x4 *src = reinterpret_cast<const u32x4 *>(src8);
        u32x4 *l4 = reinterpret_cast<u32x4 *>(lds);
        const uint32_t m4 = m / 4;
        for (uint32_t t0 = threadIdx.x; t0 < m4; t0 += PT * K) {
            u32x4 v[K];
#pragma unroll
            for (int q = 0; q < K; ++q)
                if (t0 + q * PT < m4)
                    v[q] = ldp(&src[t0 + q * PT], ntl);
#pragma unroll
            for (int q = 0; q < K; ++q)
                if (t0 + q * PT < m4)
                    l4[t0 + q * PT] = v[q];
        }
        for (uint32_t t = (m & ~3u) + threadIdx.x; t < m; t += PT)
            lds[t] = reinterpret_cast<const uint32_t *>(src8)[t];
    } else {
        const uint32_t *src = reinterpret_cast<const uint32_t *>(src8);
        for (uint32_t t = threadIdx.x; t < m; t += PT)
            lds[t] = ldp(&src[t], ntl);
    }
    __syncthreads();
    const uint32_t s0 = bstart[k], s1 = bstart[k + 1] - skew;
    const uint32_t q0 = s0 >> 2, q1 = (s1 + 3) >> 2;
    const u16x4 *up = reinterpret_cast<const u16x4 *>(upos);
    u32x4 *dst = reinterpret_cast<u32x4 *>(U);
    for (uint32_t x0 = q0 + threadIdx.x; x0 < q1; x0 += PT * K) {
        u16x4 p[K];
#pragma unroll
        for (int q = 0; q < K; ++q)
            if (x0 + q * PT < q1)
                p[q] = ldp(&up[x0 + q * PT], ntl);
#pragma unroll
        for (int q = 0; q < K; ++q) {
            const uint32_t x = x0 + q * PT;
            if (x >= q1)
                continue;
            u32x4 v;
#pragma unroll
            for (int e = 0; e < 4; ++e)
                v[e] = p[q][e] != PAD ? lds[p[q][e]] : 0u;   // padding slots written too: whole segments
            if (4 * x >= s0 && 4 * x + 4 <= s1) {
                stp(&dst[x], v, nts);
            } else {   // a quad shared with a neighbouring bucket: this bucket's slots only
                uint32_t *d1 = reinterpret_cast<uint32_t *>(U);
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    if (4 * x + e >= s0 && 4 * x + e < s1)
                        d1[4 * x + e] = v[e];
            }
        }
    }
}

// unpack pass 1', first phase: the chunk's runs from U into the LDS chunk image
template <int E, int SEGB, int NT>
__device__ __forceinline__ void load_runs(typename Elem<E>::T *lds, const uint16_t *toff, const uint32_t *tub,
                                          const uint8_t *__restrict__ U, uint32_t nb, bool ntl)
{
    using T = typename Elem<E>::T;
    constexpr uint32_t SEG = SEGB / E, NSUB = NT / SEG;
    const T *src = reinterpret_cast<const T *>(U);
    // B runs per round: their first NPF segments are loaded before any is stored (ILP: a run
    // averages 64 bytes, one 64-byte segment, so about half of them have a second; with 32-byte
    // segments the same bytes take up to four); the rare later segments follow
    constexpr int B = 8;
    constexpr int NPF = (SEGB == 32 && E <= 8) ? 4 : 2;
    const uint32_t sub = threadIdx.x / SEG, lane = threadIdx.x % SEG;
    for (uint32_t kb = sub; kb < nb; kb += NSUB * B) {
        T v[B][NPF];
        uint32_t o[B], cn[B], bb[B];
#pragma unroll
        for (int i = 0; i < B; ++i) {
            const uint32_t k = kb + uint32_t(i) * NSUB;
            cn[i] = 0;
            if (k < nb) {
                o[i] = toff[k];
                cn[i] = toff[k + 1] - o[i];
                bb[i] = tub[k];
#pragma unroll
                for (int f = 0; f < NPF; ++f)
                    if (lane + f * SEG < cn[i])
                        v[i][f] = ldp(&src[bb[i] + lane + f * SEG], ntl);
            }
        }
#pragma unroll
        for (int i = 0; i < B; ++i) {
#pragma unroll
            for (int f = 0; f < NPF; ++f)
                if (lane + f * SEG < cn[i])
                    lds[o[i] + lane + f * SEG] = v[i][f];
        }
#pragma unroll
        for (int i = 0; i < B; ++i)
            for (uint32_t q = lane + NPF * SEG; q < cn[i]; q += SEG)
                lds[o[i] + q] = src[bb[i] + q];
    }
}

// unpack pass 1': the chunk's runs into LDS, then scattered to the user side in address order
template <int E, int SEGB, int K, int CDIV>
__global__ __launch_bounds__(PT / CDIV) void k_unpack1(uint8_t *__restrict__ user, const AddrList al,
                                                       const uint16_t *__restrict__ SL, const uint16_t *__restrict__ off16,
                                                       const uint32_t *__restrict__ ub, const uint8_t *__restrict__ U,
                                                       uint32_t n, uint32_t nb, uint32_t pol)
{
    using T = typename Elem<E>::T;
    constexpr uint32_t NT = PT / CDIV;
    constexpr uint32_t CH = LDS_BYTES / E / CDIV;
    const bool ntl = pol & POL_STREAM_NTL, wt = pol & POL_USER_WT;
    __shared__ T lds[CH];
    __shared__ uint16_t toff[MAXNB / CDIV + 1];
    __shared__ uint32_t tub[MAXNB / CDIV];
    stagger(pol);
    const uint32_t c = chunk_of(blockIdx.x, gridDim.x, pol), j0 = c * CH;
    const uint32_t m = min(CH, n - j0);
    stage_tables<NT>(off16, ub, c, nb, m, toff, tub);
    __syncthreads();
    load_runs<E, SEGB, NT>(lds, toff, tub, U, (pol & POL_SKIP_RUNS) ? 0u : nb, ntl);
    __syncthreads();
    T *dst = reinterpret_cast<T *>(user);
    const uint32_t ms = (pol & POL_SKIP_USER) ? 0u : m;
    for (uint32_t t0 = threadIdx.x; t0 < ms; t0 += NT * K) {
        uint32_t a[K];
        T v[K];
#pragma unroll
        for (int q = 0; q < K; ++q) {
            const uint32_t t = t0 + q * NT;
            if (t < m) {
                a[q] = addr_at(al, j0 + t, ntl);
                v[q] = lds[ldp(&SL[j0 + t], ntl)];
            }
        }
#pragma unroll
        for (int q = 0; q < K; ++q)
            if (t0 + q * NT < m) {
                if (wt)
                    st_sc1(&dst[a[q]], v[q]);
                else
                    dst[a[q]] = v[q];
            }
    }
}


// ------------------------------------------------------------------ chunk-major U (r6)
constexpr uint32_t MAXNC = 4096;

// pass 1 of a chunk-major pack: the address-ordered gather into the LDS image, then the image
// out to U[c * cst ..] as one stream (cst = CH + the skew, a whole number of 16-byte quads)
template <int E, int K>
__global__ __launch_bounds__(PT) void k_pack1c(const uint8_t *__restrict__ user, const AddrList al,
                                               const uint16_t *__restrict__ SL, uint8_t *__restrict__ U, uint32_t n,
                                               uint32_t cst, uint32_t pol)
{
    using T = typename Elem<E>::T;
    constexpr uint32_t CH = LDS_BYTES / E;
    const bool ntl = pol & POL_STREAM_NTL, nts = pol & POL_STREAM_NTS, ntu = pol & POL_USER_NTL;
    __shared__ T lds[CH];
    const uint32_t c = blockIdx.x, j0 = c * CH;
    const uint32_t m = min(CH, n - j0);
    const T *src = reinterpret_cast<const T *>(user);
    const uint32_t mg = (pol & POL_SKIP_USER) ? 0u : m;
    for (uint32_t t0 = threadIdx.x; t0 < mg; t0 += PT * K) {
        T v[K];
        uint32_t s[K];
#pragma unroll
        for (int q = 0; q < K; ++q) {
            const uint32_t t = t0 + q * PT;
            if (t < m) {
                s[q] = ldp(&SL[j0 + t], ntl);
                v[q] = ldp(&src[addr_at(al, j0 + t, ntl)], ntu);
            }
        }
#pragma unroll
        for (int q = 0; q < K; ++q)
            if (t0 + q * PT < m)
                lds[(pol & POL_NOCONF) ? t0 + q * PT : s[q]] = v[q];
    }
    __syncthreads();
    if (pol & POL_SKIP_RUNS)
        return;
    // the image starts 16-byte aligned (c * cst * E): whole 16-byte words, then the tail
    const uint32_t mq = m * E / 16;
    u32x4 *dst = reinterpret_cast<u32x4 *>(U + size_t(c) * cst * E);
    const u32x4 *l4 = reinterpret_cast<const u32x4 *>(lds);
    for (uint32_t t = threadIdx.x; t < mq; t += PT)
        stp(&dst[t], l4[t], nts);
    T *dt = reinterpret_cast<T *>(U) + size_t(c) * cst;
    for (uint32_t t = mq * 16 / E + threadIdx.x; t < m; t += PT)
        dt[t] = lds[t];
}

// unpack pass 1' of the chunk-major layout: the image in from U[c * cst ..] as one stream, then
// scattered to the user side in address order
template <int E, int K>
__global__ __launch_bounds__(PT) void k_unpack1c(uint8_t *__restrict__ user, const AddrList al,
                                                 const uint16_t *__restrict__ SL, const uint8_t *__restrict__ U,
                                                 uint32_t n, uint32_t cst, uint32_t pol)
{
    using T = typename Elem<E>::T;
    constexpr uint32_t CH = LDS_BYTES / E;
    const bool ntl = pol & POL_STREAM_NTL, wt = pol & POL_USER_WT;
    __shared__ T lds[CH];
    const uint32_t c = blockIdx.x, j0 = c * CH;
    const uint32_t m = min(CH, n - j0);
    if (!(pol & POL_SKIP_RUNS)) {
        const uint32_t mq = m * E / 16;
        const u32x4 *src = reinterpret_cast<const u32x4 *>(U + size_t(c) * cst * E);
        u32x4 *l4 = reinterpret_cast<u32x4 *>(lds);
        for (uint32_t t0 = threadIdx.x; t0 < mq; t0 += PT * 8) {
            u32x4 v[8];
#pragma unroll
            for (int q = 0; q < 8; ++q)
                if (t0 + q * PT < mq)
                    v[q] = ldp(&src[t0 + q * PT], ntl);
#pragma unroll
            for (int q = 0; q < 8; ++q)
                if (t0 + q * PT < mq)
                    l4[t0 + q * PT] = v[q];
        }
        const T *st = reinterpret_cast<const T *>(U) + size_t(c) * cst;
        for (uint32_t t = mq * 16 / E + threadIdx.x; t < m; t += PT)
            lds[t] = st[t];
    }
    __syncthreads();
    T *dst = reinterpret_cast<T *>(user);
    const uint32_t ms = (pol & POL_SKIP_USER) ? 0u : m;
    for (uint32_t t0 = threadIdx.x; t0 < ms; t0 += PT * K) {
        uint32_t a[K];
        T v[K];
#pragma unroll
        for (int q = 0; q < K; ++q) {
            const uint32_t t = t0 + q * PT;
            if (t < m) {
                a[q] = addr_at(al, j0 + t, ntl);
                v[q] = lds[ldp(&SL[j0 + t], ntl)];
            }
        }
#pragma unroll
        for (int q = 0; q < K; ++q)
            if (t0 + q * PT < m) {
                if (wt)
                    st_sc1(&dst[a[q]], v[q]);
                else
                    dst[a[q]] = v[q];
            }
    }
}

// the bucket's run table (U element offset, first slot inside the bucket) staged in LDS
__device__ __forceinline__ void stage_cmaj(const uint32_t *__restrict__ physT, const uint16_t *__restrict__ vrelT,
                                           uint32_t k, uint32_t nc, uint32_t m, uint32_t *tph, uint16_t *tv)
{
    for (uint32_t c = threadIdx.x; c < nc; c += PT) {
        tph[c] = physT[size_t(k) * nc + c];
        tv[c] = vrelT[size_t(k) * nc + c];
    }
    if (threadIdx.x == 0)
        tv[nc] = uint16_t(m);   // m <= RG <= 32 Ki
}

// pack pass 2 of the chunk-major layout: the bucket's runs from the chunk images into LDS by
// destination (SEG lanes per run, B runs per round in flight), then streamed out
template <int E, int B, int NPF>
__global__ __launch_bounds__(PT) void k_pack2c(const uint8_t *__restrict__ U, const uint16_t *__restrict__ upos,
                                               const uint32_t *__restrict__ bstart, const uint32_t *__restrict__ physT,
                                               const uint16_t *__restrict__ vrelT, uint8_t *__restrict__ packed,
                                               uint32_t n, uint32_t nc, uint32_t pol)
{
    using T = typename Elem<E>::T;
    constexpr uint32_t RG = LDS_BYTES / E, SEG = 64 / E, NSUB = PT / SEG;
    const bool ntl = pol & POL_STREAM_NTL, nts = pol & POL_STREAM_NTS;
    __shared__ T lds[RG];
    __shared__ uint32_t tph[MAXNC];
    __shared__ uint16_t tv[MAXNC + 1];
    const uint32_t k = chunk_of(blockIdx.x, gridDim.x, (pol & POL_P2_SLAB) ? POL_XCD_SLAB : 0u);
    const uint32_t m = min(RG, n - k * RG);
    stage_cmaj(physT, vrelT, k, nc, m, tph, tv);
    __syncthreads();
    const T *src = reinterpret_cast<const T *>(U);
    const uint16_t *up = upos + bstart[k];
    const uint32_t sub = threadIdx.x / SEG, lane = threadIdx.x % SEG;
    const uint32_t ncr = (pol & POL_SKIP_RUNS) ? 0u : nc;
    for (uint32_t cb = sub; cb < ncr; cb += NSUB * B) {
        T v[B][NPF];
        uint16_t p[B][NPF];
        uint32_t o[B], cn[B], ph[B];
#pragma unroll
        for (int i = 0; i < B; ++i) {
            const uint32_t c = cb + uint32_t(i) * NSUB;
            cn[i] = 0;
            if (c < nc) {
                o[i] = tv[c];
                cn[i] = tv[c + 1] - o[i];
                ph[i] = tph[c];
#pragma unroll
                for (int f = 0; f < NPF; ++f)
                    if (lane + f * SEG < cn[i]) {
                        v[i][f] = ldp(&src[ph[i] + lane + f * SEG], ntl);
                        p[i][f] = ldp(&up[o[i] + lane + f * SEG], ntl);
                    }
            }
        }
#pragma unroll
        for (int i = 0; i < B; ++i) {
#pragma unroll
            for (int f = 0; f < NPF; ++f)
                if (lane + f * SEG < cn[i])
                    lds[p[i][f]] = v[i][f];
        }
#pragma unroll
        for (int i = 0; i < B; ++i)
            for (uint32_t q = lane + NPF * SEG; q < cn[i]; q += SEG)
                lds[up[o[i] + q]] = src[ph[i] + q];
    }
    __syncthreads();
    uint8_t *dst8 = packed + size_t(k) * RG * E;
    if ((reinterpret_cast<uintptr_t>(dst8) & 15) == 0) {
        u32x4 *dst = reinterpret_cast<u32x4 *>(dst8);
        const u32x4 *l4 = reinterpret_cast<const u32x4 *>(lds);
        const uint32_t mq = m * E / 16;
        for (uint32_t t = threadIdx.x; t < mq; t += PT)
            stp(&dst[t], l4[t], nts);
        for (uint32_t t = mq * 16 / E + threadIdx.x; t < m; t += PT)
            reinterpret_cast<T *>(dst8)[t] = lds[t];
    } else {
        T *dst = reinterpret_cast<T *>(dst8);
        for (uint32_t t = threadIdx.x; t < m; t += PT)
            stp(&dst[t], lds[t], nts);
    }
}

// unpack pass 2' of the chunk-major layout: the bucket's packed elements into LDS, then out to
// their runs' places in the chunk images
template <int E>
__global__ __launch_bounds__(PT) void k_unpack2c(const uint8_t *__restrict__ packed, const uint16_t *__restrict__ upos,
                                                 const uint32_t *__restrict__ bstart, const uint32_t *__restrict__ physT,
                                                 const uint16_t *__restrict__ vrelT, uint8_t *__restrict__ U,
                                                 uint32_t n, uint32_t nc, uint32_t pol)
{
    using T = typename Elem<E>::T;
    constexpr uint32_t RG = LDS_BYTES / E, SEG = 64 / E, NSUB = PT / SEG;
    constexpr int B = 8;
    const bool ntl = pol & POL_STREAM_NTL, nts = pol & POL_STREAM_NTS;
    __shared__ T lds[RG];
    __shared__ uint32_t tph[MAXNC];
    __shared__ uint16_t tv[MAXNC + 1];
    const uint32_t k = chunk_of(blockIdx.x, gridDim.x, (pol & POL_P2_SLAB) ? POL_XCD_SLAB : 0u);
    const uint32_t m = min(RG, n - k * RG);
    stage_cmaj(physT, vrelT, k, nc, m, tph, tv);
    const uint8_t *src8 = packed + size_t(k) * RG * E;
    if ((reinterpret_cast<uintptr_t>(src8) & 15) == 0) {
        const u32x4 *src = reinterpret_cast<const u32x4 *>(src8);
        u32x4 *l4 = reinterpret_cast<u32x4 *>(lds);
        const uint32_t mq = m * E / 16;
        for (uint32_t t0 = threadIdx.x; t0 < mq; t0 += PT * 2) {
            u32x4 v[2];
#pragma unroll
            for (int q = 0; q < 2; ++q)
                if (t0 + q * PT < mq)
                    v[q] = ldp(&src[t0 + q * PT], ntl);
#pragma unroll
            for (int q = 0; q < 2; ++q)
                if (t0 + q * PT < mq)
                    l4[t0 + q * PT] = v[q];
        }
        for (uint32_t t = mq * 16 / E + threadIdx.x; t < m; t += PT)
            lds[t] = reinterpret_cast<const T *>(src8)[t];
    } else {
        const T *src = reinterpret_cast<const T *>(src8);
        for (uint32_t t = threadIdx.x; t < m; t += PT)
            lds[t] = ldp(&src[t], ntl);
    }
    __syncthreads();
    T *dst = reinterpret_cast<T *>(U);
    const uint16_t *up = upos + bstart[k];
    const uint32_t sub = threadIdx.x / SEG, lane = threadIdx.x % SEG;
    const uint32_t ncr = (pol & POL_SKIP_RUNS) ? 0u : nc;
    for (uint32_t cb = sub; cb < ncr; cb += NSUB * B) {
        uint16_t p[B];
        uint32_t o[B], cn[B];
#pragma unroll
        for (int i = 0; i < B; ++i) {
            const uint32_t c = cb + uint32_t(i) * NSUB;
            cn[i] = 0;
            if (c < nc) {
                o[i] = tv[c];
                cn[i] = tv[c + 1] - o[i];
                if (lane < cn[i])
                    p[i] = ldp(&up[o[i] + lane], ntl);
            }
        }
#pragma unroll
        for (int i = 0; i < B; ++i) {
            const uint32_t c = cb + uint32_t(i) * NSUB;
            if (lane < cn[i])
                stp(&dst[tph[c] + lane], lds[p[i]], nts);
            for (uint32_t q = lane + SEG; q < cn[i]; q += SEG)
                stp(&dst[tph[c] + q], lds[up[o[i] + q]], nts);
        }
    }
}

// pass 2 with 4 elements per thread in flight; pass 2' with k2 (4, 8 or 16; E * k2 <= 64
// bytes).  cfg4 A/B (profiles/r2_ab_sorted_pass2_unroll.log): unpack 780 -> 751 us at 8 or 16,
// pack 575 -> 587 us, so only the unpack side takes the knob.
template <int E, int DIR>
void launch_pass2(dim3 gb, dim3 blk, hipStream_t stream, const uint8_t *src, const uint16_t *upos,
                  const uint32_t *bstart, uint8_t *dst, uint32_t n, uint32_t pol, uint32_t k2, uint32_t skew)
{
    constexpr int K16 = E == 4 ? 16 : 4, K8 = E <= 8 ? 8 : 4;
    if (E == 4 && (pol & POL_VEC2)) {   // K quads (4 K slots) per lane in flight
        if (DIR == 0)
            hipLaunchKernelGGL((k_pack2v<2>), gb, blk, 0, stream, src, upos, bstart, dst, n, pol, skew);
        else if (k2 >= 16)
            hipLaunchKernelGGL((k_unpack2v<4>), gb, blk, 0, stream, src, upos, bstart, dst, n, pol, skew);
        else if (k2 >= 8)
            hipLaunchKernelGGL((k_unpack2v<2>), gb, blk, 0, stream, src, upos, bstart, dst, n, pol, skew);
        else
            hipLaunchKernelGGL((k_unpack2v<1>), gb, blk, 0, stream, src, upos, bstart, dst, n, pol, skew);
        return;
    }
    if (DIR == 0) {
        hipLaunchKernelGGL((k_pack2<E, 4>), gb, blk, 0, stream, src, upos, bstart, dst, n, pol, skew);
    } else {
        if (k2 >= 16) hipLaunchKernelGGL((k_unpack2<E, K16>), gb, blk, 0, stream, src, upos, bstart, dst, n, pol, skew);
        else if (k2 >= 8) hipLaunchKernelGGL((k_unpack2<E, K8>), gb, blk, 0, stream, src, upos, bstart, dst, n, pol, skew);
        else hipLaunchKernelGGL((k_unpack2<E, 4>), gb, blk, 0, stream, src, upos, bstart, dst, n, pol, skew);
    }
}

uint32_t grid_for(uint64_t n, uint32_t threads)
{
    uint64_t b = (n + threads - 1) / threads;
    return uint32_t(b < 1 ? 1 : (b > 65536 ? 65536 : b));
}

template <typename T>
T *dalloc(size_t n, uint64_t &bytes)
{
    void *p = pool_alloc(n * sizeof(T) + 16);
    if (!p)
        throw std::runtime_error("sorted list: out of device memory");
    bytes += n * sizeof(T);
    return static_cast<T *>(p);
}

}  // namespace

void SortedList::take_blocks(std::vector<void *> &out)
{
    for (void **p : {(void **) &A, (void **) &A16, (void **) &Abase, (void **) &SL, (void **) &off16,
                     (void **) &ub, (void **) &bstart, (void **) &upos, (void **) &physT, (void **) &vrelT, &U})
        if (*p) {
            out.push_back(*p);
            *p = nullptr;
        }
}

SortedList::~SortedList()
{
    std::vector<void *> left;
    take_blocks(left);
    if (!left.empty() && done)
        (void) hipEventSynchronize(done);   // only a plan that was never released to the pool
    for (void *p : left)
        pool_free(p);
    if (done)
        (void) hipEventDestroy(done);
}

// Build the plan on `stream` from the device displacement list (int32, relative to the
// list's minimum displacement, every value a multiple of esz).  Returns false (and leaves
// nothing allocated) when the displacements repeat.
bool SortedList::build(const int32_t *disp, uint32_t n_, uint32_t esz_, uint64_t span_elems, uint32_t segb_,
                       hipStream_t stream, uint32_t cdiv_, uint32_t skew_bytes)
{
    n = n_;
    esz = esz_;
    segb = (segb_ == 128 || segb_ == 32) ? segb_ : SEG_DEFAULT;
    unpadded = segb_ == 1;
    rg = LDS_BYTES / esz;
    nb = (n + rg - 1) / rg;
    cdiv = (cdiv_ == 2 && nb <= MAXNB / 2) ? 2 : 1;   // half chunks: the tables must fit half the LDS
    ch = rg / cdiv;
    seg = unpadded ? 1 : segb / esz;
    nc = (n + ch - 1) / ch;
    uint32_t shift = 0;
    while ((1u << shift) < esz)
        ++shift;
    const uint64_t words = (span_elems + 31) / 32 + 1;
    const size_t runs = size_t(nc) * nb;
    uint64_t tmp_bytes = 0;
    uint32_t *bm = nullptr, *wpre = nullptr, *dup = nullptr, *cnt = nullptr, *padT = nullptr, *ubT = nullptr;
    uint16_t *rr = nullptr;
    void *scan_tmp = nullptr;
    auto release = [&] {   // the build's stream has been drained before every call
        for (void *p : {(void *) bm, (void *) wpre, (void *) dup, (void *) cnt, (void *) padT, (void *) ubT,
                        (void *) rr, scan_tmp})
            pool_free(p);
    };
    try {
        bm = dalloc<uint32_t>(words, tmp_bytes);
        wpre = dalloc<uint32_t>(words, tmp_bytes);
        dup = dalloc<uint32_t>(1, tmp_bytes);
        cnt = dalloc<uint32_t>(runs, tmp_bytes);
        padT = dalloc<uint32_t>(runs + 1, tmp_bytes);
        ubT = dalloc<uint32_t>(runs + 1, tmp_bytes);
        rr = dalloc<uint16_t>(n, tmp_bytes);
        HK(hipMemsetAsync(bm, 0, words * 4, stream));
        HK(hipMemsetAsync(dup, 0, 4, stream));
        HK(hipMemsetAsync(cnt, 0, runs * 4, stream));
        hipLaunchKernelGGL(k_bitmap, dim3(grid_for(n, BT)), dim3(BT), 0, stream, disp, n, shift, bm, dup);
        hipLaunchKernelGGL(k_popc, dim3(grid_for(words, BT)), dim3(BT), 0, stream, bm, uint32_t(words), wpre);
        size_t tb = 0, tb2 = 0;
        HK(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, wpre, wpre, int(words), stream));
        HK(hipcub::DeviceScan::ExclusiveSum(nullptr, tb2, padT, ubT, int(runs + 1), stream));
        if (!(scan_tmp = pool_alloc(std::max(tb, tb2) + 16)))
            throw std::runtime_error("sorted list: out of device memory");
        HK(hipcub::DeviceScan::ExclusiveSum(scan_tmp, tb, wpre, wpre, int(words), stream));
        uint32_t hdup = 0;
        HK(hipMemcpyAsync(&hdup, dup, 4, hipMemcpyDeviceToHost, stream));
        HK(hipStreamSynchronize(stream));
        if (hdup) {
            release();
            return false;
        }
        uint64_t bytes = 0;
        A = dalloc<uint32_t>(n, bytes);
        SL = dalloc<uint16_t>(n, bytes);
        off16 = dalloc<uint16_t>(runs, bytes);
        ub = dalloc<uint32_t>(runs, bytes);
        bstart = dalloc<uint32_t>(nb + 1, bytes);
        hipLaunchKernelGGL(k_rank, dim3(grid_for(n, BT)), dim3(BT), 0, stream, disp, n, shift, bm, wpre, ch, rg,
                           nb, A, cnt, rr);
        {   // the 16-bit form of A, kept when every 64-element group spans < 64 Ki elements
            uint64_t cb = 0;
            A16 = dalloc<uint16_t>(n, cb);
            Abase = dalloc<uint32_t>((n + 63) / 64, cb);
            HK(hipMemsetAsync(dup, 0, 4, stream));
            hipLaunchKernelGGL(k_compress, dim3(grid_for(n, BT)), dim3(BT), 0, stream, A, n, A16, Abase, dup);
            uint32_t span = 0;
            HK(hipMemcpyAsync(&span, dup, 4, hipMemcpyDeviceToHost, stream));
            HK(hipStreamSynchronize(stream));
            if (span == 0) {   // every d <= 0xFFFF
                pool_free(A);
                A = nullptr;
                bytes += cb - uint64_t(n) * 4;
            } else {
                pool_free(A16);
                pool_free(Abase);
                A16 = nullptr;
                Abase = nullptr;
            }
        }
        HK(hipMemsetAsync(padT + runs, 0, 4, stream));
        hipLaunchKernelGGL(k_chunk_tables, dim3(nc), dim3(BT), 0, stream, cnt, nc, nb, seg, off16, padT);
        HK(hipcub::DeviceScan::ExclusiveSum(scan_tmp, tb2, padT, ubT, int(runs + 1), stream));
        uint32_t total = 0;
        HK(hipMemcpyAsync(&total, ubT + runs, 4, hipMemcpyDeviceToHost, stream));
        HK(hipStreamSynchronize(stream));
        // bucket skew: whole 16-byte quads of slots (the pass-2 quads stay aligned), and the
        // 32-bit slot indices must still hold every slot
        skew = (skew_bytes / esz + 3u) & ~3u;
        if (uint64_t(total) + uint64_t(nb) * skew >= (1ull << 32))
            skew = 0;
        slots = uint64_t(total) + uint64_t(nb) * skew;
        hipLaunchKernelGGL(k_run_bases, dim3(grid_for(runs, BT)), dim3(BT), 0, stream, ubT, nc, nb, total, skew, ub,
                           bstart);
        uint64_t uslots = slots;
        cst = ch;
        if (unpadded && cdiv == 1 && nc <= MAXNC) {   // the chunk-major layout's run tables
            // chunk images `skew` slots apart too (a bucket's runs sit one per image)
            if (uint64_t(nc) * (ch + skew) < (1ull << 32))
                cst = ch + skew;
            uslots = std::max<uint64_t>(uslots, uint64_t(nc) * cst);
            physT = dalloc<uint32_t>(runs, bytes);
            vrelT = dalloc<uint16_t>(runs, bytes);
            hipLaunchKernelGGL(k_cmaj_tables, dim3(grid_for(runs, BT)), dim3(BT), 0, stream, off16, ubT, nc, nb, cst,
                               physT, vrelT);
        }
        upos = dalloc<uint16_t>(slots, bytes);
        U = dalloc<uint8_t>(size_t(uslots) * esz, bytes);
        HK(hipMemsetAsync(upos, 0xFF, size_t(slots) * 2, stream));
        hipLaunchKernelGGL(k_assign, dim3(grid_for(n, BT)), dim3(BT), 0, stream, disp, n, shift, bm, wpre, ch, rg,
                           nb, rr, off16, ub, SL, upos);
        HK(hipGetLastError());
        HK(hipEventCreateWithFlags(&done, hipEventDisableTiming));
        HK(hipStreamSynchronize(stream));
        dev_bytes = bytes;
    } catch (...) {
        (void) hipStreamSynchronize(stream);   // queued build kernels may still use the temporaries
        release();
        std::vector<void *> mine;
        take_blocks(mine);
        for (void *p : mine)
            pool_free(p);
        throw;
    }
    release();
    return true;
}

// One whole-list pack (dir 0) or unpack (dir 1) of one instance.  `user` points at the
// list's first element (minimum displacement), `packed` at the instance's packed bytes.
// `unroll`: elements per thread in flight in pack 1's address-ordered gather (4, 8, 16).  cfg4
// A/B (profiles/r2_ab_sorted_unroll.log): pack 656 / 617 / 612 us; unpack 1' keeps 4 (its
// scatter has one dependent load per element; 8 and 16 measured slower, 804 -> 818 / 842 us).
hipError_t SortedList::run(uint8_t *user, uint8_t *packed, int dir, uint32_t pol, hipStream_t stream,
                           uint32_t unroll, uint32_t k2)
{
    // U is one scratch per plan: a launch on another stream waits for the last one
    std::lock_guard<std::mutex> g(mu);
    if (used && last_stream != stream) {
        hipError_t e = hipStreamWaitEvent(stream, done, 0);
        if (e != hipSuccess)
            return e;
    }
    const dim3 gc(nc), gb(nb), blk(PT), blk1(PT / cdiv);
    const AddrList al{A, A16, Abase};
    uint8_t *u8 = static_cast<uint8_t *>(U);
    if (unpadded)   // r5 A/B (profiles/r5_ab_cfg4_unpadded.jsonl): the slabs pay only without padding
        pol |= POL_UNPADDED | POL_XCD_SLAB;
    if (physT && (pol & (dir == 0 ? POL_CMAJ_PACK : POL_CMAJ_UNPACK))) {   // chunk-major U (r6)
        pol |= POL_P2_SLAB;
#define DDT_CMAJ(E, K)                                                                                          \
    if (dir == 0) {                                                                                             \
        hipLaunchKernelGGL((k_pack1c<E, K>), gc, blk, 0, stream, user, al, SL, u8, n, cst, pol);                      \
        hipLaunchKernelGGL((k_pack2c<E, 8, 2>), gb, blk, 0, stream, u8, upos, bstart, physT, vrelT, packed, n, nc, pol); \
    } else {                                                                                                    \
        hipLaunchKernelGGL((k_unpack2c<E>), gb, blk, 0, stream, packed, upos, bstart, physT, vrelT, u8, n, nc, pol); \
        hipLaunchKernelGGL((k_unpack1c<E, 4>), gc, blk, 0, stream, user, al, SL, u8, n, cst, pol);                    \
    }
        if (esz == 4) {
            if (unroll >= 32) { DDT_CMAJ(4, 32) } else if (unroll >= 16) { DDT_CMAJ(4, 16) } else if (unroll >= 8) { DDT_CMAJ(4, 8) } else { DDT_CMAJ(4, 4) }
        } else if (esz == 8) {
            if (unroll >= 8) { DDT_CMAJ(8, 8) } else { DDT_CMAJ(8, 4) }
        } else {
            DDT_CMAJ(16, 4)
        }
#undef DDT_CMAJ
        hipError_t e = hipGetLastError();
        if (e != hipSuccess)
            return e;
        used = true;
        last_stream = stream;
        return hipEventRecord(done, stream);
    }
#define DDT_SORTED_PASS1(E, SB, K, CD)                                                                          \
    if (dir == 0)                                                                                               \
        hipLaunchKernelGGL((k_pack1<E, SB, K, CD>), gc, blk1, 0, stream, user, al, SL, off16, ub, u8, n, nb, pol); \
    else                                                                                                        \
        hipLaunchKernelGGL((k_unpack1<E, SB, 4, CD>), gc, blk1, 0, stream, user, al, SL, off16, ub, u8, n, nb, pol);
#define DDT_SORTED_LAUNCH_K(E, SB, K)                                                                           \
    if (dir == 0) {                                                                                             \
        if (cdiv == 2) { DDT_SORTED_PASS1(E, SB, K, 2) } else { DDT_SORTED_PASS1(E, SB, K, 1) }                 \
        launch_pass2<E, 0>(gb, blk, stream, u8, upos, bstart, packed, n, pol, k2, skew);                             \
    } else {                                                                                                    \
        launch_pass2<E, 1>(gb, blk, stream, packed, upos, bstart, u8, n, pol, k2, skew);                             \
        if (cdiv == 2) { DDT_SORTED_PASS1(E, SB, K, 2) } else { DDT_SORTED_PASS1(E, SB, K, 1) }                 \
    }
// K * E <= 64 bytes of elements per thread in flight: wider elements at K = 16 (or 16-byte
// ones at 8) exceed the 128 VGPRs of a 1024-thread workgroup and spill
#define DDT_SORTED_LAUNCH(E, SB)                                                                                \
    if (unroll >= 16 && E == 4) {                                                                               \
        DDT_SORTED_LAUNCH_K(E, SB, (E == 4 ? 16 : 4))                                                           \
    } else if (unroll >= 8 && E <= 8) {                                                                         \
        DDT_SORTED_LAUNCH_K(E, SB, (E <= 8 ? 8 : 4))                                                            \
    } else {                                                                                                    \
        DDT_SORTED_LAUNCH_K(E, SB, 4)                                                                           \
    }
    if (segb == 128) {
        if (esz == 4) {
            DDT_SORTED_LAUNCH(4, 128)
        } else if (esz == 8) {
            DDT_SORTED_LAUNCH(8, 128)
        } else {
            DDT_SORTED_LAUNCH(16, 128)
        }
    } else if (segb == 32) {
        if (esz == 4) {
            DDT_SORTED_LAUNCH(4, 32)
        } else if (esz == 8) {
            DDT_SORTED_LAUNCH(8, 32)
        } else {
            DDT_SORTED_LAUNCH(16, 32)
        }
    } else {
        if (esz == 4) {
            DDT_SORTED_LAUNCH(4, 64)
        } else if (esz == 8) {
            DDT_SORTED_LAUNCH(8, 64)
        } else {
            DDT_SORTED_LAUNCH(16, 64)
        }
    }
#undef DDT_SORTED_LAUNCH
#undef DDT_SORTED_LAUNCH_K
#undef DDT_SORTED_PASS1
    hipError_t e = hipGetLastError();
    if (e != hipSuccess)
        return e;
    used = true;
    last_stream = stream;
    return hipEventRecord(done, stream);
}

}  // namespace ddt
