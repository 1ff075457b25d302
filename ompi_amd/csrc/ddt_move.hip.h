// ddt_move.hip.h -- the move kernel (ddt_move_kernel / ddt_move_inline_kernel) and its
// device helpers, shared by the four translation units that instantiate it, one per
// (direction, index lists) pair (ddt_move_{p,u}{0,1}.hip), so the build compiles them in
// parallel.  Internal to libddt_hip.so; see ddt_kernels.hip for the design notes.
#pragma once

#include <cstdlib>

#include <hip/hip_runtime.h>

#include "ddt_device.h"
#include "ddt_plan.h"

namespace ddt {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
template <int U> struct Vec;
template <> struct Vec<16> { using T = u32x4; };
template <> struct Vec<8> { using T = u32x2; };
template <> struct Vec<4> { using T = uint32_t; };
template <> struct Vec<2> { using T = uint16_t; };
template <> struct Vec<1> { using T = uint8_t; };

// Nest of an item, ND dims kept in registers (ND = 0: generic MAXD path).
template <int ND> struct Nest {
    static constexpr int N = ND > 0 ? ND : MAXD;
    uint32_t ndim;
    uint32_t cnt[N];
    FastDiv fd[N];
    int64_t us[N];
    int64_t ps[N];
};

template <int ND>
__device__ __forceinline__ void load_nest(const Item *it, Nest<ND> &n)
{
    n.ndim = ND > 0 ? uint32_t(ND) : it->ndim;
#pragma unroll
    for (int j = 0; j < Nest<ND>::N; ++j) {
        n.cnt[j] = uint32_t(it->cnt[j]);
        n.fd[j] = it->fd[j];
        n.us[j] = it->ustr[j];
        n.ps[j] = it->pstr[j];
    }
}

// block index -> (user, packed) byte offsets over the nest (32-bit index path)
template <int ND>
__device__ __forceinline__ void nest_offsets32(const Nest<ND> &n, uint32_t blk, int64_t &uo, int64_t &po)
{
#pragma unroll
    for (int j = Nest<ND>::N - 1; j > 0; --j) {
        if (ND > 0 || j < int(n.ndim)) {
            uint32_t q = fastdiv(blk, n.fd[j]);
            uint32_t idx = blk - q * n.cnt[j];
            blk = q;
            uo += int64_t(idx) * n.us[j];
            po += int64_t(idx) * n.ps[j];
        }
    }
    if (ND > 0 || n.ndim > 0) {
        uo += int64_t(blk) * n.us[0];
        po += int64_t(blk) * n.ps[0];
    }
}

__device__ __forceinline__ void nest_offsets64(const Item *it, uint64_t blk, int64_t &uo, int64_t &po)
{
    for (int j = int(it->ndim) - 1; j > 0; --j) {
        uint64_t c = it->cnt[j];
        uint64_t idx = blk % c;
        blk /= c;
        uo += int64_t(idx) * it->ustr[j];
        po += int64_t(idx) * it->pstr[j];
    }
    if (it->ndim > 0) {
        uo += int64_t(blk) * it->ustr[0];
        po += int64_t(blk) * it->pstr[0];
    }
}

template <int U> constexpr int unroll() { return unroll_of(U); }

// Item::user / Item::packed are offsets from the launch's two base pointers (Bases), so one
// descriptor set serves every buffer pair with the same 16-byte alignment (ddt_convertor.cpp).
struct Bases {
    uint64_t u, p;
};

template <int U, int DIR>
__device__ __noinline__ void run_affine64(const Item *it, Bases bs, uint64_t ub, uint64_t ue)
{
    using T = typename Vec<U>::T;
    const uint64_t user = bs.u + it->user, packed = bs.p + it->packed, upb = it->upb;
    for (uint64_t u = ub + threadIdx.x; u < ue; u += THREADS) {
        uint64_t blk = u / upb, within = u - blk * upb;
        int64_t uo = int64_t(within) * U, po = uo;
        nest_offsets64(it, blk, uo, po);
        const T *src = reinterpret_cast<const T *>(DIR == 0 ? user + uo : packed + po);
        T *dst = reinterpret_cast<T *>(DIR == 0 ? packed + po : user + uo);
        *dst = *src;
    }
}

template <typename T, bool NT> __device__ __forceinline__ T ld(const T *p)
{
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}
// Write-through store (sc1): the line is not allocated dirty in L2; the bytes go on to
// the memory side with their byte mask (Item::wt, use_wt in ddt_plan.cpp).
__device__ __forceinline__ void st_wt(uint8_t *p, uint8_t v)
{
    asm volatile("global_store_byte %0, %1, off sc1" ::"v"(p), "v"(uint32_t(v)) : "memory");
}
__device__ __forceinline__ void st_wt(uint16_t *p, uint16_t v)
{
    asm volatile("global_store_short %0, %1, off sc1" ::"v"(p), "v"(uint32_t(v)) : "memory");
}
__device__ __forceinline__ void st_wt(uint32_t *p, uint32_t v)
{
    asm volatile("global_store_dword %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ void st_wt(u32x2 *p, u32x2 v)
{
    asm volatile("global_store_dwordx2 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ void st_wt(u32x4 *p, u32x4 v)
{
    asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
}

template <typename T, bool WT> __device__ __forceinline__ void st(T *p, T v)
{
    if constexpr (WT) st_wt(p, v);
    else *p = v;
}

// NT: 0 plain; 1 non-temporal user-side loads (pack of sparse gathers, Item::nt == 1);
// streaming leaves (Item::nt >= 2): 2 every load and store non-temporal, 3 loads only,
// 4 stores only, 5 loads only and only when packing (the user-side rows); 6 non-temporal
// user-side stores of an unpack (isolated narrow blocks, Item::wt == 3).
template <int U, int DIR, int ND, int NT, bool WT>
__device__ __forceinline__ void run_affine(const Item *it, Bases bs, uint32_t ub, uint32_t ue)
{
    using T = typename Vec<U>::T;
    constexpr int K = unroll<U>();
    const uint64_t user = bs.u + it->user, packed = bs.p + it->packed;
    Nest<ND> n;
    load_nest(it, n);
    const FastDiv fdu = it->fd_upb;
    const uint32_t upb = uint32_t(it->upb);
    for (uint32_t base = ub + threadIdx.x; base < ue; base += THREADS * K) {
        T v[K];
        T *dst[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint32_t u = base + uint32_t(k) * THREADS;
            dst[k] = nullptr;
            if (u < ue) {
                const uint32_t blk = fastdiv(u, fdu);
                const uint32_t within = u - blk * upb;
                int64_t uo = int64_t(within) * U, po = uo;
                nest_offsets32(n, blk, uo, po);
                const T *src = reinterpret_cast<const T *>(DIR == 0 ? user + uo : packed + po);
                dst[k] = reinterpret_cast<T *>(DIR == 0 ? packed + po : user + uo);
                v[k] = ld<T, ((NT == 1 || NT == 5) && DIR == 0) || NT == 2 || NT == 3>(src);
            }
        }
#pragma unroll
        for (int k = 0; k < K; ++k)
            if (dst[k]) {
                if constexpr (NT == 2 || NT == 4 || NT == 6)
                    __builtin_nontemporal_store(v[k], dst[k]);
                else
                    st<T, WT>(dst[k], v[k]);
            }
    }
}

// Line-dense records (round 3): blocks of blen bytes at a user stride S with blen < S <= 4 blen
// (BASELINE config 5: 20-byte records every 32 bytes), packed contiguously.  The unit loop moves
// one U-byte unit per lane (5 four-byte loads per record, partial lines per instruction); here a
// workgroup moves its task in chunks of R whole records (R * S <= DENSE_LDS bytes) through LDS:
// pack loads a chunk's user span with whole 16-byte loads (gap bytes included: they sit on lines
// the records touch anyway) and writes the packed stream with 16-byte stores when it is 16-byte
// aligned; unpack loads the packed span with 16-byte loads and writes each record with the widest
// aligned stores (gap bytes untouched).
//
// dense_write: the chunk of n records staged in LDS (its span starting `head` bytes into the LDS
// image) out to the destination: pstart = packed address of the chunk, urec = user address of its
// first record.
template <int DIR>
__device__ __forceinline__ void dense_write(const uint32_t *lds, uint32_t head, uint32_t n, uint32_t blen, uint32_t S,
                                            FastDiv fw, uint64_t pstart, uint64_t urec)
{
    if (DIR == 0) {
        const uint32_t pbytes = n * blen;
        if ((pstart & 15) == 0 && (pbytes & 15) == 0) {
            u32x4 *dst = reinterpret_cast<u32x4 *>(pstart);
            for (uint32_t c = threadIdx.x; c < pbytes / 16; c += THREADS) {
                uint32_t w[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const uint32_t q = 4 * c + uint32_t(i), r = fastdiv(q, fw);
                    w[i] = lds[(head + r * S) / 4 + (q - r * fw.d)];
                }
                dst[c] = u32x4{w[0], w[1], w[2], w[3]};
            }
        } else {
            uint32_t *dst = reinterpret_cast<uint32_t *>(pstart);
            for (uint32_t q = threadIdx.x; q < pbytes / 4; q += THREADS) {
                const uint32_t r = fastdiv(q, fw);
                dst[q] = lds[(head + r * S) / 4 + (q - r * fw.d)];
            }
        }
    } else {
        for (uint32_t r = threadIdx.x; r < n; r += THREADS) {
            uint8_t *d = reinterpret_cast<uint8_t *>(urec + uint64_t(r) * S);
            const uint32_t l0 = (head + r * blen) / 4;
            uint32_t o = 0;
            // widest stores the record's alignment allows (every record is 4-byte aligned)
            while (o < blen) {
                const uint64_t a = uint64_t(uintptr_t(d + o));
                const uint32_t w = l0 + o / 4;
                if ((a & 15) == 0 && blen - o >= 16) {
                    *reinterpret_cast<u32x4 *>(d + o) = u32x4{lds[w], lds[w + 1], lds[w + 2], lds[w + 3]};
                    o += 16;
                } else if ((a & 7) == 0 && blen - o >= 8) {
                    *reinterpret_cast<u32x2 *>(d + o) = u32x2{lds[w], lds[w + 1]};
                    o += 8;
                } else {
                    *reinterpret_cast<uint32_t *>(d + o) = lds[w];
                    o += 4;
                }
            }
        }
    }
}

// One chunk of nrec records whose first record sits at user address urec and packed address
// pstart: load its source span (16-byte loads, two per lane at most), stage it, write it out.
template <int DIR>
__device__ __forceinline__ void dense_chunk(u32x4 *buf, uint64_t urec, uint64_t pstart, uint32_t nrec, uint32_t S,
                                            FastDiv fw, bool ntl)
{
    const uint32_t blen = 4 * fw.d;
    const uint64_t a = DIR == 0 ? urec : pstart, a16 = a & ~uint64_t(15);
    const uint32_t head = uint32_t(a - a16);
    const uint32_t nvec = (head + (DIR == 0 ? (nrec - 1) * S + blen : nrec * blen) + 15) / 16;
    const u32x4 *src = reinterpret_cast<const u32x4 *>(a16);
    const uint32_t i0 = threadIdx.x, i1 = threadIdx.x + THREADS;
    u32x4 v0, v1;
    if (ntl) {
        if (i0 < nvec) v0 = __builtin_nontemporal_load(src + i0);
        if (i1 < nvec) v1 = __builtin_nontemporal_load(src + i1);
    } else {
        if (i0 < nvec) v0 = src[i0];
        if (i1 < nvec) v1 = src[i1];
    }
    if (i0 < nvec) buf[i0] = v0;
    if (i1 < nvec) buf[i1] = v1;
    __syncthreads();
    dense_write<DIR>(reinterpret_cast<const uint32_t *>(buf), head, nrec, blen, S, fw, pstart, urec);
}

// A task of one chunk (ddt_tune("dense", 1)): the workgroup finds its first record through the
// item's FastDivs and the nest, then moves the chunk.  Returns false when the records cross a
// run of the innermost dim (the caller runs the unit loop); a one-dim item never crosses (its
// unit range lies inside its leaf).
template <int DIR>
__device__ __forceinline__ bool run_dense1(const Item *it, Bases bs, uint32_t ub, uint32_t ue, u32x4 *buf)
{
    const FastDiv fdu = it->fd_upb;
    const uint32_t b0 = fastdiv(ub, fdu), nrec = fastdiv(ue - ub, fdu);
    const uint32_t nd = it->ndim;
    int64_t uo = 0, po = 0;
    uint32_t blk = b0;
    for (int j = int(nd) - 1; j > 0; --j) {
        const uint32_t q = fastdiv(blk, it->fd[j]);
        const uint32_t idx = blk - q * uint32_t(it->cnt[j]);
        if (j == int(nd) - 1 && idx + nrec > uint32_t(it->cnt[j]))
            return false;
        blk = q;
        uo += int64_t(idx) * it->ustr[j];
        po += int64_t(idx) * it->pstr[j];
    }
    uo += int64_t(blk) * it->ustr[0];
    po += int64_t(blk) * it->pstr[0];
    dense_chunk<DIR>(buf, bs.u + it->user + uint64_t(uo), bs.p + it->packed + uint64_t(po), nrec,
                     uint32_t(it->ustr[nd - 1]), it->fd_nblk, DIR == 1 || it->nt == 1);
    return true;
}

// A task of several chunks: the next chunk's loads are issued before the current chunk is
// written out (ddt_tune("dense", n) with n > 1).
template <int DIR>
__device__ __forceinline__ bool run_dense(const Item *it, Bases bs, uint32_t ub, uint32_t ue, u32x4 *buf)
{
    uint32_t *lds = reinterpret_cast<uint32_t *>(buf);
    constexpr uint32_t NV = DENSE_LDS / 16 + 2, PER = (NV + THREADS - 1) / THREADS;   // 2 vectors / lane
    const uint32_t upb = uint32_t(it->upb), U = it->U;
    const uint32_t b0 = ub / upb, nrec = (ue - ub) / upb;
    const uint32_t nd = it->ndim, inner = nd - 1;
    const uint32_t cin = uint32_t(it->cnt[inner]);
    if (b0 % cin + nrec > cin)
        return false;
    int64_t uo = 0, po = 0;
    {   // offsets of the task's first record
        uint32_t blk = b0;
        for (int j = int(nd) - 1; j > 0; --j) {
            const uint32_t q = fastdiv(blk, it->fd[j]);
            const uint32_t idx = blk - q * uint32_t(it->cnt[j]);
            blk = q;
            uo += int64_t(idx) * it->ustr[j];
            po += int64_t(idx) * it->pstr[j];
        }
        uo += int64_t(blk) * it->ustr[0];
        po += int64_t(blk) * it->pstr[0];
    }
    const uint32_t blen = upb * U, S = uint32_t(it->ustr[inner]), R = uint32_t(it->nbytes);
    const FastDiv fw = it->fd_nblk;   // division by the record's 4-byte words (blen / 4)
    const uint64_t ubase = bs.u + it->user + uint64_t(uo), pbase = bs.p + it->packed + uint64_t(po);
    const bool ntl = DIR == 1 || it->nt == 1;
    // the chunk starting at record r0: its 16-byte-aligned source span
    auto span = [&](uint32_t r0, uint32_t n, uint64_t &a16, uint32_t &head, uint32_t &nvec) {
        const uint64_t a = DIR == 0 ? ubase + uint64_t(r0) * S : pbase + uint64_t(r0) * blen;
        a16 = a & ~uint64_t(15);
        head = uint32_t(a - a16);
        nvec = (head + (DIR == 0 ? (n - 1) * S + blen : n * blen) + 15) / 16;
    };
    auto load = [&](uint32_t r0, u32x4 *v) {
        uint64_t a16;
        uint32_t head, nvec;
        span(r0, min(R, nrec - r0), a16, head, nvec);
        const u32x4 *src = reinterpret_cast<const u32x4 *>(a16);
#pragma unroll
        for (uint32_t k = 0; k < PER; ++k) {
            const uint32_t i = threadIdx.x + k * THREADS;
            if (i < nvec)
                v[k] = ntl ? __builtin_nontemporal_load(src + i) : src[i];
        }
    };
    u32x4 v[PER];
    load(0, v);
    for (uint32_t r0 = 0; r0 < nrec; r0 += R) {
        const uint32_t n = min(R, nrec - r0);
        uint64_t a16;
        uint32_t head, nvec;
        span(r0, n, a16, head, nvec);
        __syncthreads();   // the previous chunk's readers are done with the LDS
#pragma unroll
        for (uint32_t k = 0; k < PER; ++k) {
            const uint32_t i = threadIdx.x + k * THREADS;
            if (i < nvec)
                buf[i] = v[k];
        }
        __syncthreads();
        if (r0 + R < nrec)
            load(r0 + R, v);   // in flight while this chunk is written out
        dense_write<DIR>(lds, head, n, blen, S, fw, pbase + uint64_t(r0) * blen, ubase + uint64_t(r0) * S);
    }
    return true;
}

template <int U, int DIR>
__device__ __noinline__ void run_list_uni64(const Item *it, Bases bs, uint64_t ub, uint64_t ue)
{
    using T = typename Vec<U>::T;
    const uint64_t user = bs.u + it->user, packed = bs.p + it->packed, ulen = it->ulen;
    const bool d32 = it->ldisp32 != 0;
    const int32_t *disp32 = reinterpret_cast<const int32_t *>(it->ldisp);
    const int64_t *disp64 = reinterpret_cast<const int64_t *>(it->ldisp);
    const uint64_t upb = it->upb, nb = it->nblk;
    for (uint64_t u = ub + threadIdx.x; u < ue; u += THREADS) {
        uint64_t blk = u / upb, within = u - blk * upb;
        uint64_t i = blk % nb, outer = blk / nb;
        int64_t uo = 0, po = 0;
        nest_offsets64(it, outer, uo, po);
        int64_t d = d32 ? int64_t(disp32[i]) : disp64[i];
        uo += d + int64_t(within) * U;
        po += (it->same ? d : int64_t(i * ulen)) + int64_t(within) * U;
        const T *src = reinterpret_cast<const T *>(DIR == 0 ? user + uo : packed + po);
        T *dst = reinterpret_cast<T *>(DIR == 0 ? packed + po : user + uo);
        *dst = *src;
    }
}

// Index list with one block length: all K displacement loads of a round are issued
// (coalesced) before the K dependent gathers, so each round pays two memory latencies
// instead of 2K.
template <int U, int DIR, bool WT>
__device__ __forceinline__ void run_list_uni(const Item *it, Bases bs, uint32_t ub, uint32_t ue)
{
    using T = typename Vec<U>::T;
    constexpr int K = unroll<U>();
    const uint64_t user = bs.u + it->user, packed = bs.p + it->packed;
    const uint64_t ulen = it->ulen;
    const bool d32 = it->ldisp32 != 0;
    const bool same = it->same != 0;
    const int32_t *disp32 = reinterpret_cast<const int32_t *>(it->ldisp);
    const int64_t *disp64 = reinterpret_cast<const int64_t *>(it->ldisp);
    Nest<0> n;
    load_nest(it, n);
    const FastDiv fdu = it->fd_upb, fdn = it->fd_nblk;
    const uint32_t upb = uint32_t(it->upb), nb = uint32_t(it->nblk);
    for (uint32_t base = ub + threadIdx.x; base < ue; base += THREADS * K) {
        int64_t uo[K], po[K];
        uint32_t ii[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint32_t u = base + uint32_t(k) * THREADS;
            const uint32_t uu = u < ue ? u : ub;   // clamp: keeps the loads in bounds
            const uint32_t blk = fastdiv(uu, fdu);
            const uint32_t within = uu - blk * upb;
            const uint32_t outer = fastdiv(blk, fdn);
            ii[k] = blk - outer * nb;
            uo[k] = int64_t(within) * U;
            po[k] = int64_t(uint64_t(ii[k]) * ulen) + int64_t(within) * U;
            nest_offsets32(n, outer, uo[k], po[k]);
        }
        int64_t d[K];
#pragma unroll
        for (int k = 0; k < K; ++k)
            d[k] = d32 ? int64_t(disp32[ii[k]]) : disp64[ii[k]];
        if (same) {
#pragma unroll
            for (int k = 0; k < K; ++k)
                po[k] += d[k] - int64_t(uint64_t(ii[k]) * ulen);
        }
        T v[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const T *src = reinterpret_cast<const T *>(DIR == 0 ? user + uo[k] + d[k] : packed + po[k]);
            v[k] = *src;
        }
#pragma unroll
        for (int k = 0; k < K; ++k) {
            if (base + uint32_t(k) * THREADS < ue) {
                T *dst = reinterpret_cast<T *>(DIR == 0 ? packed + po[k] : user + uo[k] + d[k]);
                st<T, WT>(dst, v[k]);
            }
        }
    }
}

template <int U>
__device__ __forceinline__ void copy_run(uint8_t *dst, const uint8_t *src, uint64_t n)
{
    using T = typename Vec<U>::T;
    for (uint64_t o = 0; o < n; o += U)
        *reinterpret_cast<T *>(dst + o) = *reinterpret_cast<const T *>(src + o);
}

__device__ __forceinline__ void copy_bytes_aligned(uint8_t *dst, const uint8_t *src, uint64_t n, uint32_t U)
{
    const uint64_t a = uint64_t(uintptr_t(dst)) | uint64_t(uintptr_t(src)) | n;
    if (U >= 16 && (a & 15) == 0) copy_run<16>(dst, src, n);
    else if (U >= 8 && (a & 7) == 0) copy_run<8>(dst, src, n);
    else if (U >= 4 && (a & 3) == 0) copy_run<4>(dst, src, n);
    else if (U >= 2 && (a & 1) == 0) copy_run<2>(dst, src, n);
    else copy_run<1>(dst, src, n);
}

// Variable-length index list: one wave per group of 64 blocks.  Block packed offsets
// come from the per-group base (plan time) plus a wave-level exclusive prefix scan of
// the 64 block lengths, so no per-block packed offset is stored in HBM.
template <int DIR>
__device__ __forceinline__ void run_list_var(const Item *it, Bases bs, uint64_t ub, uint64_t ue)
{
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t user = bs.u + it->user, packed = bs.p + it->packed;
    const uint32_t *len = reinterpret_cast<const uint32_t *>(it->llen);
    const uint64_t *goff = reinterpret_cast<const uint64_t *>(it->lgoff);
    const bool d32 = it->ldisp32 != 0;
    const int32_t *disp32 = reinterpret_cast<const int32_t *>(it->ldisp);
    const int64_t *disp64 = reinterpret_cast<const int64_t *>(it->ldisp);
    const uint64_t ng = it->upb, nb = it->nblk, total = it->ulen;
    const int64_t w0 = it->w0, w1 = it->w1;
    for (uint64_t gu = ub + uint64_t(wave); gu < ue; gu += THREADS / 64) {
        const uint64_t outer = gu / ng, g = gu - outer * ng;
        int64_t uo = 0, po = 0;
        nest_offsets64(it, outer, uo, po);
        const uint64_t i = g * 64 + uint64_t(lane);
        const bool valid = i < nb;
        const uint64_t l = valid ? len[i] : 0;
        uint64_t incl = l;
#pragma unroll
        for (int s = 1; s < 64; s <<= 1) {
            uint64_t y = __shfl_up(incl, s, 64);
            if (lane >= s) incl += y;
        }
        const uint64_t excl = incl - l;
        const int64_t lx = int64_t(outer * total + goff[g] + excl);   // leaf-local offset
        const int64_t s0 = lx > w0 ? lx : w0;
        const int64_t s1 = (lx + int64_t(l)) < w1 ? lx + int64_t(l) : w1;
        if (valid && s1 > s0) {
            const int64_t d = d32 ? int64_t(disp32[i]) : disp64[i];
            const int64_t off = s0 - lx;
            uint8_t *up = reinterpret_cast<uint8_t *>(user + uo + d + off);
            uint8_t *pp = reinterpret_cast<uint8_t *>(packed + po + (it->same ? d : int64_t(goff[g] + excl)) + off);
            if (DIR == 0) copy_bytes_aligned(pp, up, uint64_t(s1 - s0), it->U);
            else copy_bytes_aligned(up, pp, uint64_t(s1 - s0), it->U);
        }
    }
}

// Deep nests (> 4 dims) are rare: their dims are re-read from the (cached) item on every
// unit instead of being held in registers, which keeps the kernel's SGPR budget small.
template <int U, int DIR, int NT, bool WT>
__device__ __forceinline__ void run_affine_deep(const Item *it, Bases bs, uint32_t ub, uint32_t ue)
{
    using T = typename Vec<U>::T;
    const uint64_t user = bs.u + it->user, packed = bs.p + it->packed;
    const FastDiv fdu = it->fd_upb;
    const uint32_t upb = uint32_t(it->upb);
    const int nd = int(it->ndim);
    for (uint32_t u = ub + threadIdx.x; u < ue; u += THREADS) {
        uint32_t blk = fastdiv(u, fdu);
        const uint32_t within = u - blk * upb;
        int64_t uo = int64_t(within) * U, po = uo;
        for (int j = nd - 1; j > 0; --j) {
            const uint32_t q = fastdiv(blk, it->fd[j]);
            const uint32_t idx = blk - q * uint32_t(it->cnt[j]);
            blk = q;
            uo += int64_t(idx) * it->ustr[j];
            po += int64_t(idx) * it->pstr[j];
        }
        uo += int64_t(blk) * it->ustr[0];
        po += int64_t(blk) * it->pstr[0];
        const T *src = reinterpret_cast<const T *>(DIR == 0 ? user + uo : packed + po);
        T *dst = reinterpret_cast<T *>(DIR == 0 ? packed + po : user + uo);
        st<T, WT>(dst, ld<T, NT == 1 && DIR == 0>(src));
    }
}

template <int U, int DIR, int NT, bool WT>
__device__ __forceinline__ void dispatch_affine_u(const Item *it, Bases bs, uint32_t ub, uint32_t ue)
{
    switch (it->ndim) {
    case 1: run_affine<U, DIR, 1, NT, WT>(it, bs, ub, ue); break;
    case 2: run_affine<U, DIR, 2, NT, WT>(it, bs, ub, ue); break;
    case 3: run_affine<U, DIR, 3, NT, WT>(it, bs, ub, ue); break;
    case 4: run_affine<U, DIR, 4, NT, WT>(it, bs, ub, ue); break;
    default: run_affine_deep<U, DIR, NT, WT>(it, bs, ub, ue); break;
    }
}

template <int DIR, int NT, bool WT>
__device__ __forceinline__ void dispatch_affine(const Item *it, Bases bs, uint32_t ub, uint32_t ue)
{
    switch (it->U) {
    case 16: dispatch_affine_u<16, DIR, NT, WT>(it, bs, ub, ue); break;
    case 8: dispatch_affine_u<8, DIR, NT, WT>(it, bs, ub, ue); break;
    case 4: dispatch_affine_u<4, DIR, NT, WT>(it, bs, ub, ue); break;
    case 2: dispatch_affine_u<2, DIR, NT, WT>(it, bs, ub, ue); break;
    default: dispatch_affine_u<1, DIR, NT, WT>(it, bs, ub, ue); break;
    }
}

// wt = 1 asks for write-through user-side stores (unpack); wt = 2 for every store.
template <int DIR>
__device__ __forceinline__ bool wt_stores(const Item *it)
{
    return it->wt == 2 || (DIR == 1 && (it->wt == 1 || it->wt == 3));
}

template <int DIR, bool WT>
__device__ __forceinline__ void dispatch_list_uni(const Item *it, Bases bs, uint32_t ub, uint32_t ue)
{
    switch (it->U) {
    case 16: run_list_uni<16, DIR, WT>(it, bs, ub, ue); break;
    case 8: run_list_uni<8, DIR, WT>(it, bs, ub, ue); break;
    case 4: run_list_uni<4, DIR, WT>(it, bs, ub, ue); break;
    case 2: run_list_uni<2, DIR, WT>(it, bs, ub, ue); break;
    default: run_list_uni<1, DIR, WT>(it, bs, ub, ue); break;
    }
}

// LISTS = false: affine + fragment items only (vector/hvector/subarray/struct nests), a
// lean register budget; LISTS = true adds the index-list paths.
// Task b of a launch: its item (scalar binary search over task_begin) and unit range.
__device__ __forceinline__ const Item *locate_task(const Item *__restrict__ items, uint32_t nitems, uint32_t b,
                                                   uint64_t &ub, uint64_t &ue)
{
    uint32_t lo = 0, hi = nitems - 1;
    while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) >> 1;
        if (items[mid].task_begin <= b) lo = mid;
        else hi = mid - 1;
    }
    const Item *it = items + lo;
    uint32_t t = b - it->task_begin;
    if (it->slab) {
        // Workgroups are dispatched round-robin over the 8 XCDs, so the item's local task t
        // runs on XCD (task_begin + t) % 8.  Give each XCD one contiguous slab of the item's
        // tasks instead of every 8th one (a bijection on [0, ntasks)).
        const uint32_t T = it->ntasks;
        if (it->slab == SLAB_FULL) {
            const uint32_t x = t & 7u, i = t >> 3, per = T >> 3, rem = T & 7u;
            t = x * per + (x < rem ? x : rem) + i;
        } else {
            // runs of C tasks per XCD inside groups of 8C (the tail stays round-robin)
            const uint32_t C = it->slab, G = C * 8u;
            if (t < T - T % G) {
                const uint32_t r = t % G;
                t = t - r + (r & 7u) * C + (r >> 3);
            }
        }
    }
    ub = it->u0 + t * it->units_per_task;
    ue = ub + it->units_per_task;
    if (ue > it->u1) ue = it->u1;
    return it;
}

template <int DIR, bool LISTS>
__device__ __forceinline__ void move_task(const Item *__restrict__ items, uint32_t nitems, Bases bs, uint32_t b)
{
    uint64_t ub, ue;
    const Item *it = locate_task(items, nitems, b, ub, ue);
    switch (it->kind) {
    case ITEM_AFFINE:
        if (it->idx64) {
            switch (it->U) {
            case 16: run_affine64<16, DIR>(it, bs, ub, ue); break;
            case 8: run_affine64<8, DIR>(it, bs, ub, ue); break;
            case 4: run_affine64<4, DIR>(it, bs, ub, ue); break;
            case 2: run_affine64<2, DIR>(it, bs, ub, ue); break;
            default: run_affine64<1, DIR>(it, bs, ub, ue); break;
            }
        } else {
            if (it->nt >= 2 && it->U == 16) {
                if (it->nt == 3) dispatch_affine_u<16, DIR, 3, false>(it, bs, uint32_t(ub), uint32_t(ue));
                else if (it->nt == 4) dispatch_affine_u<16, DIR, 4, false>(it, bs, uint32_t(ub), uint32_t(ue));
                else if (it->nt == 5) dispatch_affine_u<16, DIR, 5, false>(it, bs, uint32_t(ub), uint32_t(ue));
                else dispatch_affine_u<16, DIR, 2, false>(it, bs, uint32_t(ub), uint32_t(ue));
            } else if (DIR == 1 && it->wt == 3) {
                dispatch_affine<DIR, 6, false>(it, bs, uint32_t(ub), uint32_t(ue));
            } else if (wt_stores<DIR>(it)) {
                if (DIR == 0 && it->nt == 1) dispatch_affine<DIR, 1, true>(it, bs, uint32_t(ub), uint32_t(ue));
                else dispatch_affine<DIR, 0, true>(it, bs, uint32_t(ub), uint32_t(ue));
            } else {
                if (DIR == 0 && it->nt == 1) dispatch_affine<DIR, 1, false>(it, bs, uint32_t(ub), uint32_t(ue));
                else dispatch_affine<DIR, 0, false>(it, bs, uint32_t(ub), uint32_t(ue));
            }
        }
        break;
    case ITEM_LIST_UNI:
        if (!LISTS) break;
        if (it->idx64) {
            switch (it->U) {
            case 16: run_list_uni64<16, DIR>(it, bs, ub, ue); break;
            case 8: run_list_uni64<8, DIR>(it, bs, ub, ue); break;
            case 4: run_list_uni64<4, DIR>(it, bs, ub, ue); break;
            case 2: run_list_uni64<2, DIR>(it, bs, ub, ue); break;
            default: run_list_uni64<1, DIR>(it, bs, ub, ue); break;
            }
        } else {
            if (wt_stores<DIR>(it)) dispatch_list_uni<DIR, true>(it, bs, uint32_t(ub), uint32_t(ue));
            else dispatch_list_uni<DIR, false>(it, bs, uint32_t(ub), uint32_t(ue));
        }
        break;
    case ITEM_LIST_VAR:
        if (LISTS) run_list_var<DIR>(it, bs, ub, ue);
        break;
    default:   // ITEM_FRAG
        if (threadIdx.x == 0) {
            const uint8_t *src = reinterpret_cast<const uint8_t *>(DIR == 0 ? bs.u + it->user : bs.p + it->packed);
            uint8_t *dst = reinterpret_cast<uint8_t *>(DIR == 0 ? bs.p + it->packed : bs.u + it->user);
            for (uint64_t k = 0; k < it->nbytes; ++k)
                dst[k] = src[k];
        }
        break;
    }
}

// The fallback of a line-dense task whose records cross a run of the innermost dim: one U-byte
// unit per lane as 4-byte words, generic nest (few registers, so the dense kernel keeps its
// occupancy).
template <int DIR>
__device__ __forceinline__ void run_units_light(const Item *it, Bases bs, uint32_t ub, uint32_t ue)
{
    const uint64_t user = bs.u + it->user, packed = bs.p + it->packed;
    const uint32_t U = it->U, upb = uint32_t(it->upb), nd = it->ndim;
    const FastDiv fdu = it->fd_upb;
    for (uint32_t u = ub + threadIdx.x; u < ue; u += THREADS) {
        uint32_t blk = fastdiv(u, fdu);
        const uint32_t within = u - blk * upb;
        int64_t uo = int64_t(within) * U, po = uo;
        for (int j = int(nd) - 1; j > 0; --j) {
            const uint32_t q = fastdiv(blk, it->fd[j]);
            const uint32_t idx = blk - q * uint32_t(it->cnt[j]);
            blk = q;
            uo += int64_t(idx) * it->ustr[j];
            po += int64_t(idx) * it->pstr[j];
        }
        uo += int64_t(blk) * it->ustr[0];
        po += int64_t(blk) * it->pstr[0];
        const uint32_t *src = reinterpret_cast<const uint32_t *>(DIR == 0 ? user + uo : packed + po);
        uint32_t *dst = reinterpret_cast<uint32_t *>(DIR == 0 ? packed + po : user + uo);
        for (uint32_t w = 0; w < U / 4; ++w)
            dst[w] = src[w];
    }
}

// A launch whose items are all line-dense (Item::nbytes, ItemSet::all_dense) runs this kernel;
// in a launch that mixes them with other items they take the unit loop of the general kernel.
// Kept apart so neither kernel pays the other's registers or LDS (the general kernel stays at
// 56-58 VGPRs, 8 waves per SIMD, for pack and unpack; this one needs 28).
// SPLIT (the unpack): each task runs as two workgroups, the first taking the first half of its
// chunks; 16 workgroups per 8 tasks, workgroup b takes task (b / 16) * 8 + b % 8, so it stays
// on the XCD the task's slab was meant for (dense_grid on the host sizes the launch).  The
// unpack moves one chunk per workgroup that way (cfg5: 2043 -> 1949 us against two chunks,
// profiles/r3_ab_dense_chunks.jsonl) while the pack keeps two, its load of the next chunk in
// flight (1183 against 1483 us with one).
template <int DIR, bool SPLIT>
__device__ __forceinline__ void dense_body(const Item *__restrict__ items, uint32_t nitems, Bases bs, uint32_t ntasks)
{
    __shared__ u32x4 buf[DENSE_LDS / 16 + 2];   // one chunk's span (+ head alignment)
    const uint32_t nv = SPLIT ? (ntasks + 7) / 8 * 16 : ntasks;
    for (uint32_t b = blockIdx.x; b < nv; b += gridDim.x) {
        if (b != blockIdx.x)
            __syncthreads();
        uint64_t ub, ue;
        const uint32_t task = SPLIT ? (b >> 4) * 8 + (b & 7) : b;
        if (SPLIT && task >= ntasks)
            continue;
        const Item *it = locate_task(items, nitems, task, ub, ue);
        if (SPLIT) {
            const uint64_t upb = it->upb, R = it->nbytes;
            const uint64_t nch = ((ue - ub) / upb + R - 1) / R, mid = ub + (nch + 1) / 2 * R * upb;
            if (b & 8)
                ub = mid < ue ? mid : ue;
            else
                ue = mid < ue ? mid : ue;
            if (ub >= ue)
                continue;
        }
        const bool moved = ue - ub <= it->nbytes * it->upb
                               ? run_dense1<DIR>(it, bs, uint32_t(ub), uint32_t(ue), buf)
                               : run_dense<DIR>(it, bs, uint32_t(ub), uint32_t(ue), buf);
        if (!moved)
            run_units_light<DIR>(it, bs, uint32_t(ub), uint32_t(ue));
    }
}

template <int DIR, bool SPLIT>
__global__ __launch_bounds__(THREADS) void ddt_dense_kernel(const Item *__restrict__ items, uint32_t nitems,
                                                            uint64_t ubase, uint64_t pbase, uint32_t ntasks)
{
    dense_body<DIR, SPLIT>(items, nitems, Bases{ubase, pbase}, ntasks);
}

template <int DIR, bool SPLIT, uint32_t NI>
__global__ __launch_bounds__(THREADS) void ddt_dense_inline_kernel(ItemBlockN<NI> blk)
{
    const ItemBlockN<NI> *kb = reinterpret_cast<const ItemBlockN<NI> *>(
        (const void *) __builtin_amdgcn_kernarg_segment_ptr());
    dense_body<DIR, SPLIT>(kb->items, kb->n, Bases{kb->ubase, kb->pbase}, kb->ntasks);
}

// A single line-dense item whose chunks never cross a run of the innermost dim, launched with
// its few fields BY VALUE (ItemArgs, ~170 bytes of kernel arguments: one batch of scalar loads)
// and one workgroup per chunk, task structure and XCD slabs ignored.  Every cycle before a
// workgroup's first load lengthens its ~2 us life, and at 8 workgroups per CU the chip's bytes
// in flight shrink with it (Little's law).  On config 5's pack the engine's descriptor path --
// kernarg -> item pointer -> item fields, the task search and slab remap, a branch between the
// one- and multi-chunk routines, each a dependent round of scalar loads -- took 1142-1221 us
// where the same chunk routine called with the fields at hand took 1100 and a bare kernel with
// compile-time shape 1075 (scripts/ubench_dense4.hip, profiles/r3_ubench_dense4.log).
// (ItemArgs: ddt_device.h)

template <int DIR>
__global__ __launch_bounds__(THREADS) void ddt_dense1_kernel(ItemArgs args)
{
    __shared__ u32x4 buf[DENSE_LDS / 16 + 2];
    const ItemArgs *k = reinterpret_cast<const ItemArgs *>((const void *) __builtin_amdgcn_kernarg_segment_ptr());
    const uint32_t ub = k->u0 + blockIdx.x * k->cu;
    const uint32_t ue = min(ub + k->cu, k->u1);
    const uint32_t b0 = fastdiv(ub, k->fdu), nrec = fastdiv(ue - ub, k->fdu);
    const uint32_t nd = k->nd;
    int64_t uo = 0, po = 0;
    uint32_t blk = b0;
#pragma unroll
    for (int j = int(ITEM_ARG_DIMS) - 1; j > 0; --j) {
        if (j < int(nd)) {
            const uint32_t q = fastdiv(blk, k->fd[j]);
            const uint32_t idx = blk - q * k->cnt[j];
            blk = q;
            uo += int64_t(idx) * k->ustr[j];
            po += int64_t(idx) * k->pstr[j];
        }
    }
    uo += int64_t(blk) * k->ustr[0];
    po += int64_t(blk) * k->pstr[0];
    dense_chunk<DIR>(buf, k->ubase + uint64_t(uo), k->pbase + uint64_t(po), nrec, uint32_t(k->ustr[nd - 1]), k->fw,
                     DIR == 1 || k->nt == 1);
}

// One workgroup per task, or -- when the launch is capped below the task count (a window
// in pinned host memory, where PCIe and not the CU count is the limit: a few hundred
// workgroups keep it full, thousands of them contend for it, scripts/ubench_pcie.hip) --
// a grid-stride loop over the tasks.  A cap that is a multiple of 8 keeps every task on
// the XCD the slab mapping chose for it.
template <int DIR, bool LISTS>
__device__ __forceinline__ void move_body(const Item *__restrict__ items, uint32_t nitems, Bases bs, uint32_t ntasks)
{
    for (uint32_t b = blockIdx.x; b < ntasks; b += gridDim.x) {
        if (b != blockIdx.x)
            __syncthreads();   // LDS of the previous task (list scans) is free again
        move_task<DIR, LISTS>(items, nitems, bs, b);
    }
}

template <int DIR, bool LISTS>
__global__ __launch_bounds__(THREADS) void ddt_move_kernel(const Item *__restrict__ items, uint32_t nitems,
                                                           uint64_t ubase, uint64_t pbase, uint32_t ntasks)
{
    move_body<DIR, LISTS>(items, nitems, Bases{ubase, pbase}, ntasks);
}

// Argument-free launches (round 5).  Under HIP's default device-resident kernel arguments ANY
// launch with arguments costs the host ~2.9 us (the arguments are written across PCIe and read
// back before the doorbell), one without arguments 0.7 us (scripts/hostcost.cpp,
// profiles/r5_hostcost.jsonl): for a small message that is most of a call.  A hot descriptor set
// launched again and again on the same buffers (a persistent halo exchange, a fragment loop on
// fixed staging slots) is bound to one of NSLOT launch records in device memory, written once;
// the slot's kernel reads its record and takes no arguments at all -- no gridDim either (that
// would add hidden arguments): one workgroup per task.  One record table per translation unit
// (direction, lists); ddt_convertor.cpp binds and releases the slots.
// constant address space: the record loads are scalar and uniform (as kernel arguments are);
// from a __device__ array the compiler kept the fields in vector registers (92 VGPRs against
// the pointer kernel's 56) and large launches lost occupancy
static __constant__ LaunchRec g_launch[NSLOT + 1];   // [NSLOT]: never bound, ntasks 0

// The record index of an argument-free launch of slot kernel HI: the LDS size of the wave's
// workgroup from HW_REG_LDS_ALLOC (bits 12..20, 256-byte units; a scalar register read, no
// memory), which the launch set to (k % SLOT_PER_KERNEL + 1) x SLOT_LDS_UNIT.  Out of range (a
// launch that asked for no slot LDS, or more): NSLOT, the never-bound record.  slot_probe checks
// the decoding on each device before any record is bound.
constexpr int kHwRegLdsSize = ((9 - 1) << 11) | (12 << 6) | 6;   // HW_REG_LDS_ALLOC[20:12]

template <uint32_t HI>
__device__ __forceinline__ uint32_t slot_index()
{
    const uint32_t units = uint32_t(__builtin_amdgcn_s_getreg(kHwRegLdsSize));   // 256-byte units
    const uint32_t lo = units * 256u / SLOT_LDS_UNIT - 1u;
    return lo < SLOT_PER_KERNEL ? HI * SLOT_PER_KERNEL + lo : NSLOT;
}

template <int DIR, bool LISTS, uint32_t HI>
__global__ __launch_bounds__(THREADS) void ddt_move_slot_kernel()
{
    // no branch on the index: the record table's address load issues beside the register read,
    // and an out-of-range launch reads the never-bound record [NSLOT] (no tasks)
    const LaunchRec &r = g_launch[slot_index<HI>()];
    // the descriptor set is read-only for the kernel's lifetime, as a kernel-argument pointer is:
    // in the constant address space its uniform loads are scalar (a plain pointer loaded from
    // memory gives flat vector loads and twice the registers)
    using CItem = const __attribute__((address_space(4))) Item;
    const Item *items = (const Item *) (CItem *) r.items;
    if (blockIdx.x < r.ntasks)
        move_task<DIR, LISTS>(items, r.nitems, Bases{r.ubase, r.pbase}, blockIdx.x);
}

// slot_probe: the index launch k of slot kernel k / SLOT_PER_KERNEL reads back (out[k]), and
// out[NSLOT] for a launch without slot LDS (must be NSLOT: no record)
template <uint32_t HI>
static __global__ __attribute__((unused)) __launch_bounds__(64) void ddt_slot_probe_kernel(uint32_t *out)
{
    if (threadIdx.x == 0)
        out[0] = slot_index<HI>();
}

template <int DIR, bool LISTS>
static void launch_slot(uint32_t k, uint32_t grid, hipStream_t stream)
{
    const uint32_t lds = (k % SLOT_PER_KERNEL + 1) * SLOT_LDS_UNIT;
    if (k < SLOT_PER_KERNEL)
        hipLaunchKernelGGL((ddt_move_slot_kernel<DIR, LISTS, 0>), dim3(grid), dim3(THREADS), lds, stream);
    else
        hipLaunchKernelGGL((ddt_move_slot_kernel<DIR, LISTS, 1>), dim3(grid), dim3(THREADS), lds, stream);
}
static_assert(NSLOT == 2 * SLOT_PER_KERNEL, "launch_slot dispatches two slot kernels");

// Small launches carry their descriptors in the kernel-argument segment: no device
// buffer, no upload, no cache entry (fragment pipelines, windows, one-off messages).
template <int DIR, bool LISTS, uint32_t NI>
__global__ __launch_bounds__(THREADS) void ddt_move_inline_kernel(ItemBlockN<NI> blk)
{
    // read the block in place from the kernarg segment (taking the address of `blk`
    // would copy it to scratch)
    const ItemBlockN<NI> *kb = reinterpret_cast<const ItemBlockN<NI> *>(
        (const void *) __builtin_amdgcn_kernarg_segment_ptr());
    move_body<DIR, LISTS>(kb->items, kb->n, Bases{kb->ubase, kb->pbase}, kb->ntasks);
}

template <int DIR, bool LISTS, uint32_t NI>
static void launch_inline_n(const ItemBlock &blk, uint32_t ntasks, uint32_t grid, uint64_t ubase,
                            uint64_t pbase, hipStream_t stream)
{
    ItemBlockN<NI> b;
    b.n = blk.n;
    b.ntasks = ntasks;
    b.ubase = ubase;
    b.pbase = pbase;
    for (uint32_t i = 0; i < blk.n; ++i)
        b.items[i] = blk.items[i];
    hipLaunchKernelGGL((ddt_move_inline_kernel<DIR, LISTS, NI>), dim3(grid), dim3(THREADS), 0,
                       stream, b);
}

template <int DIR, uint32_t NI>
static void launch_dense_inline_n(const ItemBlock &blk, uint32_t ntasks, uint32_t grid, uint64_t ubase,
                                  uint64_t pbase, hipStream_t stream, bool split)
{
    ItemBlockN<NI> b;
    b.n = blk.n;
    b.ntasks = ntasks;
    b.ubase = ubase;
    b.pbase = pbase;
    for (uint32_t i = 0; i < blk.n; ++i)
        b.items[i] = blk.items[i];
    if (split)
        hipLaunchKernelGGL((ddt_dense_inline_kernel<DIR, true, NI>), dim3(grid), dim3(THREADS), 0, stream, b);
    else
        hipLaunchKernelGGL((ddt_dense_inline_kernel<DIR, false, NI>), dim3(grid), dim3(THREADS), 0, stream, b);
}

template <int DIR, bool LISTS>
static void launch_inline(const ItemBlock &blk, uint32_t ntasks, uint32_t grid, uint64_t ubase, uint64_t pbase,
                          hipStream_t stream)
{
    if (blk.n == 1) launch_inline_n<DIR, LISTS, 1>(blk, ntasks, grid, ubase, pbase, stream);
    else if (blk.n == 2) launch_inline_n<DIR, LISTS, 2>(blk, ntasks, grid, ubase, pbase, stream);
    else if (blk.n <= 4) launch_inline_n<DIR, LISTS, 4>(blk, ntasks, grid, ubase, pbase, stream);
    else launch_inline_n<DIR, LISTS, INLINE_ITEMS>(blk, ntasks, grid, ubase, pbase, stream);
}

// The line-dense launchers of one direction (instantiated with the LISTS = false units).
#define DDT_DENSE_INSTANCE(DIRV, TAG)                                                                   \
    hipError_t launch_dense_inline_##TAG(const ItemBlock &blk, uint32_t ntasks, uint32_t grid,          \
                                         uint64_t ubase, uint64_t pbase, hipStream_t stream, bool split) \
    {                                                                                                   \
        if (blk.n == 1) launch_dense_inline_n<DIRV, 1>(blk, ntasks, grid, ubase, pbase, stream, split); \
        else if (blk.n == 2) launch_dense_inline_n<DIRV, 2>(blk, ntasks, grid, ubase, pbase, stream, split); \
        else launch_dense_inline_n<DIRV, INLINE_ITEMS>(blk, ntasks, grid, ubase, pbase, stream, split); \
        return hipGetLastError();                                                                       \
    }                                                                                                   \
    hipError_t launch_dense1_##TAG(const ItemArgs &a, uint32_t nchunks, hipStream_t stream)            \
    {                                                                                                   \
        hipLaunchKernelGGL((ddt_dense1_kernel<DIRV>), dim3(nchunks), dim3(THREADS), 0, stream, a);      \
        return hipGetLastError();                                                                       \
    }                                                                                                   \
    hipError_t launch_dense_##TAG(const Item *d_items, uint32_t nitems, uint32_t ntasks, uint32_t grid, \
                                  uint64_t ubase, uint64_t pbase, hipStream_t stream, bool split)       \
    {                                                                                                   \
        if (split)                                                                                      \
            hipLaunchKernelGGL((ddt_dense_kernel<DIRV, true>), dim3(grid), dim3(THREADS), 0, stream,    \
                               d_items, nitems, ubase, pbase, ntasks);                                  \
        else                                                                                            \
            hipLaunchKernelGGL((ddt_dense_kernel<DIRV, false>), dim3(grid), dim3(THREADS), 0, stream,   \
                               d_items, nitems, ubase, pbase, ntasks);                                  \
        return hipGetLastError();                                                                       \
    }

// One (direction, lists) instance of the launchers: ddt_kernels.hip dispatches to them.
#define DDT_MOVE_INSTANCE(DIRV, LISTSV, TAG)                                                           \
    hipError_t launch_move_inline_##TAG(const ItemBlock &blk, uint32_t ntasks, uint32_t grid,          \
                                        uint64_t ubase, uint64_t pbase, hipStream_t stream)            \
    {                                                                                                  \
        launch_inline<DIRV, LISTSV>(blk, ntasks, grid, ubase, pbase, stream);                          \
        return hipGetLastError();                                                                      \
    }                                                                                                  \
    hipError_t launch_move_##TAG(const Item *d_items, uint32_t nitems, uint32_t ntasks, uint32_t grid, \
                                 uint64_t ubase, uint64_t pbase, hipStream_t stream)                   \
    {                                                                                                  \
        hipLaunchKernelGGL((ddt_move_kernel<DIRV, LISTSV>), dim3(grid), dim3(THREADS), 0, stream,      \
                           d_items, nitems, ubase, pbase, ntasks);                                     \
        return hipGetLastError();                                                                      \
    }

// The argument-free launchers of the affine kernel families (LISTS = false units only: index-list
// launches keep their arguments; eight slot kernels per direction are a large part of the code).
#define DDT_SLOT_INSTANCE(DIRV, TAG)                                                                   \
    hipError_t launch_move_slot_##TAG(uint32_t k, uint32_t ntasks, hipStream_t stream)                 \
    {                                                                                                  \
        launch_slot<DIRV, false>(k, ntasks, stream);                                                   \
        return hipGetLastError();                                                                      \
    }                                                                                                  \
    hipError_t slot_table_##TAG(void **addr)                                                           \
    {                                                                                                  \
        return hipGetSymbolAddress(addr, HIP_SYMBOL(g_launch));                                        \
    }                                                                                                  \
    hipError_t slot_probe_##TAG(uint32_t *d_out, hipStream_t stream)                                   \
    {                                                                                                  \
        for (uint32_t k = 0; k < NSLOT; ++k) {                                                         \
            const uint32_t lds = (k % SLOT_PER_KERNEL + 1) * SLOT_LDS_UNIT;                            \
            if (k < SLOT_PER_KERNEL)                                                                   \
                hipLaunchKernelGGL(ddt_slot_probe_kernel<0>, dim3(1), dim3(64), lds, stream, d_out + k); \
            else                                                                                       \
                hipLaunchKernelGGL(ddt_slot_probe_kernel<1>, dim3(1), dim3(64), lds, stream, d_out + k); \
        }                                                                                              \
        hipLaunchKernelGGL(ddt_slot_probe_kernel<0>, dim3(1), dim3(64), 0, stream, d_out + NSLOT);     \
        return hipGetLastError();                                                                      \
    }

}  // namespace ddt
