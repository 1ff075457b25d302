// ddt_kernels.hip -- gfx950 gather/scatter kernels of the derived-datatype engine.
//
// One launch moves every leaf stream of a plan (ddt_plan.cpp).  Work is cut into
// tasks of ~32 KiB of packed bytes; workgroup b finds its item by a scalar binary
// search over items[].task_begin and then streams units of U bytes (U = 16 when
// user and packed addresses, block length and every stride are 16-byte aligned):
// consecutive lanes take consecutive units, so the packed side is a fully
// coalesced dwordx4 stream and the user side is coalesced whenever blocks are
// >= 64*U bytes.  Each lane keeps K independent loads in flight before its stores
// (ILP for HBM latency).  Index arithmetic is 32-bit with invariant-divisor
// multiply-high division (FastDiv); 64-bit only when a leaf has >= 2^32 units.
//
// Replaces the per-block cbmemcpy loop of opal_pack_accelerator_simple /
// opal_unpack_accelerator_simple (opal_datatype_pack_accelerator.c:161-295,
// opal_datatype_unpack_accelerator.c:210-368).
#include <hip/hip_runtime.h>

#include "ddt_device.h"
#include "ddt_plan.h"

namespace ddt {

template <int U> struct Vec;
template <> struct Vec<16> { using T = uint4; };
template <> struct Vec<8> { using T = uint2; };
template <> struct Vec<4> { using T = uint32_t; };
template <> struct Vec<2> { using T = uint16_t; };
template <> struct Vec<1> { using T = uint8_t; };

struct Nest {
    uint32_t ndim;
    uint32_t cnt[MAXD];
    FastDiv fd[MAXD];
    int64_t us[MAXD];
    int64_t ps[MAXD];
};

__device__ __forceinline__ void load_nest(const Item *it, Nest &n)
{
    n.ndim = it->ndim;
#pragma unroll
    for (int j = 0; j < MAXD; ++j) {
        n.cnt[j] = uint32_t(it->cnt[j]);
        n.fd[j] = it->fd[j];
        n.us[j] = it->ustr[j];
        n.ps[j] = it->pstr[j];
    }
}

// block index -> (user, packed) byte offsets over the nest (32-bit index path)
__device__ __forceinline__ void nest_offsets32(const Nest &n, uint32_t blk, int64_t &uo, int64_t &po)
{
#pragma unroll
    for (int j = MAXD - 1; j > 0; --j) {
        if (j < int(n.ndim)) {
            uint32_t q = fastdiv(blk, n.fd[j]);
            uint32_t idx = blk - q * n.cnt[j];
            blk = q;
            uo += int64_t(idx) * n.us[j];
            po += int64_t(idx) * n.ps[j];
        }
    }
    if (n.ndim > 0) {
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

template <int U, int DIR>
__device__ __forceinline__ void run_affine(const Item *it, uint64_t ub, uint64_t ue)
{
    using T = typename Vec<U>::T;
    constexpr int K = U >= 16 ? 4 : 8;
    const uint64_t user = it->user, packed = it->packed;
    if (it->idx64) {
        const uint64_t upb = it->upb;
        for (uint64_t u = ub + threadIdx.x; u < ue; u += THREADS) {
            uint64_t blk = u / upb, within = u - blk * upb;
            int64_t uo = int64_t(within) * U, po = uo;
            nest_offsets64(it, blk, uo, po);
            const T *src = reinterpret_cast<const T *>(DIR == 0 ? user + uo : packed + po);
            T *dst = reinterpret_cast<T *>(DIR == 0 ? packed + po : user + uo);
            *dst = *src;
        }
        return;
    }
    Nest n;
    load_nest(it, n);
    const FastDiv fdu = it->fd_upb;
    const uint32_t upb = uint32_t(it->upb);
    const uint32_t e = uint32_t(ue);
    for (uint32_t base = uint32_t(ub) + threadIdx.x; base < e; base += THREADS * K) {
        T v[K];
        T *dst[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint32_t u = base + uint32_t(k) * THREADS;
            dst[k] = nullptr;
            if (u < e) {
                const uint32_t blk = fastdiv(u, fdu);
                const uint32_t within = u - blk * upb;
                int64_t uo = int64_t(within) * U, po = uo;
                nest_offsets32(n, blk, uo, po);
                const T *src = reinterpret_cast<const T *>(DIR == 0 ? user + uo : packed + po);
                dst[k] = reinterpret_cast<T *>(DIR == 0 ? packed + po : user + uo);
                v[k] = *src;
            }
        }
#pragma unroll
        for (int k = 0; k < K; ++k)
            if (dst[k])
                *dst[k] = v[k];
    }
}

template <int U, int DIR>
__device__ __forceinline__ void run_list_uni(const Item *it, uint64_t ub, uint64_t ue)
{
    using T = typename Vec<U>::T;
    constexpr int K = U >= 16 ? 4 : 8;
    const uint64_t user = it->user, packed = it->packed;
    const uint64_t ulen = it->ulen;
    const bool d32 = it->ldisp32 != 0;
    const int32_t *disp32 = reinterpret_cast<const int32_t *>(it->ldisp);
    const int64_t *disp64 = reinterpret_cast<const int64_t *>(it->ldisp);
    if (it->idx64) {
        const uint64_t upb = it->upb, nb = it->nblk;
        for (uint64_t u = ub + threadIdx.x; u < ue; u += THREADS) {
            uint64_t blk = u / upb, within = u - blk * upb;
            uint64_t i = blk % nb, outer = blk / nb;
            int64_t uo = 0, po = 0;
            nest_offsets64(it, outer, uo, po);
            int64_t d = d32 ? int64_t(disp32[i]) : disp64[i];
            uo += d + int64_t(within) * U;
            po += int64_t(i * ulen + within * U);
            const T *src = reinterpret_cast<const T *>(DIR == 0 ? user + uo : packed + po);
            T *dst = reinterpret_cast<T *>(DIR == 0 ? packed + po : user + uo);
            *dst = *src;
        }
        return;
    }
    Nest n;
    load_nest(it, n);
    const FastDiv fdu = it->fd_upb, fdn = it->fd_nblk;
    const uint32_t upb = uint32_t(it->upb), nb = uint32_t(it->nblk);
    const uint32_t e = uint32_t(ue);
    for (uint32_t base = uint32_t(ub) + threadIdx.x; base < e; base += THREADS * K) {
        T v[K];
        T *dst[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint32_t u = base + uint32_t(k) * THREADS;
            dst[k] = nullptr;
            if (u < e) {
                const uint32_t blk = fastdiv(u, fdu);
                const uint32_t within = u - blk * upb;
                const uint32_t outer = fastdiv(blk, fdn);
                const uint32_t i = blk - outer * nb;
                int64_t uo = 0, po = 0;
                nest_offsets32(n, outer, uo, po);
                const int64_t d = d32 ? int64_t(disp32[i]) : disp64[i];
                uo += d + int64_t(within) * U;
                po += int64_t(uint64_t(i) * ulen) + int64_t(within) * U;
                const T *src = reinterpret_cast<const T *>(DIR == 0 ? user + uo : packed + po);
                dst[k] = reinterpret_cast<T *>(DIR == 0 ? packed + po : user + uo);
                v[k] = *src;
            }
        }
#pragma unroll
        for (int k = 0; k < K; ++k)
            if (dst[k])
                *dst[k] = v[k];
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
__device__ __forceinline__ void run_list_var(const Item *it, uint64_t ub, uint64_t ue)
{
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t user = it->user, packed = it->packed;
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
            uint8_t *pp = reinterpret_cast<uint8_t *>(packed + po + int64_t(goff[g] + excl) + off);
            if (DIR == 0) copy_bytes_aligned(pp, up, uint64_t(s1 - s0), it->U);
            else copy_bytes_aligned(up, pp, uint64_t(s1 - s0), it->U);
        }
    }
}

template <int DIR>
__global__ __launch_bounds__(THREADS) void ddt_move_kernel(const Item *__restrict__ items, uint32_t nitems)
{
    const uint32_t b = blockIdx.x;
    uint32_t lo = 0, hi = nitems - 1;
    while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) >> 1;
        if (items[mid].task_begin <= b) lo = mid;
        else hi = mid - 1;
    }
    const Item *it = items + lo;
    const uint64_t t = b - it->task_begin;
    const uint64_t ub = it->u0 + t * it->units_per_task;
    uint64_t ue = ub + it->units_per_task;
    if (ue > it->u1) ue = it->u1;
    switch (it->kind) {
    case ITEM_AFFINE:
        switch (it->U) {
        case 16: run_affine<16, DIR>(it, ub, ue); break;
        case 8: run_affine<8, DIR>(it, ub, ue); break;
        case 4: run_affine<4, DIR>(it, ub, ue); break;
        case 2: run_affine<2, DIR>(it, ub, ue); break;
        default: run_affine<1, DIR>(it, ub, ue); break;
        }
        break;
    case ITEM_LIST_UNI:
        switch (it->U) {
        case 16: run_list_uni<16, DIR>(it, ub, ue); break;
        case 8: run_list_uni<8, DIR>(it, ub, ue); break;
        case 4: run_list_uni<4, DIR>(it, ub, ue); break;
        case 2: run_list_uni<2, DIR>(it, ub, ue); break;
        default: run_list_uni<1, DIR>(it, ub, ue); break;
        }
        break;
    case ITEM_LIST_VAR:
        run_list_var<DIR>(it, ub, ue);
        break;
    default:   // ITEM_FRAG
        if (threadIdx.x == 0) {
            const uint8_t *src = reinterpret_cast<const uint8_t *>(DIR == 0 ? it->user : it->packed);
            uint8_t *dst = reinterpret_cast<uint8_t *>(DIR == 0 ? it->packed : it->user);
            for (uint64_t k = 0; k < it->nbytes; ++k)
                dst[k] = src[k];
        }
        break;
    }
}

hipError_t launch_move(const Item *d_items, uint32_t nitems, uint32_t ntasks, int dir,
                       hipStream_t stream)
{
    if (ntasks == 0 || nitems == 0)
        return hipSuccess;
    if (dir == 0)
        hipLaunchKernelGGL(ddt_move_kernel<0>, dim3(ntasks), dim3(THREADS), 0, stream, d_items, nitems);
    else
        hipLaunchKernelGGL(ddt_move_kernel<1>, dim3(ntasks), dim3(THREADS), 0, stream, d_items, nitems);
    return hipGetLastError();
}

}  // namespace ddt
