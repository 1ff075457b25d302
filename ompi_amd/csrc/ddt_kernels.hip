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
#include <cstdlib>

#include <hip/hip_runtime.h>

#include "ddt_device.h"
#include "ddt_plan.h"

// The move kernel itself lives in ddt_move.hip.h and is instantiated in four translation
// units (ddt_move_{p,u}{0,1}.hip: pack / unpack x without / with index lists) that the build
// compiles in parallel; this file dispatches to them and holds the external32 kernel.

namespace ddt {

#define DDT_MOVE_DECLARE(TAG)                                                                          \
    hipError_t launch_move_inline_##TAG(const ItemBlock &blk, uint32_t ntasks, uint32_t grid,          \
                                        uint64_t ubase, uint64_t pbase, hipStream_t stream);           \
    hipError_t launch_move_##TAG(const Item *d_items, uint32_t nitems, uint32_t ntasks, uint32_t grid, \
                                 uint64_t ubase, uint64_t pbase, hipStream_t stream);
DDT_MOVE_DECLARE(p0)
DDT_MOVE_DECLARE(p1)
DDT_MOVE_DECLARE(u0)
DDT_MOVE_DECLARE(u1)
#undef DDT_MOVE_DECLARE
hipError_t launch_dense_inline_p0(const ItemBlock &, uint32_t, uint32_t, uint64_t, uint64_t, hipStream_t, bool);
hipError_t launch_dense_inline_u0(const ItemBlock &, uint32_t, uint32_t, uint64_t, uint64_t, hipStream_t, bool);
hipError_t launch_dense_p0(const Item *, uint32_t, uint32_t, uint32_t, uint64_t, uint64_t, hipStream_t, bool);
hipError_t launch_dense_u0(const Item *, uint32_t, uint32_t, uint32_t, uint64_t, uint64_t, hipStream_t, bool);
hipError_t launch_dense1_p0(const ItemArgs &, uint32_t, hipStream_t);
hipError_t launch_dense1_u0(const ItemArgs &, uint32_t, hipStream_t);

// The line-dense unpack runs each task as two workgroups (ddt_tune "dsplit", dense_body):
// 16 workgroups per 8 tasks.
static bool dense_split(int dir, uint32_t ntasks)
{
    return dir == 1 && tuning().dsplit != 0 && ntasks < 0x70000000u;
}
static uint32_t dense_grid(bool split, uint32_t ntasks, uint32_t grid_cap)
{
    const uint32_t nv = split ? (ntasks + 7) / 8 * 16 : ntasks;
    return grid_cap && grid_cap < nv ? grid_cap : nv;
}

// The by-value single-item launch: a large launch of ONE line-dense item whose chunks all lie
// inside one run of the innermost dim passes the item's fields in the kernel arguments (ItemArgs)
// instead of a descriptor in memory, one workgroup per chunk (ddt_dense1_kernel; ddt_tune
// "dfast", default: pack).  Returns false when the item does not qualify (the caller launches the
// descriptor set as usual).  Small launches keep the descriptor path: ~170 bytes of kernel
// arguments cost ~1 us more host time per launch than a descriptor pointer (device-resident
// kernel arguments, profiles/r1_hostbench.log).  The same launch form for streaming items of
// 16-byte units (a y or z face over 512 fields) was built and measured within box noise of the
// descriptor kernel, its unpacks slower (commit 05bf71b, profiles/r3_ubench_face1.log,
// r3_ab_faces_afast.jsonl), and dropped: a 16 KiB streaming task hides its prologue, a 4 KiB
// dense chunk does not.
static bool fill_args(const Item &it, uint64_t ubase, uint64_t pbase, uint64_t cu, ItemArgs &a)
{
    if (it.kind != ITEM_AFFINE || it.idx64 || it.ndim < 1 || it.ndim > ITEM_ARG_DIMS || it.upb == 0 || cu == 0)
        return false;
    const uint64_t n = (it.u1 - it.u0 + cu - 1) / cu;
    // the kernel's 32-bit unit arithmetic: the last chunk's end (u0 + n * cu) must not wrap
    if (n < 1024 || n >= 0x7fffffffull || it.u0 + n * cu >= 0xffffffffull)
        return false;
    a = ItemArgs{};
    a.ubase = ubase + it.user;
    a.pbase = pbase + it.packed;
    a.u0 = uint32_t(it.u0);
    a.u1 = uint32_t(it.u1);
    a.cu = uint32_t(cu);
    a.nd = it.ndim;
    a.fdu = it.fd_upb;
    a.fw = it.fd_nblk;
    a.nt = it.nt;
    for (uint32_t j = 0; j < it.ndim; ++j) {
        a.cnt[j] = uint32_t(it.cnt[j]);
        a.fd[j] = it.fd[j];
        a.ustr[j] = it.ustr[j];
        a.pstr[j] = it.pstr[j];
    }
    return true;
}

bool launch_single_item(const Item &it, int dir, uint64_t ubase, uint64_t pbase, hipStream_t stream,
                        hipError_t *err)
{
    // line-dense only (Item::nbytes = records per chunk)
    if (it.kind != ITEM_AFFINE || it.upb == 0 || !it.nbytes || !(tuning().dfast & (dir == 0 ? 1 : 2))
        || it.u0 % it.upb != 0)
        return false;
    const uint64_t R = it.nbytes, cin = it.cnt[it.ndim ? it.ndim - 1 : 0];
    if (it.ndim > 1 && (cin % R != 0 || ((it.u0 / it.upb) % cin) % R != 0))
        return false;   // a chunk could cross an inner run
    ItemArgs a;
    if (!fill_args(it, ubase, pbase, R * it.upb, a))
        return false;
    const uint32_t n = uint32_t((it.u1 - it.u0 + a.cu - 1) / a.cu);
    *err = dir == 0 ? launch_dense1_p0(a, n, stream) : launch_dense1_u0(a, n, stream);
    return true;
}

hipError_t launch_move_inline(const ItemBlock &blk, uint32_t ntasks, int dir, bool lists, uint64_t ubase,
                              uint64_t pbase, hipStream_t stream, uint32_t grid_cap, bool dense)
{
    if (ntasks == 0 || blk.n == 0)
        return hipSuccess;
    const uint32_t g = grid_cap && grid_cap < ntasks ? grid_cap : ntasks;
    if (dense && !lists) {
        const bool sp = dense_split(dir, ntasks);
        const uint32_t gs = dense_grid(sp, ntasks, grid_cap);
        return dir == 0 ? launch_dense_inline_p0(blk, ntasks, gs, ubase, pbase, stream, false)
                        : launch_dense_inline_u0(blk, ntasks, gs, ubase, pbase, stream, sp);
    }
    if (dir == 0)
        return lists ? launch_move_inline_p1(blk, ntasks, g, ubase, pbase, stream)
                     : launch_move_inline_p0(blk, ntasks, g, ubase, pbase, stream);
    return lists ? launch_move_inline_u1(blk, ntasks, g, ubase, pbase, stream)
                 : launch_move_inline_u0(blk, ntasks, g, ubase, pbase, stream);
}

hipError_t launch_move(const Item *d_items, uint32_t nitems, uint32_t ntasks, int dir, bool lists,
                       uint64_t ubase, uint64_t pbase, hipStream_t stream, uint32_t grid_cap, bool dense)
{
    if (ntasks == 0 || nitems == 0)
        return hipSuccess;
    const uint32_t g = grid_cap && grid_cap < ntasks ? grid_cap : ntasks;
    if (dense && !lists) {
        const bool sp = dense_split(dir, ntasks);
        const uint32_t gs = dense_grid(sp, ntasks, grid_cap);
        return dir == 0 ? launch_dense_p0(d_items, nitems, ntasks, gs, ubase, pbase, stream, false)
                        : launch_dense_u0(d_items, nitems, ntasks, gs, ubase, pbase, stream, sp);
    }
    if (dir == 0)
        return lists ? launch_move_p1(d_items, nitems, ntasks, g, ubase, pbase, stream)
                     : launch_move_p0(d_items, nitems, ntasks, g, ubase, pbase, stream);
    return lists ? launch_move_u1(d_items, nitems, ntasks, g, ubase, pbase, stream)
                 : launch_move_u0(d_items, nitems, ntasks, g, ubase, pbase, stream);
}

hipError_t launch_move_slot_p0(uint32_t k, uint32_t ntasks, hipStream_t stream);
hipError_t launch_move_slot_u0(uint32_t k, uint32_t ntasks, hipStream_t stream);
hipError_t slot_table_p0(void **addr);
hipError_t slot_table_u0(void **addr);
hipError_t slot_probe_p0(uint32_t *d_out, hipStream_t stream);
hipError_t slot_probe_u0(uint32_t *d_out, hipStream_t stream);

hipError_t launch_move_slot(int dir, uint32_t k, uint32_t ntasks, hipStream_t stream)
{
    return dir == 0 ? launch_move_slot_p0(k, ntasks, stream) : launch_move_slot_u0(k, ntasks, stream);
}

hipError_t slot_table(int dir, void **addr)
{
    return dir == 0 ? slot_table_p0(addr) : slot_table_u0(addr);
}

hipError_t slot_probe(int dir, uint32_t *d_out, hipStream_t stream)
{
    return dir == 0 ? slot_probe_p0(d_out, stream) : slot_probe_u0(d_out, stream);
}

// ---------------------------------------------------------------- completion signal
// A synchronous call (MPI_Pack / MPI_Unpack, a convertor without ACCELERATOR_ASYNC) must return
// with the data in place (pack.c.in:129-150).  HIP's completion round trip costs ~9.5 us for a
// kernel of any size (profiles/r5_hostcost_sync.jsonl); instead, the call enqueues behind its move
// kernels the argument-free kernel of a signal slot S, which bumps S's device counter and stores
// the new value to S's word of a pinned, host-coherent page with a system-scope release, and the
// host spins on that word (ddt_convertor.cpp: complete_sync).  The kernel starts only after the
// stream's previous work completed, and so after that work's end-of-kernel release.
constexpr int NSIG_KERNEL = 16;   // = kSigSlots (ddt_plan.h)
constexpr int SIG_STRIDE = 16;    // words between slots: one 64-byte line each
static __device__ uint32_t *g_sig_host;
static __device__ uint32_t g_sig_count[NSIG_KERNEL];

template <int S>
__global__ __launch_bounds__(64) void ddt_signal_kernel()
{
    if (threadIdx.x == 0) {
        const uint32_t v = __hip_atomic_fetch_add(&g_sig_count[S], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
        __hip_atomic_store(g_sig_host + S * SIG_STRIDE, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

hipError_t signal_setup(uint32_t *host_page, hipStream_t s)
{
    hipError_t e = hipMemcpyToSymbolAsync(HIP_SYMBOL(g_sig_host), &host_page, sizeof(host_page), 0,
                                          hipMemcpyHostToDevice, s);
    return e != hipSuccess ? e : hipStreamSynchronize(s);
}

hipError_t launch_signal(int k, hipStream_t stream)
{
    const dim3 g(1), b(64);
    switch (k) {
    case 0: hipLaunchKernelGGL(ddt_signal_kernel<0>, g, b, 0, stream); break;
    case 1: hipLaunchKernelGGL(ddt_signal_kernel<1>, g, b, 0, stream); break;
    case 2: hipLaunchKernelGGL(ddt_signal_kernel<2>, g, b, 0, stream); break;
    case 3: hipLaunchKernelGGL(ddt_signal_kernel<3>, g, b, 0, stream); break;
    case 4: hipLaunchKernelGGL(ddt_signal_kernel<4>, g, b, 0, stream); break;
    case 5: hipLaunchKernelGGL(ddt_signal_kernel<5>, g, b, 0, stream); break;
    case 6: hipLaunchKernelGGL(ddt_signal_kernel<6>, g, b, 0, stream); break;
    case 7: hipLaunchKernelGGL(ddt_signal_kernel<7>, g, b, 0, stream); break;
    case 8: hipLaunchKernelGGL(ddt_signal_kernel<8>, g, b, 0, stream); break;
    case 9: hipLaunchKernelGGL(ddt_signal_kernel<9>, g, b, 0, stream); break;
    case 10: hipLaunchKernelGGL(ddt_signal_kernel<10>, g, b, 0, stream); break;
    case 11: hipLaunchKernelGGL(ddt_signal_kernel<11>, g, b, 0, stream); break;
    case 12: hipLaunchKernelGGL(ddt_signal_kernel<12>, g, b, 0, stream); break;
    case 13: hipLaunchKernelGGL(ddt_signal_kernel<13>, g, b, 0, stream); break;
    case 14: hipLaunchKernelGGL(ddt_signal_kernel<14>, g, b, 0, stream); break;
    case 15: hipLaunchKernelGGL(ddt_signal_kernel<15>, g, b, 0, stream); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// ---------------------------------------------------------------- external32
// One thread per basic element of the type signature: locate the element's segment and
// run (binary searches over tiny tables), then move it between the native packed stream
// and the big-endian external32 stream (opal_copy_functions_heterogeneous.c semantics,
// see ddt_external.cpp).  DIR 0 = native -> external (pack), 1 = external -> native.
template <typename T> __device__ __forceinline__ T bswap(T v);
template <> __device__ __forceinline__ uint16_t bswap(uint16_t v) { return __builtin_bswap16(v); }
template <> __device__ __forceinline__ uint32_t bswap(uint32_t v) { return __builtin_bswap32(v); }
template <> __device__ __forceinline__ uint64_t bswap(uint64_t v) { return __builtin_bswap64(v); }

template <typename T>
__device__ __forceinline__ bool swap_words(const uint8_t *from, uint8_t *to, uint32_t n)
{
    if ((reinterpret_cast<uintptr_t>(from) | reinterpret_cast<uintptr_t>(to)) % sizeof(T))
        return false;
    for (uint32_t b = 0; b < n; b += sizeof(T))
        *reinterpret_cast<T *>(to + b) = bswap(*reinterpret_cast<const T *>(from + b));
    return true;
}

// A 2*sizeof(H)-byte component whose addresses are only sizeof(H)-aligned (an 8-byte double
// at offset 4 of a packed struct{int; double}): swap each half and exchange the halves.
template <typename H>
__device__ __forceinline__ bool swap_halves(const uint8_t *from, uint8_t *to, uint32_t n)
{
    if ((reinterpret_cast<uintptr_t>(from) | reinterpret_cast<uintptr_t>(to)) % sizeof(H))
        return false;
    for (uint32_t b = 0; b < n; b += 2 * sizeof(H)) {
        const H lo = *reinterpret_cast<const H *>(from + b), hi = *reinterpret_cast<const H *>(from + b + sizeof(H));
        *reinterpret_cast<H *>(to + b) = bswap(hi);
        *reinterpret_cast<H *>(to + b + sizeof(H)) = bswap(lo);
    }
    return true;
}

// One long double component (the external stream is byte aligned: bytewise access).
// Pack: x87 80-bit -> IEEE quad, exact (libgcc __extendxftf2 semantics: the explicit bit is
// dropped unchecked, a NaN is quieted).  A pseudo-denormal (exponent 0, explicit bit set) has
// no single reference answer -- the same libgcc conversion gives exponent 0 on the Intel
// container and exponent 1 on the GPU box's host -- so it becomes the value it denotes.  Unpack: quad -> x87 rounded to nearest even (__trunctfxf2), then the
// reference's in-place store: value bytes 0..9, bytes 10..15 keep the quad's.
template <int DIR>
__device__ __forceinline__ void convert_ldbl(const uint8_t *from, uint8_t *to)
{
    constexpr uint64_t TOP = 1ull << 63, QBIT = 1ull << 62, M63 = TOP - 1;
    if (DIR == 0) {
        uint64_t m = 0;
        for (int k = 0; k < 8; ++k)
            m |= uint64_t(from[k]) << (8 * k);
        const uint32_t se = uint32_t(from[8]) | (uint32_t(from[9]) << 8);
        const uint64_t sign = se >> 15;
        uint64_t e = se & 0x7FFF, f = m & M63;   // 63 fraction bits
        if (e == 0x7FFF && f)
            f |= QBIT;                           // NaN: quieted
        else if (e == 0 && (m & TOP))
            e = 1;                               // pseudo-denormal: the normal 1.f x 2^-16382 it denotes
        const uint64_t lo = f << 49, hi = (f >> 15) | (e << 48) | (sign << 63);
        for (int k = 0; k < 8; ++k) {
            to[k] = uint8_t(hi >> (8 * (7 - k)));
            to[8 + k] = uint8_t(lo >> (8 * (7 - k)));
        }
    } else {
        uint64_t hi = 0, lo = 0;
        for (int k = 0; k < 8; ++k) {
            hi = (hi << 8) | from[k];
            lo = (lo << 8) | from[8 + k];
        }
        const uint64_t sign = hi >> 63;
        uint64_t e = (hi >> 48) & 0x7FFF;
        const uint64_t fh = hi & ((1ull << 48) - 1);
        const uint64_t f63 = (fh << 15) | (lo >> 49), rest = lo & ((1ull << 49) - 1);
        uint64_t m;
        if (e == 0x7FFF) {
            m = (fh | lo) ? (TOP | QBIT | f63) : TOP;
        } else {
            m = (e ? TOP : 0) | f63;
            const uint64_t half = 1ull << 48;
            if (rest > half || (rest == half && (m & 1))) {
                ++m;
                if (m == 0) {                    // carried out of a normal: next binade
                    m = TOP;
                    ++e;
                } else if (e == 0 && m == TOP) { // a denormal rounded up to the smallest normal
                    e = 1;
                }
            }
            if (e == 0x7FFF)
                m = TOP;                         // rounded past the largest finite: infinity
        }
        for (int k = 0; k < 8; ++k)
            to[k] = uint8_t(m >> (8 * k));
        const uint32_t se = uint32_t((sign << 15) | e);
        to[8] = uint8_t(se);
        to[9] = uint8_t(se >> 8);
        for (int k = 10; k < 16; ++k)
            to[k] = uint8_t(hi >> (8 * (k - 8)));
    }
}

template <int DIR>
__device__ __forceinline__ void convert_elem(const ConvRun &r, const uint8_t *from, uint8_t *to)
{
    if (r.kind == CONV_LDBL) {
        for (uint32_t b = 0; b < r.nsz; b += 16)
            convert_ldbl<DIR>(from + b, to + b);
        return;
    }
    if (r.kind == CONV_LONG || r.kind == CONV_ULONG) {
        // external 4 big-endian bytes <-> native 8 little-endian bytes
        for (int k = 0; k < 4; ++k)
            to[k] = from[3 - k];
        if (DIR == 1) {
            const uint8_t fill = (r.kind == CONV_LONG && (from[0] & 0x80)) ? 0xFF : 0x00;
            for (int k = 4; k < 8; ++k)
                to[k] = fill;
        }
        return;
    }
    const uint32_t n = r.nsz;
    if (r.kind == CONV_COPY || r.comp == 1) {
        for (uint32_t b = 0; b < n; ++b)
            to[b] = from[b];
        return;
    }
    const uint32_t c = r.comp;
    if (c == 8 && swap_words<uint64_t>(from, to, n)) return;
    if (c == 8 && swap_halves<uint32_t>(from, to, n)) return;
    if (c == 4 && swap_words<uint32_t>(from, to, n)) return;
    if (c == 4 && swap_halves<uint16_t>(from, to, n)) return;
    if (c == 2 && swap_words<uint16_t>(from, to, n)) return;
    for (uint32_t base = 0; base < n; base += c)
        for (uint32_t k = 0; k < c; ++k)
            to[base + k] = from[base + c - 1 - k];
}

// General conversion: one thread per element.  The segment/run tables are staged in LDS
// when they fit (TAB): every element reads a segment (64 B) and a run (40 B) plus the
// binary-search keys, which from global memory cost more vector loads than the element.
template <int DIR, bool TAB>
__global__ __launch_bounds__(THREADS) void ddt_ext_kernel(const ConvSeg *__restrict__ gsegs, uint32_t nseg,
                                                          const ConvRun *__restrict__ gruns, uint32_t nruns,
                                                          uint64_t E, uint64_t total, uint64_t Sn,
                                                          uint64_t Se, uint8_t *native, uint8_t *ext)
{
    extern __shared__ uint64_t tab[];
    const ConvSeg *segs = gsegs;
    const ConvRun *runs = gruns;
    if (TAB) {
        constexpr uint32_t SW = sizeof(ConvSeg) / 8, RW = sizeof(ConvRun) / 8;
        const uint64_t *gs = reinterpret_cast<const uint64_t *>(gsegs), *gr = reinterpret_cast<const uint64_t *>(gruns);
        for (uint32_t i = threadIdx.x; i < nseg * SW; i += THREADS)
            tab[i] = gs[i];
        for (uint32_t i = threadIdx.x; i < nruns * RW; i += THREADS)
            tab[nseg * SW + i] = gr[i];
        __syncthreads();
        segs = reinterpret_cast<const ConvSeg *>(tab);
        runs = reinterpret_cast<const ConvRun *>(tab + nseg * SW);
    }
    const uint64_t stride = uint64_t(gridDim.x) * THREADS;
    for (uint64_t g = uint64_t(blockIdx.x) * THREADS + threadIdx.x; g < total; g += stride) {
        const uint64_t inst = g / E, r = g - inst * E;
        uint32_t lo = 0, hi = nseg - 1;
        while (lo < hi) {
            const uint32_t mid = (lo + hi + 1) >> 1;
            if (segs[mid].e0 <= r) lo = mid; else hi = mid - 1;
        }
        const ConvSeg &s = segs[lo];
        const uint64_t local = r - s.e0;
        const uint64_t rep = local / s.body_elems, k = local - rep * s.body_elems;
        uint32_t a = s.run0, b = s.run0 + s.nruns - 1;
        while (a < b) {
            const uint32_t mid = (a + b + 1) >> 1;
            if (runs[mid].e0 <= k) a = mid; else b = mid - 1;
        }
        const ConvRun ru = runs[a];
        const uint64_t j = k - ru.e0;
        uint8_t *np = native + inst * Sn + s.nbase + rep * s.nbody + ru.noff + j * ru.nsz;
        uint8_t *ep = ext + inst * Se + s.ebase + rep * s.ebody + ru.eoff + j * ru.esz;
        if (DIR == 0) convert_elem<0>(ru, np, ep);
        else convert_elem<1>(ru, ep, np);
    }
}

// Uniform conversion: every element of the signature is a C-byte word swap (or a copy, C = 1)
// and native and external layouts coincide, so the stream is an array of C-byte words (all
// of MPI_DOUBLE, of MPI_FLOAT, ...).  16 bytes per lane where both ends are 16-byte aligned,
// then one byte per lane for the tail (or the whole stream when misaligned).  The swap is
// its own inverse: one kernel serves pack and unpack.
template <int C>
__device__ __forceinline__ uint32_t swap_in_word(uint32_t x)
{
    if (C == 4) return __builtin_bswap32(x);
    if (C == 2) return ((x & 0x00FF00FFu) << 8) | ((x >> 8) & 0x00FF00FFu);
    return x;
}

template <int C>
__global__ __launch_bounds__(THREADS) void ddt_ext_uniform_kernel(const uint8_t *__restrict__ from,
                                                                  uint8_t *__restrict__ to, uint64_t nvec,
                                                                  uint64_t nbytes)
{
    typedef unsigned int v4 __attribute__((ext_vector_type(4)));
    const uint64_t stride = uint64_t(gridDim.x) * THREADS, t0 = uint64_t(blockIdx.x) * THREADS + threadIdx.x;
    const v4 *f = reinterpret_cast<const v4 *>(from);
    v4 *o = reinterpret_cast<v4 *>(to);
    for (uint64_t i = t0; i < nvec; i += stride) {
        const v4 v = f[i];
        v4 w;
        if (C == 16) {
            w.x = __builtin_bswap32(v.w);
            w.y = __builtin_bswap32(v.z);
            w.z = __builtin_bswap32(v.y);
            w.w = __builtin_bswap32(v.x);
        } else if (C == 8) {
            w.x = __builtin_bswap32(v.y);
            w.y = __builtin_bswap32(v.x);
            w.z = __builtin_bswap32(v.w);
            w.w = __builtin_bswap32(v.z);
        } else {
            w.x = swap_in_word<C>(v.x);
            w.y = swap_in_word<C>(v.y);
            w.z = swap_in_word<C>(v.z);
            w.w = swap_in_word<C>(v.w);
        }
        o[i] = w;
    }
    for (uint64_t b = nvec * 16 + t0; b < nbytes; b += stride) {
        const uint64_t k = b % C;
        to[b] = from[b - k + (C - 1 - k)];
    }
}

hipError_t launch_ext(const ConvSeg *segs, uint32_t nseg, const ConvRun *runs, uint32_t nruns, uint64_t E,
                      uint64_t count, uint64_t Sn, uint64_t Se, void *native, void *ext, int dir,
                      uint32_t uniform, hipStream_t stream)
{
    const uint64_t total = E * count;
    if (total == 0 || nseg == 0)
        return hipSuccess;
    uint8_t *n8 = static_cast<uint8_t *>(native), *e8 = static_cast<uint8_t *>(ext);
    if (uniform) {
        const uint64_t nbytes = Sn * count;
        const uint8_t *from = dir == 0 ? n8 : e8;
        uint8_t *to = dir == 0 ? e8 : n8;
        const bool al = ((reinterpret_cast<uintptr_t>(from) | reinterpret_cast<uintptr_t>(to)) % 16) == 0;
        const uint64_t nvec = al ? nbytes / 16 : 0, work = nvec ? nvec : nbytes;
        uint64_t blocks = (work + THREADS - 1) / THREADS;
        if (blocks > (1u << 14))
            blocks = 1u << 14;   // 64 workgroups per CU, grid-stride beyond
        const dim3 grid{uint32_t(blocks)}, block{THREADS};
        switch (uniform) {
        case 16: hipLaunchKernelGGL(ddt_ext_uniform_kernel<16>, grid, block, 0, stream, from, to, nvec, nbytes); break;
        case 8: hipLaunchKernelGGL(ddt_ext_uniform_kernel<8>, grid, block, 0, stream, from, to, nvec, nbytes); break;
        case 4: hipLaunchKernelGGL(ddt_ext_uniform_kernel<4>, grid, block, 0, stream, from, to, nvec, nbytes); break;
        case 2: hipLaunchKernelGGL(ddt_ext_uniform_kernel<2>, grid, block, 0, stream, from, to, nvec, nbytes); break;
        case 1: hipLaunchKernelGGL(ddt_ext_uniform_kernel<1>, grid, block, 0, stream, from, to, nvec, nbytes); break;
        default: return hipErrorInvalidValue;
        }
        return hipGetLastError();
    }
    uint64_t blocks = (total + THREADS - 1) / THREADS;
    if (blocks > (1u << 16))
        blocks = 1u << 16;   // grid-stride beyond 16 M threads (64 waves per CU)
    const size_t tb = size_t(nseg) * sizeof(ConvSeg) + size_t(nruns) * sizeof(ConvRun);
    const bool tab = tb <= kExtTabLds;
    const size_t lds = tab ? tb : 0;
    const dim3 grid{uint32_t(blocks)}, block{THREADS};
    if (dir == 0) {
        if (tab) hipLaunchKernelGGL((ddt_ext_kernel<0, true>), grid, block, lds, stream, segs, nseg, runs, nruns, E, total, Sn, Se, n8, e8);
        else hipLaunchKernelGGL((ddt_ext_kernel<0, false>), grid, block, 0, stream, segs, nseg, runs, nruns, E, total, Sn, Se, n8, e8);
    } else {
        if (tab) hipLaunchKernelGGL((ddt_ext_kernel<1, true>), grid, block, lds, stream, segs, nseg, runs, nruns, E, total, Sn, Se, n8, e8);
        else hipLaunchKernelGGL((ddt_ext_kernel<1, false>), grid, block, 0, stream, segs, nseg, runs, nruns, E, total, Sn, Se, n8, e8);
    }
    return hipGetLastError();
}

}  // namespace ddt
