// ddt_device.h -- launch descriptors shared by the host plan compiler and the
// gfx950 kernels (ddt_move.hip.h, ddt_kernels.hip).  Plain-old-data only.
#pragma once

#include <cstdint>

#ifndef __HIPCC__
#define DDT_HD inline
#else
#define DDT_HD __host__ __device__ inline
#endif

namespace ddt {

constexpr int MAXD = 8;             // affine dims per item, instance dim included
constexpr int THREADS = 256;        // workgroup size (4 wave64)
constexpr uint32_t SLAB_FULL = 0xffffffffu;
// units each thread loads before storing, per pass of the affine loop
constexpr int unroll_of(uint32_t U) { return U >= 16 ? 4 : 8; }
// user-span bytes a workgroup stages in LDS per task of the line-dense path (run_dense)
constexpr uint32_t DENSE_LDS = 4096;

enum LeafKind : int { LEAF_AFFINE = 0, LEAF_LIST = 1 };

enum ItemKind : uint32_t {
    ITEM_AFFINE = 0,    // units of U bytes over an affine nest
    ITEM_LIST_UNI = 1,  // units of U bytes over an index list with one block length
    ITEM_LIST_VAR = 2,  // one wave per 64-block group of a variable-length index list
    ITEM_FRAG = 3,      // a sub-unit byte fragment at a window edge
};

// Exact unsigned 32-bit division by an invariant divisor d >= 1:
//   l = ceil(log2 d), m = floor(2^32 (2^l - d) / d) + 1,
//   n / d = (umulhi(n, m) + n) >> l      for every n < 2^32.
struct FastDiv {
    uint32_t d = 1, m = 1, l = 0, pad = 0;
};

DDT_HD FastDiv make_fastdiv(uint32_t d)
{
    FastDiv f;
    f.d = d;
    uint32_t l = 0;
    while (l < 32 && (uint64_t(1) << l) < d) ++l;
    f.l = l;
    f.m = uint32_t(((uint64_t(1) << 32) * ((uint64_t(1) << l) - d)) / d + 1);
    return f;
}

DDT_HD uint32_t fastdiv(uint32_t n, const FastDiv &f)
{
#ifdef __HIP_DEVICE_COMPILE__
    uint32_t hi = __umulhi(n, f.m);
#else
    uint32_t hi = uint32_t((uint64_t(n) * f.m) >> 32);
#endif
    return uint32_t((uint64_t(hi) + n) >> f.l);
}

struct Item {
    uint32_t kind;
    uint32_t U;             // unit bytes: 1, 2, 4, 8, 16
    uint32_t ndim;          // dims in use (outer -> inner), instance dim first
    uint32_t idx64;         // 1: total units >= 2^32, use 64-bit index arithmetic
    uint64_t u0, u1;        // unit range [u0, u1) of this item
    uint64_t units_per_task;
    uint32_t task_begin;    // first workgroup of this item
    uint32_t ntasks;
    uint64_t upb;           // units per block (affine / list-uniform)
    FastDiv fd_upb;
    uint64_t user;          // user-side address, relative to the launch's user base
    uint64_t packed;        // packed-side address, relative to the launch's packed base
    uint64_t cnt[MAXD];
    FastDiv fd[MAXD];
    int64_t ustr[MAXD];     // user-side stride per dim (bytes)
    int64_t pstr[MAXD];     // packed-side stride per dim (bytes)
    // index lists
    uint64_t ldisp;         // device pointer: int32 or int64 displacement per block
    uint64_t llen;          // device pointer: uint32 length per block (LIST_VAR)
    uint64_t lgoff;         // device pointer: uint64 packed offset per 64-block group (LIST_VAR)
    uint64_t nblk;          // blocks in the list
    FastDiv fd_nblk;
    uint64_t ulen;          // uniform block bytes (LIST_UNI)
    uint32_t ldisp32;       // displacement array is int32
    uint32_t leaf;          // plan leaf this item belongs to (diagnostics)
    uint32_t same;          // typed copy: the packed side uses the user-side layout too
    uint32_t nt;            // user-side accesses non-temporal (sparse gathers over > MALL spans)
    int64_t w0, w1;         // LIST_VAR / FRAG: window [w0, w1) in packed-stream coordinates
    uint64_t nbytes;        // FRAG: bytes.  AFFINE: records per task of the line-dense path
                            // (run_dense, LDS-staged whole-line accesses), 0 = the unit loop
    uint32_t wt;            // store policy: 1 = user-side stores (unpack) write through L2 (sc1);
                            // 2 = every store of the launch sc1; 3 = user-side stores of an
                            // unpack non-temporal (affine leaves)
    uint32_t slab;          // XCD task mapping (move_body): 0 round-robin, SLAB_FULL one
                            // contiguous slab per XCD, else runs of `slab` tasks per XCD;
                            // keeps sizeof(Item) == 512
};

// Descriptors passed by value in the kernel-argument segment (<= 4 KiB).
constexpr uint32_t INLINE_ITEMS = 7;
// Kernel-argument block of NI descriptors: the launch copies only sizeof(ItemBlockN<NI>)
// bytes of arguments, so a one-leaf type pays for 528 B, not 3.6 KB.
template <uint32_t NI>
struct ItemBlockN {
    uint32_t n;
    uint32_t ntasks;        // tasks of the launch (a capped grid loops over them)
    uint64_t ubase, pbase;  // the launch's base pointers (Item::user / Item::packed are relative)
    uint64_t pad2;
    Item items[NI];
};
using ItemBlock = ItemBlockN<INLINE_ITEMS>;
static_assert(sizeof(Item) == 512, "Item layout is shared with tests/plan_emu.py");
static_assert(sizeof(ItemBlock) <= 4096, "kernel argument segment limit");

// One affine item's fields passed BY VALUE in the kernel arguments (~170 bytes: one batch of
// scalar loads, no descriptor pointer to chase): the single-item line-dense launch of
// ddt_dense1_kernel (launch_single_item, ddt_kernels.hip).
struct ItemArgs {
    uint64_t ubase, pbase;      // user / packed address of the item's unit 0
    uint32_t u0, u1;            // unit range of the item
    uint32_t cu, nd;            // units per workgroup (dense: one chunk of R records); dims in use
    FastDiv fdu, fw;            // units per block; (dense) 4-byte words per record
    uint32_t nt, pad;           // Item::nt
    uint32_t cnt[4];
    FastDiv fd[4];
    int64_t ustr[4], pstr[4];
};
constexpr uint32_t ITEM_ARG_DIMS = 4;

// The launch record of an argument-free move launch (ddt_move.hip.h, ddt_move_slot_kernel):
// NSLOT records per (direction, lists) kernel family per device, bound by the host to hot
// descriptor sets on fixed buffers (ddt_plan.cpp: slot_bind).  Record k is served by slot
// kernel k / SLOT_PER_KERNEL, launched with ((k % SLOT_PER_KERNEL) + 1) x SLOT_LDS_UNIT bytes of
// dynamic LDS, which the kernel (static LDS 0) reads back from the hardware register
// HW_REG_LDS_ALLOC -- no memory access (r6: two kernels per direction serve 32 records; r5 had one
// inlined kernel per record, 8 per direction; reading the dispatch packet instead costs 14 us
// per launch, profiles/r6_ldsprobe.log).  SLOT_LDS_UNIT is gfx950's LDS allocation granule
// (1280 bytes: LDS_SIZE counts 256-byte units in steps of 5); at most 16 x 1280 = 20 KiB, so
// eight 256-thread workgroups still fit a CU's 160 KiB.
constexpr uint32_t NSLOT = 32;
constexpr uint32_t SLOT_PER_KERNEL = 16;
constexpr uint32_t SLOT_LDS_UNIT = 1280;
struct LaunchRec {
    uint64_t items;    // const Item * in device memory
    uint64_t ubase, pbase;
    uint32_t nitems, ntasks;
};

// ---- external32 conversion (ddt_external.cpp, ddt_ext_kernel) ----
// CONV_LDBL: each 16-byte component x87 80-bit (native) <-> IEEE quad big-endian (external)
enum ConvKind : uint32_t { CONV_COPY = 0, CONV_SWAP = 1, CONV_LONG = 2, CONV_ULONG = 3, CONV_LDBL = 4 };

// `n` consecutive elements of one basic type inside a segment body.
struct ConvRun {
    uint64_t e0;            // index of the first element within the body
    uint64_t noff, eoff;    // byte offset of the first element in the body: native / external
    uint32_t nsz, esz;      // element bytes: native / external
    uint32_t comp;          // byte-swap unit (component size for complex types)
    uint32_t kind;          // ConvKind
};

// `reps` repetitions of a body of runs, consecutive in both streams.
struct ConvSeg {
    uint64_t e0;            // index of the first element within one instance
    uint64_t reps, body_elems;
    uint64_t nbase, ebase;  // byte offset of the segment within one instance
    uint64_t nbody, ebody;  // bytes per repetition
    uint32_t run0, nruns;
};

}  // namespace ddt
