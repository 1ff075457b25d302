// ddt_plan.h -- plan compiler and kernel launch interface (internal).
#pragma once

#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include <hip/hip_runtime.h>

#include "ddt_core.h"

namespace ddt {

// Tuning knobs (environment DDT_NT / DDT_TASK_KB, or ddt_tune()): for A/B sweeps.
struct Tuning {
    int nt = -1;       // user-side non-temporal loads: -1 auto (off, use_nt), 0 off, 1 on
    long task_kb = 0;  // packed KiB per workgroup task: 0 = adaptive
    long interleave = 0;  // >0: interleave items in runs of this many tasks (pack, typed copy)
    long uinterleave = 256;  // the same for an unpack (-1: as `interleave`); see assign_tasks
    long slots = 1;       // argument-free launches of hot descriptor sets (ddt_move_slot_kernel); 0 off
    long slot_max_kb = 4096;  // ... for launches of at most this many packed KiB
    long sfloor = 2;      // sparse-gather task floor (4 units per lane): 0 pack, 1 unpack, 2 both, -1 off
    int policy = 1;       // task sizing: 0 = v0 (~6 K tasks), 1 = per-leaf passes
    int wt = -1;          // write-through (sc1) stores: -1 auto, 0 off, 1 sparse user side, 2 all
    long sorted = -1;     // address-ordered list engine: -1 auto, 0 off, n > 0 from n blocks up
    long spol = 0;        // address-ordered engine access policy bits (ddt_sorted.hip POL_*)
    int ptr = 1;          // 1: a reused inline descriptor set is launched by pointer; 0: always inline
    int xcd = -1;         // XCD-contiguous task slabs: -1 auto (line-dense affine items), 0 off, 1 all
    long xchunk = 0;      // tasks per XCD run for slab items: 0 = one slab per XCD
    int snt = -1;         // streaming leaves (U = 16, blocks >= 256 B): non-temporal loads and
                          // stores; -1 auto (blocks >= 64 KiB), 0 off, 1 on
    long spass = 1;       // task of a streaming leaf: this many unrolled workgroup passes
    long stask = 0;       // task of a streaming leaf in bytes (overrides spass; 0 = spass passes)
    int dense = -1;       // line-dense records through LDS (run_dense): -1 auto, 0 off, n > 0 n chunks per task
    int dsplit = 1;       // line-dense unpack: each task as two workgroups (dense_body SPLIT)
    int dfast = 1;        // single-item line-dense launches by value, a workgroup per chunk
                          // (ddt_dense1_kernel): bit 0 pack, bit 1 unpack
    int hostdirect = 3;   // pinned host iovecs moved by the kernel itself over PCIe (no HBM
                          // staging): bit 0 unpack, bit 1 pack (end to end)
    long stage_mb = 256;  // HBM staging buffer (one per convertor) for pageable host iovecs: the
                          // largest piece of a host window moved in one kernel/copy overlap
    long hd_grid = 256;   // workgroup cap of an unpack launch reading pinned host memory (0 = none):
                          // PCIe reads lose rate to thousands of workgroups, writes do not
                          // (scripts/ubench_pcie.hip, profiles/r2_ubench_pcie.log)
    long hd_grid_pack = 0;   // the same cap for a pack writing pinned host memory
    long sunroll = 16;    // address-ordered engine: pack 1 elements per thread in flight (4, 8, 16)
    long s2unroll = 8;    // the same for its unpack pass 2' 
    long sigsync = 1;     // synchronous calls complete on the signal kernel's host word (r6); 0: hipStreamSynchronize
    long sigspin_us = 20000;  // ... spinning at most this long before blocking in hipStreamSynchronize
    long s2vec = 1;       // address-ordered engine, 4-byte elements: pass 2 / 2' four slots per lane (r6)
    long sskew = 4160;    // address-ordered engine: bytes of U between buckets, read at build (r6:
                          // 128 KiB-apart buckets camped on one DRAM channel; cfg4 pack 620 -> 585 us)
    long slayout = 1;     // address-ordered engine: chunk-major U for the pack (1) / the unpack (2) (r6:
                          // cfg4 pack 586 -> 514 us; the unpack's scattered run writes lose, 737 -> 871+)
    long sstagger = 0;    // address-ordered engine: pass 1 / 1' first-wave stagger, s_sleep(127) units (r6 A/B)
    long sseg = 1;        // address-ordered engine: U run padding, read at plan build: 1 = none (runs end
                          // to end, pass-1 chunks in XCD slabs; r5) or whole 32/64/128-byte segments
    long schunk = 1;      // address-ordered engine: 2 = half-size chunks, two pass-1 workgroups per
                          // CU (read at plan build)
    int sorted_commit = 1;   // build the address-ordered tables at commit / bridge import (1) or
                             // at the first whole-message move (0)
    // The commit optimizer's run-time parameters, read at commit like the reference's MCA
    // variables opal_datatype_optimize_{max_desc_growth, loop_unroll_max_items,
    // loop_unroll_max_data_bytes, preserve_type} (opal_datatype_module.c:85-90, :347-383); their
    // environment form OMPI_MCA_opal_datatype_optimize_* sets the initial values
    long opt_growth = 10;         // clamped to 1024 (OPAL_DATATYPE_OPTIMIZE_MAX_DESC_GROWTH_CAP)
    long opt_unroll_items = 8;
    long opt_unroll_bytes = 128;
    int opt_preserve = 1;         // 0: fused mixed-type regions travel as UINT1 (:586-588)
    // MCA ompi_datatype_consolidate_threshold (ompi_datatype_module.c:527-532; environment
    // OMPI_MCA_datatype_consolidate_threshold): the count from which ddt_type_consolidate builds
    // the MPI_Pack / MPI_Unpack consolidated type (pack.c.in:118-125)
    long consolidate = 250;
};
Tuning &tuning();
Tuning tuning_defaults();   // the defaults with the environment's DDT_* / OMPI_MCA_* values applied
// Synchronous host -> device copy on a library-private stream (capture-safe).
hipError_t upload(void *dst, const void *src, size_t n);
// While one lives, this thread's stream-capture mode is relaxed: the event queries, allocations
// and private-stream waits of descriptor uploads and slot binds are then this thread's own
// business and leave another thread's global-mode capture intact
// (profiles/r5_probe_capture.log); device-wide waits stay off (PoolNoDeviceSync).
struct RelaxedCapture {
    hipStreamCaptureMode mode = hipStreamCaptureModeRelaxed;
    bool swapped;
    RelaxedCapture() : swapped(hipThreadExchangeStreamCaptureMode(&mode) == hipSuccess) { (void) hipGetLastError(); }
    ~RelaxedCapture()
    {
        if (swapped)
            (void) hipThreadExchangeStreamCaptureMode(&mode);
    }
    RelaxedCapture(const RelaxedCapture &) = delete;
    RelaxedCapture &operator=(const RelaxedCapture &) = delete;
};
// The library-private non-blocking stream of the current device (uploads, table builds).
hipError_t private_stream(hipStream_t *out);

void build_items(const ddt_datatype *t, const Plan &P, uint64_t count, uint64_t user, uint64_t pk,
                 uint64_t W0, uint64_t W1, bool same_layout, std::vector<Item> &items);
// Task sizes and order of a launch's items; dir 1 (unpack) interleaves by tuning().uinterleave.
void assign_tasks(std::vector<Item> &items, int dir = 0);
long interleave_of(int dir);
// Launch-level cache policy of streaming items (see ddt_plan.cpp).
void stream_policy(std::vector<Item> &items);
// The address-ordered engine of plan P for a whole-message pack/unpack, built on first use;
// null when the plan does not qualify (or `user` is misaligned for it).
SortedList *sorted_plan(const ddt_datatype *t, Plan &P, uint64_t user, hipStream_t stream);
// XCD-contiguous task mapping for this item (Item::slab; tuning().xcd)
bool use_slab(const Item &it);
uint32_t total_tasks(const std::vector<Item> &items);

// ddt_kernels.hip: dir 0 = pack / typed copy (user side -> packed side), 1 = unpack.
// grid_cap > 0: at most that many workgroups, looping over the tasks (host-direct windows);
// dense: every item is line-dense (Item::nbytes), run by the dedicated dense kernel
hipError_t launch_move_inline(const ItemBlock &blk, uint32_t ntasks, int dir, bool lists, uint64_t ubase,
                              uint64_t pbase, hipStream_t stream, uint32_t grid_cap = 0, bool dense = false);
bool launch_single_item(const Item &it, int dir, uint64_t ubase, uint64_t pbase, hipStream_t stream,
                        hipError_t *err);
hipError_t launch_move(const Item *d_items, uint32_t nitems, uint32_t ntasks, int dir, bool lists,
                       uint64_t ubase, uint64_t pbase, hipStream_t stream, uint32_t grid_cap = 0,
                       bool dense = false);
// The argument-free launch of slot k's record (grid = ntasks) and the device address of a kernel
// family's record table (current device).
hipError_t launch_move_slot(int dir, uint32_t k, uint32_t ntasks, hipStream_t stream);
hipError_t slot_table(int dir, void **addr);
// Launches the slot-index probe of direction dir on `stream`: d_out[k] = the index a slot launch
// of record k decodes (k < NSLOT), d_out[NSLOT] = what a launch without slot LDS decodes (NSLOT).
hipError_t slot_probe(int dir, uint32_t *d_out, hipStream_t stream);
// Completion signal of synchronous calls (ddt_kernels.hip): kSigSlots argument-free signal
// kernels; signal_setup points the current device's kernels at a pinned host page (one 64-byte
// line per slot), launch_signal enqueues slot k's kernel.
constexpr int kSigSlots = 16;
constexpr int kSigStride = 16;   // uint32 words between slots
hipError_t signal_setup(uint32_t *host_page, hipStream_t s);
hipError_t launch_signal(int k, hipStream_t stream);
// Launch slots (ddt_plan.cpp; affine launches only).  slot_bind: a free slot of direction `dir`
// on device `dev` whose last binding's launches have passed, with `rec` written into it
// (uploaded and waited for on the private stream) and its generation in *gen, or -1 (then a
// binding idle for long may have been ended for the next try).  slot_launch: the argument-free
// launch of slot k if binding `gen` still holds it (false: launch with arguments).
// slot_release: binding `gen` ends; the slot is free once `fence_streams` (null: none) pass
// the events recorded now.
int slot_bind(int dev, int dir, const LaunchRec &rec, uint32_t *gen);
bool slot_launch(int dev, int dir, int k, uint32_t gen, uint32_t ntasks, hipStream_t stream, hipError_t *err);
void slot_release(int dev, int dir, int k, uint32_t gen, const std::vector<hipStream_t> *fence_streams);
// every binding ends behind fences on its streams (ddt_trim)
void slot_trim();
// out4 = [pack slots bound on dev, unpack slots bound, binds so far, argument-free launches so far]
void slot_stats(int dev, int64_t *out4);
// bit 0 bound, bit 1 ending, bits 8.. streams of the binding; -1: no such family (ddt_slot_state)
int slot_debug_state(int dev, int dir, int k);

// external32 conversion between a native packed stream and its big-endian form.
// uniform = C in {1,2,4,8,16}: every element is a C-byte word swap (C = 1: a copy) with identical native
// and external layouts -- one vectorised word-swap pass instead of the per-element walk.
// Tables of at most kExtTabLds bytes are staged in LDS by the per-element kernel.
constexpr size_t kExtTabLds = 32 << 10;
hipError_t launch_ext(const ConvSeg *segs, uint32_t nseg, const ConvRun *runs, uint32_t nruns, uint64_t E,
                      uint64_t count, uint64_t Sn, uint64_t Se, void *native, void *ext, int dir,
                      uint32_t uniform, hipStream_t stream);

// ddt_external.cpp: the external32 signature of a committed type (built once, cached).
struct ExtPlan {
    std::vector<ConvSeg> segs;
    std::vector<ConvRun> runs;
    uint64_t E = 0;      // elements per instance
    uint64_t Se = 0;     // external bytes per instance
    uint32_t uniform = 0;   // C when the whole signature is C-byte word swaps (see launch_ext)
    ConvSeg *d_segs = nullptr;
    ConvRun *d_runs = nullptr;
    int error = 0;       // DDT_ERR_* when the type has no external32 form
    std::string what;
    ~ExtPlan();
};
std::shared_ptr<ExtPlan> get_ext_plan(ddt_datatype *t);
int ext_upload(ExtPlan &X);

}  // namespace ddt
