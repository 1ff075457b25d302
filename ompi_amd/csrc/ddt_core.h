// ddt_core.h -- host-side type map, commit normalisation and device plan for the
// MI355X derived-datatype engine.  Internal to libddt_hip.so.
//
// The type map is kept as a tree that mirrors the committed Open MPI description
// (opal_datatype_internal.h:119-160): DATA entries (count blocks of blen bytes,
// stride extent, first block at disp) and LOOP entries (loops iterations of a body,
// stride extent).  A third node kind, LIST, is a compact run of single-block DATA
// entries produced by the indexed constructors (the reference stores one 32-byte
// DATA entry per block: 1 GiB of opt_desc for 64 M blocks).
#pragma once

#include <atomic>
#include <cstddef>
#include <cstdint>
#include <map>
#include <memory>
#include <sched.h>
#include <mutex>
#include <vector>

#include <hip/hip_runtime.h>

#include "ddt_device.h"
#include "ddt_sorted.h"

namespace ddt {

// A lock for short critical sections taken on every pack / unpack call (a plan's descriptor
// cache, a type's plan table, a launch slot): it spins briefly, then yields, and never parks the
// thread in the kernel.  Under MPI_THREAD_MULTIPLE threads sharing one datatype take its plan's
// lock several times per call; a futex-based mutex convoyed there (r6, scripts/bridgethreads.c
// shared: 8 threads 31.7 us per call, profiles/r6_threads.jsonl).
class SpinMutex {
public:
    void lock()
    {
        for (unsigned spins = 0; flag_.exchange(true, std::memory_order_acquire);) {
            while (flag_.load(std::memory_order_relaxed)) {
                if (++spins < 2048)
                    __builtin_ia32_pause();
                else
                    sched_yield();   // the holder is descheduled or in a long section (an upload)
            }
        }
    }
    bool try_lock() { return !flag_.exchange(true, std::memory_order_acquire); }
    void unlock() { flag_.store(false, std::memory_order_release); }

private:
    std::atomic<bool> flag_{false};
};


enum : uint32_t {
    F_PREDEFINED = 0x0002u,
    F_COMMITTED = 0x0004u,
    F_OVERLAP = 0x0008u,
    F_CONTIGUOUS = 0x0010u,
    F_NO_GAPS = 0x0020u,
    F_USER_LB = 0x0040u,
    F_USER_UB = 0x0080u,
    F_DATA = 0x0100u,
};

// LP64 x86-64 sizes of opal_datatype_local_sizes (opal_datatype_module.c:143-180) and natural
// alignment (opal_datatype_constructors.h:87-96), by OPAL predefined id.
inline constexpr int64_t kOpalSize[29] = {0, 0, 0, 0, 1, 2, 4, 8, 16, 1, 2, 4, 8, 16, 2,
                                          4, 8, 16, 16, 4, 8, 16, 32, 1, 4, 8, 8, 32, 0};
inline constexpr int64_t kOpalAlign[29] = {0, 0, 0, 0, 1, 2, 4, 8, 16, 1, 2, 4, 8, 16, 2,
                                           4, 8, 16, 16, 2, 4, 8, 16, 1, 4, 8, 8, 16, 0};

// Element boundaries inside one block of a merged mixed-type DATA run: the element
// start offsets within one period.  Null pattern = every multiple of esize.
struct Pattern {
    uint64_t period = 0;
    std::vector<uint32_t> starts;  // sorted, starts[0] == 0
};

struct IndexList {
    std::vector<int64_t> disp;   // byte displacement of each block (before Node::disp shift)
    std::vector<uint64_t> len;   // bytes of each block; empty => all blocks are `ulen`
    uint64_t ulen = 0;
    int64_t esize = 1;
    // derived at commit
    std::vector<uint64_t> poff;  // packed offset of each block (variable lengths only)
    uint64_t total = 0;          // packed bytes of the whole list
    int64_t min_disp = 0, max_end = 0;
    uint64_t disp_gcd = 0;       // gcd of all displacements (alignment of the gather side)
    uint64_t len_gcd = 0;
    size_t nblk() const { return disp.size(); }
};

struct Node {
    enum Kind : uint8_t { DATA, LOOP, LIST } kind = DATA;
    int64_t esize = 1;      // DATA/LIST: basic element size
    uint16_t tid = 0;       // DATA/LIST: OPAL id of the elements (0 = mixed, after commit merges)
    uint64_t count = 1;     // DATA: blocks; LOOP: iterations
    uint64_t blen = 0;      // DATA: bytes per block
    int64_t extent = 0;     // DATA: block stride; LOOP: iteration stride
    int64_t disp = 0;       // DATA: first block displacement; LIST: shift for every block
    uint32_t flags = 0;     // uncommitted form: the entry's Open MPI flags (DATA/LIST: the element's,
                            // LOOP: the repeated type's, opal_datatype_add.c:328-343, :406-409)
    std::vector<Node> body; // LOOP
    uint64_t body_size = 0; // LOOP: packed bytes per iteration (== END_LOOP size)
    std::shared_ptr<const IndexList> list;  // LIST
    std::shared_ptr<const Pattern> pat;     // DATA merged from mixed element sizes
    uint64_t packed_bytes() const;
};

// One affine "leaf stream" of the plan: blocks of blen bytes whose source address is
// src_off + sum_j idx_j*sstr_j and packed offset dst_off + sum_j idx_j*dstr_j, with
// idx_j in [0, cnt_j).  dims are ordered outer -> inner; packed offsets are monotone
// in the lexicographic order of idx (type-map order).
struct LeafDim {
    uint64_t cnt;
    int64_t sstr;
    int64_t dstr;
};

struct Leaf {
    int kind = LEAF_AFFINE;       // LEAF_AFFINE or LEAF_LIST
    uint64_t blen = 0;            // affine: bytes per block
    int64_t src_off = 0;
    int64_t dst_off = 0;
    std::vector<LeafDim> dims;    // outer -> inner (without the instance dim)
    std::shared_ptr<const IndexList> list;  // LEAF_LIST
    int64_t list_shift = 0;
    uint64_t bytes_per_iter = 0;  // packed bytes of the leaf per iteration of the dims (blen or list total)
};

struct DevList {                  // device copy of an IndexList
    void *disp = nullptr;         // int32 or int64 per block (relative to min_disp when 32-bit)
    uint32_t *len = nullptr;      // variable lengths
    uint64_t *goff = nullptr;     // packed offset of every 64-block group (variable lengths)
    bool disp32 = false;
    int64_t disp_base = 0;
};

// Launch descriptors of one (count, buffers, windows) request, resident in HBM.
// Repeated requests (the halo-exchange pattern: same type, same buffers every
// iteration) reuse them with no host work and no upload.
// Items hold addresses relative to the launch's two bases (16-byte aligned), so the key is
// the request's shape and alignment only: a double-buffered halo, a staged pipeline's HBM
// slots or a PML fragment stream reuse one set across buffers.
struct alignas(128) ItemSet {   // written on every call: a line of its own (r6)
    std::vector<uint64_t> key;
    std::vector<Item> items;
    Item *d_items = nullptr;
    uint32_t ntasks = 0;
    uint64_t bytes = 0;           // packed bytes the launch moves
    bool has_lists = false;
    bool all_dense = false;       // every item line-dense: the dense kernel runs the launch
    bool inline_ok = false;       // <= INLINE_ITEMS: launched from the kernarg segment
    uint32_t uses = 0;            // launches so far; a reused inline set is uploaded once and
                                  // launched by pointer (see run_windows)
    bool pinned = false;          // launched by pointer inside a stream capture: a graph holds
                                  // d_items, so it lives as long as the plan
    std::vector<hipStream_t> streams;  // streams that launched d_items (retirement events)
    // A launch by pointer is enqueued outside the plan lock: `inflight` counts launches
    // between taking d_items and enqueuing them, and a launch that finds the set evicted
    // meanwhile records a `late` event behind itself for the retirement to wait on too.
    std::atomic<uint32_t> inflight{0};   // raised under the plan lock; lowered without it unless retired
    std::atomic<bool> retired{false};
    std::vector<hipEvent_t> late;
    ItemBlock blk{};
    // argument-free launches (run_windows): up to kSetBind launch-slot bindings, each for one
    // direction and one pair of buffers (a double-buffered exchange alternates two; threads
    // sharing a type each bring theirs, r6), and the buffers of the kHist previous launches by
    // pointer (a set binds buffers seen again within them)
    static constexpr int kSetBind = 8, kHist = 8;
    struct Binding {
        int slot = -1;            // (dir << 8) | k, -1 none
        uint32_t gen = 0;
        uint64_t ubase = 0, pbase = 0;
        uint64_t used = 0;        // launches of the set when last used
    };
    Binding bind[kSetBind];
    int slot_dev = -1;
    uint64_t launches = 0;
    uint64_t bind_backoff = 0;    // no bind attempt before `launches` reaches this
    uint64_t hist_u[kHist], hist_p[kHist];
    uint32_t hist_at = 0;
    ItemSet()
    {
        for (int i = 0; i < kHist; ++i)
            hist_u[i] = hist_p[i] = ~0ull;
    }
    ~ItemSet();
};

// Device memory of retired descriptor sets, kept for reuse (hipFree implies a device-wide
// synchronisation; a destroyed plan hands its buffers to the pool, ddt_pool.h).
struct DevBlock {
    void *p = nullptr;
    size_t bytes = 0;
};

// An evicted descriptor set waits here until every stream that launched it has passed the
// event recorded at eviction (no device-wide synchronisation).
struct Retired {
    std::shared_ptr<ItemSet> set;
    std::vector<hipEvent_t> events;
};

struct ExtPlan;
struct DescForm;

struct alignas(128) Plan {
    std::vector<Leaf> leaves;
    std::vector<DevList> dev;     // one per LIST leaf (index in Leaf order, others empty)
    uint64_t dev_bytes = 0;       // device metadata bytes
    std::atomic<bool> dev_ready{false};   // index lists uploaded (read without the lock)
    SpinMutex mu;
    std::atomic<int> device{-1};  // HIP device holding this plan's device state (first use)
    std::vector<std::shared_ptr<ItemSet>> cache;      // most recent first
    std::vector<Retired> graveyard;                   // evicted, freed once their events pass
    std::vector<std::shared_ptr<ItemSet>> pinned;     // evicted but held by captured graphs
    std::vector<DevBlock> spare;                      // reusable descriptor memory (recycled)
    std::vector<hipStream_t> streams;                 // every stream that launched this plan's work
    bool captured = false;                            // a launch was enqueued inside a capture
    // address-ordered plan of a one-leaf single-element index list (ddt_sorted.hip):
    // 0 = not tried yet, 1 = built, -1 = not applicable
    // (atomic: the commit hook or a bridge import may build it on one thread while another
    // thread's first move reads it)
    std::atomic<int> sorted_state{0};
    std::unique_ptr<SortedList> sorted;
    ~Plan();
};

}  // namespace ddt

uint64_t ddt_next_serial();   // ddt_typemap.cpp: process-unique datatype serial numbers

struct ddt_datatype {
    // process-unique, never reused (a convertor re-prepared with the datatype it already holds
    // keeps its plan: an address alone could belong to a destroyed type's successor)
    const uint64_t serial = ddt_next_serial();
    uint16_t id = 0;              // predefined OPAL id, 0 for derived
    uint32_t flags = ddt::F_CONTIGUOUS;
    int64_t size = 0;
    int64_t lb = INT64_MAX, ub = INT64_MIN;
    int64_t true_lb = INT64_MAX, true_ub = INT64_MIN;
    int64_t align = 1;
    uint64_t nbElems = 0;
    // opal_datatype_t::bdt_used (opal_datatype.h:175): one bit per predefined id the type map
    // holds, LB / UB markers included (opal_datatype_add.c:163,175,306)
    uint32_t bdt_used = 0;
    // opal_datatype_t::stack_depth after commit: the deeper LOOP nesting of desc and opt_desc
    // (opal_datatype_opt_update_stack_depth, opal_datatype_optimize.c:222-261, :1777)
    uint32_t stack_depth = 0;
    std::vector<ddt::Node> desc;  // type map (uncommitted form)
    std::vector<ddt::Node> opt;   // committed + normalised form
    bool imported = false;        // desc is already a committed opt_desc (ddt_type_from_opal_desc)
    uint32_t opt_flags = 0;       // OPAL_DATATYPE_OPTIMIZED_RESTRICTED after commit (ddt_optimize.h)
    std::vector<uint64_t> opt_prefix;  // packed offset of each top-level opt node
    ddt::SpinMutex plan_mu;
    // one plan per HIP device the type is moved on (index = device ordinal): a plan's descriptor
    // sets, lists and tables live in that device's HBM
    std::vector<std::shared_ptr<ddt::Plan>> plans;
    std::shared_ptr<ddt::ExtPlan> ext;   // external32 signature (lazy)
    // a consolidated type (ddt_type_consolidate): its opt_desc, built from the old type's
    // (opal_datatype_optimize_from_contiguous) rather than from its own desc
    std::shared_ptr<const ddt::DescForm> opt_form;
    int64_t extent() const { return ub - lb; }
};

namespace ddt {
// typemap.cpp
ddt_datatype *new_type();
int commit(ddt_datatype *t);
// Open MPI's opt_desc of a committed type, as ddt_optimize.cpp derives it (false: not expressible)
bool opt_desc_of(const ddt_datatype *t, DescForm &out);
void normalize(std::vector<Node> &nodes);
// Largest element boundary <= p (p in [0, count*size]) of the packed stream.
uint64_t snap_down_to_element(const ddt_datatype *t, uint64_t p);
// plan.cpp
std::shared_ptr<Plan> get_plan(ddt_datatype *t);
void ensure_device_lists(Plan &P);
// commit / import time device setup of the address-ordered engine (ddt_plan.cpp)
int prebuild_device(ddt_datatype *t);
}  // namespace ddt
