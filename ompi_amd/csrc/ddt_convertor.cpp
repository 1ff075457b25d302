// ddt_convertor.cpp -- convertor state machine, HIP execution and the C ABI of
// libddt_hip.so.
//
// Mirrors opal_convertor_t semantics (opal/datatype/opal_convertor.h:125-170,
// opal_convertor.c:255-349, 526-696): prepare records (type, count, buffer) and
// the packed size; pack/unpack consume iovecs from the current position
// (bConverted) and return 1 once the whole message is converted.  Resume state is
// just bConverted: every window is recomputed from the packed position in O(leaves)
// (the reference keeps a descriptor stack, opal_convertor.h:111-117, and walks to
// it in opal_convertor_generic_simple_position, opal_datatype_position.c:167-367).
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <string>

#include <hip/hip_runtime.h>

#include "ddt_core.h"
#include "ddt_hip.h"
#include "ddt_plan.h"
#include "ddt_pool.h"

using namespace ddt;

namespace {

thread_local std::string g_last_error;

int fail(int code, const std::string &msg)
{
    g_last_error = msg;
    return code;
}

#define HIPCHK(call)                                                                   \
    do {                                                                               \
        hipError_t _e = (call);                                                        \
        if (_e != hipSuccess)                                                          \
            return fail(DDT_ERR_HIP, std::string(#call) + ": " + hipGetErrorString(_e)); \
    } while (0)

enum MemKind { MEM_DEVICE, MEM_HOST };

MemKind classify(const void *p)
{
    hipPointerAttribute_t a;
    hipError_t e = hipPointerGetAttributes(&a, p);
    if (e != hipSuccess) {
        (void) hipGetLastError();
        return MEM_HOST;
    }
    if (a.type == hipMemoryTypeDevice || a.type == hipMemoryTypeManaged
        || a.type == hipMemoryTypeUnified || a.isManaged)
        return MEM_DEVICE;
    return MEM_HOST;
}

// Pinned (page-locked, device-mapped) host memory: the device address of [p, p + n), or 0
// for pageable memory, device memory or a range not inside ONE pinned allocation or
// registration.  On ROCm a pinned page's device address equals its host address, so matching
// ends would also accept a range running from one registration through unregistered pages
// into another, and the kernel would fault on the gap: the runtime's range attributes
// (start and size, reported for hipHostMalloc and hipHostRegister memory alike,
// scripts/probe_hostrange.cpp) decide.  Anything the runtime cannot describe is staged.
uint64_t pinned_device_range(const void *p, uint64_t n)
{
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void) hipGetLastError();
        return 0;
    }
    if (a.type != hipMemoryTypeHost || !a.devicePointer)
        return 0;
    const uint64_t d0 = uint64_t(uintptr_t(a.devicePointer));
    if (n == 0)
        return d0;
    void *start = nullptr;
    size_t size = 0;
    hipDeviceptr_t q = reinterpret_cast<hipDeviceptr_t>(const_cast<void *>(p));
    if (hipPointerGetAttribute(&start, HIP_POINTER_ATTRIBUTE_RANGE_START_ADDR, q) != hipSuccess
        || hipPointerGetAttribute(&size, HIP_POINTER_ATTRIBUTE_RANGE_SIZE, q) != hipSuccess || !start) {
        (void) hipGetLastError();
        return 0;
    }
    const uint64_t s0 = uint64_t(uintptr_t(start)), h = uint64_t(uintptr_t(p));
    return h >= s0 && n <= size && h - s0 <= size - n ? d0 : 0;
}

struct Window {
    uint64_t w0, w1;   // packed-stream byte range
    uint64_t ptr;      // device pointer holding byte w0
};

constexpr size_t kCacheEntries = 32;
constexpr size_t kRetiredMax = 64;
uint64_t stage_bytes() { return uint64_t(tuning().stage_mb) << 20; }   // host staging slot

bool capturing(hipStream_t s)
{
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(s, &cs) != hipSuccess) {
        (void) hipGetLastError();
        return true;   // unknown: treat as captured (the safe side: keep the memory)
    }
    return cs != hipStreamCaptureStatusNone;
}

// ---------------------------------------------------------------- synchronous completion
// A synchronous call returns once the device says its work is done.  HIP's own answer
// (hipStreamSynchronize) is a ~9.5 us round trip whatever the kernel; the engine instead enqueues
// a signal kernel (ddt_kernels.hip) behind the call's work and spins on the pinned host word it
// writes, falling back to hipStreamSynchronize when no signal slot is free, the stream captures,
// the setup failed, or the word does not arrive within kSigSpin (the work is long, or faulted:
// hipStreamSynchronize then reports the error).
struct SigDev {
    std::mutex mu;
    bool tried = false, ok = false;
    uint32_t *page = nullptr;                 // kSigSlots lines of a pinned host page
    std::atomic<uint32_t> busy{0};            // one bit per slot owned by a call
    uint32_t expect[kSigSlots] = {};          // the slot owner's count of its signals
};
std::atomic<int64_t> g_sig_fast{0}, g_sig_fallback{0}, g_sig_plain{0};

SigDev *sig_device()
{
    static SigDev devs[64];
    int d = 0;
    if (hipGetDevice(&d) != hipSuccess || d < 0 || d >= 64) {
        (void) hipGetLastError();
        return nullptr;
    }
    SigDev &D = devs[d];
    std::lock_guard<std::mutex> g(D.mu);
    if (!D.tried) {
        D.tried = true;
        void *p = nullptr;
        hipStream_t ps = nullptr;
        if (hipHostMalloc(&p, 4096, hipHostMallocMapped | hipHostMallocCoherent) == hipSuccess) {
            std::memset(p, 0, 4096);
            void *dp = nullptr;
            if (hipHostGetDevicePointer(&dp, p, 0) == hipSuccess && private_stream(&ps) == hipSuccess
                && signal_setup(static_cast<uint32_t *>(dp), ps) == hipSuccess) {
                D.page = static_cast<uint32_t *>(p);
                D.ok = true;
            }
        }
        (void) hipGetLastError();
    }
    return D.ok ? &D : nullptr;
}

hipError_t complete_sync(hipStream_t s, bool signal_ok)
{
    SigDev *D = (signal_ok && tuning().sigsync && !capturing(s)) ? sig_device() : nullptr;
    int k = -1;
    if (D) {
        uint32_t b = D->busy.load(std::memory_order_relaxed);
        while (k < 0 && b != (1u << kSigSlots) - 1u) {
            const int f = __builtin_ctz(~b);
            if (D->busy.compare_exchange_weak(b, b | (1u << f), std::memory_order_acquire))
                k = f;
        }
    }
    if (k < 0) {
        ++g_sig_plain;
        return hipStreamSynchronize(s);
    }
    const uint32_t want = ++D->expect[k];
    hipError_t e = launch_signal(k, s);
    if (e != hipSuccess) {
        --D->expect[k];   // the kernel did not run: the device count did not move
        D->busy.fetch_and(~(1u << k), std::memory_order_release);
        ++g_sig_plain;
        (void) hipGetLastError();
        return hipStreamSynchronize(s);
    }
    const volatile uint32_t *w = D->page + k * kSigStride;
    bool seen = false;
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t i = 1;; ++i) {
        if (int32_t(__atomic_load_n(const_cast<const uint32_t *>(w), __ATOMIC_ACQUIRE) - want) >= 0) {
            seen = true;
            break;
        }
        if ((i & 1023u) == 0
            && std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count()
                   > double(tuning().sigspin_us))
            break;
        __builtin_ia32_pause();
    }
    D->busy.fetch_and(~(1u << k), std::memory_order_release);
    if (seen) {
        ++g_sig_fast;
        return hipSuccess;
    }
    ++g_sig_fallback;
    return hipStreamSynchronize(s);
}

// A capture this call can see: on its stream, or one that makes the legacy stream unusable
// (another thread's global-mode capture).  Only then do its allocations skip the device-wide
// settle of fenceless releases (PoolNoDeviceSync).
bool capture_seen(hipStream_t s)
{
    return capturing(s) || (s != nullptr && capturing(nullptr));
}

bool events_passed(const std::vector<hipEvent_t> &evs)
{
    for (hipEvent_t e : evs) {
        if (hipEventQuery(e) != hipSuccess) {
            (void) hipGetLastError();   // hipErrorNotReady must not look like a launch error
            return false;
        }
    }
    return true;
}

// A retired set whose readers have all passed: its events go, its device memory goes back
// to the plan's spare list for the next set that needs as much (no hipFree: that API
// synchronises the whole device, and a free inside a stream capture would break it).
void recycle(Plan &P, Retired &r)   // P.mu held
{
    for (hipEvent_t e : r.events)
        (void) hipEventDestroy(e);
    r.events.clear();
    ItemSet &S = *r.set;
    for (hipEvent_t e : S.late)
        (void) hipEventDestroy(e);
    S.late.clear();
    for (ItemSet::Binding &b : S.bind)
        if (b.slot >= 0) {   // every launch of the set has passed: its record is free
            slot_release(S.slot_dev, b.slot >> 8, b.slot & 255, b.gen, nullptr);
            b.slot = -1;
        }
    if (S.d_items) {
        P.spare.push_back({S.d_items, S.items.size() * sizeof(Item)});
        S.d_items = nullptr;
    }
}

// Recycle retired descriptor sets whose eviction events (and the late events of launches
// enqueued after the eviction) every launching stream has passed.  With `block` (never
// inside a capture), wait for the oldest until at most kRetiredMax remain: a host wait on
// those streams' events, not a device-wide synchronisation.  A set with a launch still
// being enqueued by another thread (inflight) is never touched.
void reap(Plan &P, bool block)   // P.mu held
{
    for (size_t i = 0; i < P.graveyard.size();) {
        Retired &r = P.graveyard[i];
        if (r.set->inflight || !events_passed(r.events) || !events_passed(r.set->late)) {
            ++i;
            continue;
        }
        recycle(P, r);
        P.graveyard.erase(P.graveyard.begin() + long(i));
    }
    while (block && P.graveyard.size() > kRetiredMax && !P.graveyard.front().set->inflight) {
        Retired &r = P.graveyard.front();
        for (hipEvent_t e : r.events)
            (void) hipEventSynchronize(e);
        for (hipEvent_t e : r.set->late)
            (void) hipEventSynchronize(e);
        recycle(P, r);
        P.graveyard.erase(P.graveyard.begin());
    }
}

// Device memory for `bytes` of descriptors: the smallest spare block that fits, else new.
// Retired sets are reaped here, when memory is wanted, and not on every new set: the event
// queries of a reap (like any allocation or upload) would invalidate a global-mode stream
// capture running in another thread (scripts/probe_capture.cpp), while an inline set -- a
// new window shape of a small type -- needs no HIP call but its launch.
Item *take_items_memory(Plan &P, size_t bytes, bool block)   // P.mu held
{
    reap(P, block);
    size_t best = P.spare.size();
    for (size_t i = 0; i < P.spare.size(); ++i)
        if (P.spare[i].bytes >= bytes && (best == P.spare.size() || P.spare[i].bytes < P.spare[best].bytes))
            best = i;
    if (best < P.spare.size()) {
        Item *d = static_cast<Item *>(P.spare[best].p);
        P.spare.erase(P.spare.begin() + long(best));
        return d;
    }
    return static_cast<Item *>(pool_alloc(bytes));
}

// A retired set (still in the graveyard) that a captured graph now holds: pinned for the
// plan's lifetime instead of recycled.
void pin_retired(Plan &P, const std::shared_ptr<ItemSet> &S)   // P.mu held
{
    S->pinned = true;
    for (size_t i = 0; i < P.graveyard.size(); ++i) {
        if (P.graveyard[i].set == S) {
            for (hipEvent_t e : P.graveyard[i].events)
                (void) hipEventDestroy(e);
            P.graveyard.erase(P.graveyard.begin() + long(i));
            P.pinned.push_back(S);
            return;
        }
    }
}

// An evicted set's device descriptors may still be read by launches in flight: record an
// event behind them on every stream that launched the set, recycle it once they pass.  A
// set a captured graph holds (or whose stream cannot take an event) lives as long as the plan.
void retire(Plan &P, const std::shared_ptr<ItemSet> &S)   // P.mu held
{
    S->retired = true;
    if (!S->d_items) {
        // nothing on the device; a call that looked it up still holds a plain pointer to it
        // until its launch is enqueued: the graveyard keeps the object until then
        if (S->inflight)
            P.graveyard.push_back(Retired{S, {}});
        return;
    }
    if (S->pinned) {
        P.pinned.push_back(S);
        return;
    }
    Retired r{S, {}};
    for (hipStream_t st : S->streams) {
        hipEvent_t e = nullptr;
        if (capturing(st) || hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess
            || hipEventRecord(e, st) != hipSuccess) {
            (void) hipGetLastError();
            if (e)
                (void) hipEventDestroy(e);
            for (hipEvent_t x : r.events)
                (void) hipEventDestroy(x);
            S->pinned = true;
            P.pinned.push_back(S);
            return;
        }
        r.events.push_back(e);
    }
    P.graveyard.push_back(std::move(r));
}

// Every stream that launched work reading a plan's device memory: the plan's destruction
// fences its memory behind them (~Plan, ddt_pool.h).  A launch inside a capture marks the
// plan: a graph may read its memory after the datatype is gone.
void note_stream_locked(Plan &P, hipStream_t stream, int cap = -1)   // P.mu held; cap: known capture state
{
    if (std::find(P.streams.begin(), P.streams.end(), stream) == P.streams.end())
        P.streams.push_back(stream);
    if (cap < 0 ? capturing(stream) : cap != 0)
        P.captured = true;
}

void note_stream(Plan &P, hipStream_t stream)
{
    std::lock_guard<SpinMutex> g(P.mu);
    note_stream_locked(P, stream);
}

// Find or build the descriptor set of one launch and run it on `stream`.
//
// Descriptor sets are independent of the absolute buffers: items address the user side
// relative to ubase = user rounded down to 16 bytes and the packed side relative to pbase
// (the first window's pointer rounded down), and the cache key holds only the low four
// bits of the pointers (all a unit-size choice depends on) plus the windows' shape.  A
// double-buffered halo, a fragment stream or the staging slots of a host pipeline hit the
// same set whatever buffers they use.
int run_windows(ddt_datatype *t, Plan &P, uint64_t count, uint64_t user,
                const std::vector<Window> &wins, bool same_layout, int dir, hipStream_t stream,
                uint32_t grid_cap = 0)
{
    if (wins.empty())
        return DDT_SUCCESS;
    int dev = 0;
    HIPCHK(hipGetDevice(&dev));
    int none = -1;
    if (P.device.load(std::memory_order_relaxed) < 0)   // a plan made without a device takes this one
        (void) P.device.compare_exchange_strong(none, dev);
    if (P.device != dev)
        return fail(DDT_ERR_NOT_SUPPORTED, "convertor prepared on device " + std::to_string(P.device)
                                               + "; current device is " + std::to_string(dev)
                                               + " (prepare it again on this device)");
    const uint64_t ubase = user & ~uint64_t(15), pbase = wins[0].ptr & ~uint64_t(15);
    std::vector<uint64_t> key;
    key.reserve(4 + 3 * wins.size());
    key.push_back(count);
    key.push_back(user - ubase);
    key.push_back(same_layout ? 1 : 0);
    key.push_back(uint64_t(same_layout ? interleave_of(0) : interleave_of(dir)));   // item order
    for (const Window &w : wins) {
        key.push_back(w.w0);
        key.push_back(w.w1);
        key.push_back(w.ptr - pbase);
    }
    try {
        ensure_device_lists(P);
    } catch (const std::exception &ex) {
        return fail(DDT_ERR_OUT_OF_RESOURCE, ex.what());
    }
    // a whole-message move of a large single-element index list: address-ordered engine
    if (!same_layout && wins.size() == 1 && wins[0].w0 == 0 && wins[0].w1 == count * uint64_t(t->size)
        && (wins[0].ptr % 16) == 0) {
        SortedList *SL = nullptr;
        try {
            SL = sorted_plan(t, P, user, stream);
        } catch (const std::exception &ex) {
            return fail(DDT_ERR_OUT_OF_RESOURCE, ex.what());
        }
        // every instance must keep the element alignment the address-ordered kernels load
        // with (sorted_plan checked instance 0): a resized extent that is not a multiple of
        // the element size sends instance i > 0 to the per-block kernel instead
        if (SL && count > 1 && uint64_t(t->extent() < 0 ? -t->extent() : t->extent()) % SL->esz != 0)
            SL = nullptr;
        if (SL) {
            note_stream(P, stream);
            const Leaf &L = P.leaves[0];
            for (uint64_t i = 0; i < count; ++i) {
                uint8_t *u = reinterpret_cast<uint8_t *>(user + uint64_t(L.list_shift) + uint64_t(P.dev[0].disp_base)
                                                         + i * uint64_t(t->extent()));
                uint8_t *pk = reinterpret_cast<uint8_t *>(wins[0].ptr + i * uint64_t(t->size));
                // spol bits, plus the pass-2 quads (256) and the pass-1 stagger (bits 16..23)
                const uint32_t pol = uint32_t(tuning().spol) | (tuning().s2vec ? 256u : 0u)
                                     | (uint32_t(tuning().slayout & 3) << 10)
                                     | (uint32_t(std::min<long>(tuning().sstagger, 255)) << 16);
                HIPCHK(SL->run(u, pk, dir, pol, stream, uint32_t(tuning().sunroll),
                               uint32_t(tuning().s2unroll)));
            }
            return DDT_SUCCESS;
        }
    }
    // The launch is enqueued outside the plan lock, so another thread may evict the set
    // meanwhile.  This call holds it (`inflight`, taken with the lookup) so its memory is not
    // recycled, and if it was retired, a launch by pointer leaves a late event behind it for
    // the retirement to wait on.  A retired set that fits in the kernel arguments is launched
    // from them instead.  (The local shared_ptr S keeps the object; Hold only points at it.)
    struct Hold {
        Plan &P;
        ItemSet *S;
        hipStream_t stream;
        bool by_pointer = false;
        ~Hold()
        {
            if (!S)
                return;
            // Not retired when the launch was already enqueued: a later retirement records its
            // fences after this launch, so the hold ends without the plan lock.  Retired before
            // the launch: the late event and the release are made under the lock, where reap
            // cannot come between them.
            if (!(by_pointer && S->retired.load())) {
                S->inflight.fetch_sub(1);
                return;
            }
            std::lock_guard<SpinMutex> g(P.mu);
            --S->inflight;
            if (!S->pinned) {
                hipEvent_t e = nullptr;
                if (hipEventCreateWithFlags(&e, hipEventDisableTiming) == hipSuccess
                    && hipEventRecord(e, stream) == hipSuccess) {
                    S->late.push_back(e);
                } else {
                    (void) hipGetLastError();
                    if (e)
                        (void) hipEventDestroy(e);
                    for (const auto &sp : P.graveyard)   // pin_retired wants the owning pointer
                        if (sp.set.get() == S) {
                            const std::shared_ptr<ItemSet> keep = sp.set;
                            pin_retired(P, keep);
                            break;
                        }
                    S->pinned = true;
                }
            }
        }
    };
    // A descriptor set travels in the kernel-argument segment on its first launch (no upload
    // for one-off windows).  From its second launch on it is launched by pointer from HBM:
    // with device-resident kernel arguments every 64-byte line of arguments is a host write
    // across PCIe, and a 528-byte block costs 2.6 us of host time per launch against 0.7 us
    // for a pointer (scripts/hostbench.cpp, profiles/r1_hostbench.log).
    Item *d_items = nullptr;
    int slot_k = -1, slot_b = -1;
    uint32_t slot_gen = 0;
    // the stream's capture state, queried before the plan lock: HIP answers under a global lock
    // of its own, and threads sharing this plan must not queue behind it (r6 thread scaling)
    const bool cap = capturing(stream);
    Hold hold{P, nullptr, stream};
    // S points into the plan's cache (or graveyard): `inflight` keeps the object alive until the
    // launch is enqueued (retire parks a held set in the graveyard), so no shared_ptr copy --
    // an atomic on a line every thread of a shared datatype writes -- is taken per call
    ItemSet *S = nullptr;
    const std::shared_ptr<ItemSet> *owner = nullptr;   // valid inside the plan lock only
    // The launch decision for set S (plan lock held): by pointer or inline, capture pinning, the
    // launch slot.  A cache hit makes it in the same critical section as its lookup: threads
    // sharing a datatype take the plan lock twice per call (here and in Hold), not four times,
    // and write the set's shared lines only when something changes (r6 thread scaling).
    // a set with no items moves nothing; a single line-dense item may launch by value
    // (launch_single_item): both skip the decision unless the by-value launch declines
    auto maybe_direct = [&]() { return S->items.empty() || (S->items.size() == 1 && grid_cap == 0 && S->all_dense); };
    auto decide = [&]() {
        if (S->inline_ok && !S->retired && S->uses < 2 && ++S->uses >= 2 && !S->d_items && tuning().ptr) {
            size_t bytes = S->items.size() * sizeof(Item);
            RelaxedCapture relaxed;
            PoolNoDeviceSync no_sync(capture_seen(stream));
            Item *d = take_items_memory(P, bytes, !cap);
            if (d) {
                if (upload(d, S->items.data(), bytes) == hipSuccess)
                    S->d_items = d;
                else
                    P.spare.push_back({d, bytes});
            }
        }
        d_items = (S->inline_ok && (!tuning().ptr || S->retired)) ? nullptr : S->d_items;
        if (!d_items)
            return;
        if (cap) {
            // the graph keeps this pointer: never recycle it before the plan goes
            if (S->retired && !S->pinned)
                pin_retired(P, *owner);
            S->pinned = true;
        } else if (tuning().slots && grid_cap == 0 && !S->all_dense && !S->has_lists && !S->retired
                   && S->bytes <= uint64_t(tuning().slot_max_kb) << 10) {
            // an argument-free launch (ddt_move.hip.h, ddt_move_slot_kernel): a set bound to
            // a slot for these buffers and this direction; buffers seen again within the set's
            // last kHist launches bind one (its record is in device memory before this launch;
            // two bindings serve a double-buffered exchange).  Small launches only: a slot
            // kernel's workgroups first load the record (one more dependent load than
            // arguments preloaded into registers), which a large launch of latency-bound
            // gathers pays (the halo's 48 MiB pack 66.4 -> 68.2 us), while the host's 2.2 us
            // saving only matters where the kernel is as short as a launch
            const int fam = dir << 8;
            ++S->launches;
            int hit = -1;
            for (int i = 0; i < ItemSet::kSetBind; ++i)
                if (S->bind[i].slot >= 0 && (S->bind[i].slot & ~255) == fam && S->bind[i].ubase == ubase
                    && S->bind[i].pbase == pbase)
                    hit = i;
            bool seen = hit >= 0;
            for (int i = 0; i < ItemSet::kHist && !seen; ++i)
                seen = S->hist_u[i] == ubase && S->hist_p[i] == pbase;
            if (hit < 0 && seen && S->launches >= S->bind_backoff) {
                // bind these buffers in a free binding, else in place of the least recently
                // used one if it sat idle for kSetIdle launches of the set (given up behind
                // fences on the set's streams).  A binding in use is never taken: threads
                // sharing the set on more buffer pairs than it holds bindings keep theirs,
                // the rest launch with arguments (round 6: taking turns rebound on every
                // call, a synchronous record upload each, bridgethreads shared 4 threads
                // 16.8 us per call)
                constexpr uint64_t kSetIdle = 32, kBindBackoff = 32;
                int pick = -1, lru = 0;
                for (int i = 0; i < ItemSet::kSetBind && pick < 0; ++i)
                    if (S->bind[i].slot < 0)
                        pick = i;
                    else if (S->bind[i].used < S->bind[lru].used)
                        lru = i;
                if (pick < 0 && S->launches - S->bind[lru].used >= kSetIdle)
                    pick = lru;
                if (pick >= 0) {
                    ItemSet::Binding &B = S->bind[pick];
                    if (B.slot >= 0) {
                        slot_release(S->slot_dev, B.slot >> 8, B.slot & 255, B.gen, &S->streams);
                        B.slot = -1;
                    }
                    const LaunchRec rec{uint64_t(uintptr_t(d_items)), ubase, pbase, uint32_t(S->items.size()),
                                        S->ntasks};
                    const int k = slot_bind(P.device, dir, rec, &B.gen);
                    if (k >= 0) {
                        B.slot = fam | k;
                        B.ubase = ubase;
                        B.pbase = pbase;
                        S->slot_dev = P.device;
                        hit = pick;
                    }
                }
                // every binding of the set in use: do not rescan on every call (a full slot
                // table is retried at once: each attempt ages the table's idle bindings)
                if (pick < 0)
                    S->bind_backoff = S->launches + kBindBackoff;
            }
            if (hit >= 0) {
                S->bind[hit].used = S->launches;
                slot_k = S->bind[hit].slot & 255;
                slot_gen = S->bind[hit].gen;
                slot_b = hit;
            } else {   // the history matters only for buffers not bound yet
                S->hist_u[S->hist_at] = ubase;
                S->hist_p[S->hist_at] = pbase;
                S->hist_at = (S->hist_at + 1) % ItemSet::kHist;
            }
        }
        if (std::find(S->streams.begin(), S->streams.end(), stream) == S->streams.end())
            S->streams.push_back(stream);
        note_stream_locked(P, stream, cap ? 1 : 0);   // one capture query per call (HIP takes a global lock)
        hold.by_pointer = true;
    };
    {
        std::lock_guard<SpinMutex> g(P.mu);
        for (size_t i = 0; i < P.cache.size(); ++i) {
            if (P.cache[i]->key == key) {
                // least recently used order, but the two most recent sets (a pack and an unpack
                // alternating) are not swapped on every call
                if (i >= 2) {
                    std::rotate(P.cache.begin(), P.cache.begin() + long(i), P.cache.begin() + long(i) + 1);
                    i = 0;
                }
                owner = &P.cache[i];
                S = owner->get();
                ++S->inflight;   // held until this call has enqueued its launch (Hold)
                hold.S = S;
                if (!maybe_direct())
                    decide();
                break;
            }
        }
    }
    std::shared_ptr<ItemSet> fresh;
    if (!S) {
        fresh = std::make_shared<ItemSet>();
        S = fresh.get();
        S->key = key;
        try {
            for (const Window &w : wins)
                build_items(t, P, count, user - ubase, w.ptr - pbase, w.w0, w.w1, same_layout, S->items);
        } catch (const std::exception &ex) {
            return fail(DDT_ERR_NOT_SUPPORTED, ex.what());
        }
        assign_tasks(S->items, same_layout ? 0 : dir);
        stream_policy(S->items);
        S->ntasks = total_tasks(S->items);
        for (const Item &it : S->items)
            S->bytes += it.kind == ITEM_FRAG ? it.nbytes : (it.u1 - it.u0) * it.U;
        for (Item &it : S->items)
            it.slab = use_slab(it) ? (tuning().xchunk > 0 ? uint32_t(tuning().xchunk) : SLAB_FULL) : 0;
        S->all_dense = !S->items.empty();
        for (const Item &it : S->items) {
            S->has_lists = S->has_lists || it.kind == ITEM_LIST_UNI || it.kind == ITEM_LIST_VAR;
            S->all_dense = S->all_dense && it.kind == ITEM_AFFINE && it.nbytes && !it.idx64;
        }
        if (S->items.size() <= INLINE_ITEMS) {
            // small sets travel in the kernel-argument segment: no device allocation
            S->inline_ok = true;
            S->blk.n = uint32_t(S->items.size());
            for (size_t i = 0; i < S->items.size(); ++i)
                S->blk.items[i] = S->items[i];
        } else if (!S->items.empty()) {
            size_t bytes = S->items.size() * sizeof(Item);
            RelaxedCapture relaxed;   // reap queries, allocation, upload: leave other threads' captures be
            PoolNoDeviceSync no_sync(capture_seen(stream));
            {
                std::lock_guard<SpinMutex> g(P.mu);
                S->d_items = take_items_memory(P, bytes, !cap);
            }
            if (!S->d_items)
                return fail(DDT_ERR_OUT_OF_RESOURCE, "descriptor memory");
            const hipError_t e = upload(S->d_items, S->items.data(), bytes);
            if (e != hipSuccess)
                return fail(DDT_ERR_HIP, std::string("item upload: ") + hipGetErrorString(e));
        }
        std::lock_guard<SpinMutex> g(P.mu);
        ++S->inflight;
        hold.S = S;
        P.cache.insert(P.cache.begin(), fresh);
        if (P.cache.size() > kCacheEntries) {
            retire(P, P.cache.back());
            P.cache.pop_back();
        }
        owner = &P.cache[0];
        if (!maybe_direct())
            decide();
    }
    if (S->items.empty())
        return DDT_SUCCESS;
    if (maybe_direct()) {
        // a large single-item line-dense launch carries the item's fields by value
        hipError_t e = hipSuccess;
        if (launch_single_item(S->items[0], dir, ubase, pbase, stream, &e)) {
            HIPCHK(e);
            return DDT_SUCCESS;
        }
        std::lock_guard<SpinMutex> g(P.mu);   // declined: the ordinary decision
        owner = nullptr;
        for (const auto &sp : P.cache)
            if (sp.get() == S)
                owner = &sp;
        for (const Retired &r : P.graveyard)
            if (!owner && r.set.get() == S)
                owner = &r.set;
        for (const auto &sp : P.pinned)
            if (!owner && sp.get() == S)
                owner = &sp;
        if (!owner)   // a held set is always in one of them (retire parks it)
            return fail(DDT_ERROR, "descriptor set lost while held");
        decide();
    }
    if (!d_items && S->has_lists)
        note_stream(P, stream);   // an inline launch of index lists reads the plan's lists
    if (slot_k >= 0) {
        hipError_t e = hipSuccess;
        if (slot_launch(P.device, dir, slot_k, slot_gen, S->ntasks, stream, &e)) {
            HIPCHK(e);
            return DDT_SUCCESS;
        }
        std::lock_guard<SpinMutex> g(P.mu);   // the binding was ended (evicted): launch with arguments
        ItemSet::Binding &B = S->bind[slot_b];
        if (B.slot == ((dir << 8) | slot_k) && B.gen == slot_gen)
            B.slot = -1;
    }
    if (!d_items)
        HIPCHK(launch_move_inline(S->blk, S->ntasks, dir, S->has_lists, ubase, pbase, stream, grid_cap,
                                  S->all_dense));
    else
        HIPCHK(launch_move(d_items, uint32_t(S->items.size()), S->ntasks, dir, S->has_lists, ubase, pbase,
                           stream, grid_cap, S->all_dense));
    return DDT_SUCCESS;
}

}  // namespace

struct alignas(128) ddt_convertor {   // per-thread objects on lines of their own (r6)
    ddt_datatype *dt = nullptr;
    uint64_t dt_serial = 0;   // dt->serial when prepared (a recycled address is another type)
    std::shared_ptr<Plan> plan;
    uint64_t count = 0;
    uint64_t base = 0;
    bool send = false;
    bool prepared = false;
    bool completed = false;
    uint64_t local_size = 0;
    uint64_t bConverted = 0;
    hipStream_t stream = nullptr;
    bool async = false;
    // host-iovec staging (one HBM buffer of up to stage_mb MiB, one copy stream).  The
    // buffer state lives with the convertor, not with one call: the buffer is rewritten
    // only after the last reader of its previous contents -- the D2H copies of a pack or
    // the kernels of an unpack (ev_free), possibly queued by an earlier asynchronous call
    // -- has passed (pml_ob1_recvreq.c:627-663 issues such back-to-back async unpacks).
    // The buffer grows with the largest piece a call stages (1 MiB steps, doubling, up to
    // stage_mb): a convertor that stages kilobyte fragments holds a megabyte, not 256.
    void *stage = nullptr;
    uint64_t stage_size = 0;
    std::vector<void *> outgrown;   // earlier, smaller buffers: freed with the convertor
    hipStream_t copy_stream = nullptr;
    hipEvent_t ev_chunk[2] = {nullptr, nullptr};
    hipEvent_t ev_free = nullptr;
    bool rec_free = false;
    bool staged_in_capture = false;   // a staged call was enqueued into a stream capture
    // No host wait: a convertor without host staging holds no device memory, and the staging
    // buffers of one that has it go to the engine's pool behind fences, like a destroyed
    // plan's (ddt_pool.h): ev_free, recorded after the last reader of the buffer on whichever
    // stream the last staged call used (each staged call waits for the previous ev_free, so it
    // covers them all -- ADVICE r3: the stream may have been changed since, and the bridge
    // resets it to NULL after every call), plus the current user and copy streams.  So an
    // OBJ_RELEASE of a convertor never stalls, even during another thread's stream capture.
    ~ddt_convertor()
    {
        if (stage || !outgrown.empty()) {
            std::vector<void *> blocks(outgrown);
            if (stage)
                blocks.push_back(stage);
            std::vector<hipEvent_t> fences;
            bool unknown = false;
            std::vector<hipStream_t> ss{stream};
            if (copy_stream)
                ss.push_back(copy_stream);
            if (!staged_in_capture && pool_fences(ss, fences, unknown)) {
                if (rec_free && ev_free) {
                    fences.push_back(ev_free);   // the pool owns and destroys it
                    ev_free = nullptr;
                }
                pool_release(blocks, fences, unknown);
            } else {   // a capturing stream: its graph may read the staging buffer
                for (hipEvent_t e : fences)
                    (void) hipEventDestroy(e);
                for (void *p : blocks)
                    pool_keep(p);
            }
        }
        if (copy_stream)
            (void) hipStreamDestroy(copy_stream);   // queued copies still complete
        for (hipEvent_t e : {ev_chunk[0], ev_chunk[1], ev_free})
            if (e)
                (void) hipEventDestroy(e);
    }
    // a staging buffer of at least min(need, stage_mb) bytes
    int ensure_staging(uint64_t need)
    {
        if (!copy_stream) {
            HIPCHK(hipStreamCreateWithFlags(&copy_stream, hipStreamNonBlocking));
            for (hipEvent_t *e : {&ev_chunk[0], &ev_chunk[1], &ev_free})
                HIPCHK(hipEventCreateWithFlags(e, hipEventDisableTiming));
        }
        const uint64_t cap = std::max<uint64_t>(stage_bytes(), 1u << 20), mib = 1u << 20;
        uint64_t want = (std::min(need, cap) + mib - 1) / mib * mib;
        if (stage_size >= want)
            return DDT_SUCCESS;
        want = std::max(want, std::min(cap, stage_size * 2));
        void *p = pool_alloc(want);
        if (!p)
            return fail(DDT_ERR_OUT_OF_RESOURCE, "staging buffer");
        if (stage)
            outgrown.push_back(stage);   // may still be read by queued work: kept until destruction
        stage = p;
        stage_size = want;
        return DDT_SUCCESS;
    }
};

namespace {

constexpr uint64_t kSplitMin = 24ull << 20;   // host pieces split into two overlapped chunks

// Move the packed windows of a convertor call: device iovecs (and pinned host iovecs the
// kernel reaches over PCIe) in one launch; other host iovecs through the HBM staging buffer,
// kernels on the user stream, copies on copy_stream, in pieces of at most stage_size.
//
// A piece of >= 24 MiB is split in two chunks so that kernels and copies overlap, with the short chunk
// where it is exposed (round 2; profiles/r2_e2e_pageable.jsonl): a pack queues BOTH chunk
// kernels first (short chunk first) and only then the copies -- a copy from or to pageable
// memory blocks the calling thread, so a kernel queued after it would start only when it
// ends; an unpack copies the long chunk first and ends on the short one, so only the short
// chunk's copy and kernel are not hidden.
int execute(ddt_convertor *c, const std::vector<Window> &dev_wins,
            const std::vector<std::pair<Window, void *>> &host_wins, int dir, bool pcie = false)
{
    // a window in pinned host memory: PCIe is the limit, and a capped grid keeps the reads
    // of an unpack at the link rate where thousands of workgroups contending for it lose 5 %
    // (scripts/ubench_pcie.hip); a multiple of 8 keeps the XCD slab mapping
    const long capv = dir == 0 ? tuning().hd_grid_pack : tuning().hd_grid;
    const uint32_t cap = pcie ? uint32_t(std::max<long>(capv, 0) & ~7L) : 0;
    int rc = run_windows(c->dt, *c->plan, c->count, c->base, dev_wins, false, dir, c->stream, cap);
    if (rc != DDT_SUCCESS)
        return rc;
    if (!host_wins.empty()) {
        uint64_t need = 0;
        for (const auto &hw : host_wins)
            need = std::max(need, hw.first.w1 - hw.first.w0);
        if ((rc = c->ensure_staging(need)) != DDT_SUCCESS)
            return rc;
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        if (hipStreamIsCapturing(c->stream, &cs) != hipSuccess)
            (void) hipGetLastError();   // the legacy stream under a foreign capture: not captured
        else if (cs != hipStreamCaptureStatusNone)
            c->staged_in_capture = true;
        char *st = static_cast<char *>(c->stage);
        for (const auto &hw : host_wins) {
            for (uint64_t off = hw.first.w0; off < hw.first.w1;) {
                const uint64_t piece = std::min<uint64_t>(c->stage_size, hw.first.w1 - off);
                const uint64_t small = std::min<uint64_t>(piece, std::max<uint64_t>(piece / 16, 1u << 20));
                const uint64_t len[2] = {dir == 0 ? small : piece - small, dir == 0 ? piece - small : small};
                char *hp = static_cast<char *>(hw.second) + (off - hw.first.w0);
                if (piece < kSplitMin) {
                    // one kernel and one copy, both on the user stream: below ~24 MiB a second
                    // chunk hides less kernel time than its extra copy costs (16 MiB pageable:
                    // 35.7 GiB/s split against 44.9 in one; 24 and 48 MiB gain 2 % from the split,
                    // profiles/r2_e2e_pageable.jsonl)
                    if (c->rec_free)
                        HIPCHK(hipStreamWaitEvent(c->stream, c->ev_free, 0));
                    std::vector<Window> w{{off, off + piece, uint64_t(uintptr_t(st))}};
                    if (dir == 0) {
                        if ((rc = run_windows(c->dt, *c->plan, c->count, c->base, w, false, 0, c->stream)))
                            return rc;
                        HIPCHK(hipMemcpyAsync(hp, st, piece, hipMemcpyDeviceToHost, c->stream));
                    } else {
                        HIPCHK(hipMemcpyAsync(st, hp, piece, hipMemcpyHostToDevice, c->stream));
                        if ((rc = run_windows(c->dt, *c->plan, c->count, c->base, w, false, 1, c->stream)))
                            return rc;
                    }
                    HIPCHK(hipEventRecord(c->ev_free, c->stream));
                } else if (dir == 0) {   // pack: both kernels, then both D2H copies
                    if (c->rec_free)
                        HIPCHK(hipStreamWaitEvent(c->stream, c->ev_free, 0));   // last call's copies
                    for (int j = 0; j < 2; ++j) {
                        const uint64_t b0 = j ? len[0] : 0;
                        if (!len[j])
                            continue;
                        std::vector<Window> w{{off + b0, off + b0 + len[j], uint64_t(uintptr_t(st + b0))}};
                        if ((rc = run_windows(c->dt, *c->plan, c->count, c->base, w, false, 0, c->stream)))
                            return rc;
                        HIPCHK(hipEventRecord(c->ev_chunk[j], c->stream));
                    }
                    for (int j = 0; j < 2; ++j) {
                        const uint64_t b0 = j ? len[0] : 0;
                        if (!len[j])
                            continue;
                        HIPCHK(hipStreamWaitEvent(c->copy_stream, c->ev_chunk[j], 0));
                        HIPCHK(hipMemcpyAsync(hp + b0, st + b0, len[j], hipMemcpyDeviceToHost, c->copy_stream));
                    }
                    HIPCHK(hipEventRecord(c->ev_free, c->copy_stream));
                } else {          // unpack: per chunk H2D copy, then its kernel
                    if (c->rec_free)
                        HIPCHK(hipStreamWaitEvent(c->copy_stream, c->ev_free, 0));   // last kernels
                    for (int j = 0; j < 2; ++j) {
                        const uint64_t b0 = j ? len[0] : 0;
                        if (!len[j])
                            continue;
                        HIPCHK(hipMemcpyAsync(st + b0, hp + b0, len[j], hipMemcpyHostToDevice, c->copy_stream));
                        HIPCHK(hipEventRecord(c->ev_chunk[j], c->copy_stream));
                        HIPCHK(hipStreamWaitEvent(c->stream, c->ev_chunk[j], 0));
                        std::vector<Window> w{{off + b0, off + b0 + len[j], uint64_t(uintptr_t(st + b0))}};
                        if ((rc = run_windows(c->dt, *c->plan, c->count, c->base, w, false, 1, c->stream)))
                            return rc;
                    }
                    HIPCHK(hipEventRecord(c->ev_free, c->stream));
                }
                c->rec_free = true;
                off += piece;
            }
        }
        // the user stream observes completion of this call's copies (an event the caller
        // records on it after the call covers the whole message)
        if (dir == 0)
            HIPCHK(hipStreamWaitEvent(c->stream, c->ev_free, 0));
    }
    // data in place on return: the signal kernel when every window is device memory (the
    // staged and PCIe paths end in host memory written by copies or over the link)
    if (!c->async)
        HIPCHK(complete_sync(c->stream, host_wins.empty() && !pcie));
    return DDT_SUCCESS;
}

int prepare(ddt_convertor *c, const ddt_datatype *t, size_t count, const void *buf, bool send)
{
    if (!c || !t)
        return fail(DDT_ERR_BAD_PARAM, "null convertor or datatype");
    if (!(t->flags & F_COMMITTED))
        return fail(DDT_ERR_NOT_COMMITTED, "datatype not committed");
    ddt_datatype *dt = const_cast<ddt_datatype *>(t);
    const bool same_type = c->dt == dt && c->dt_serial == dt->serial && c->plan;
    c->dt = dt;
    c->dt_serial = dt->serial;
    c->count = count;
    c->base = uint64_t(uintptr_t(buf));
    c->send = send;
    c->local_size = uint64_t(t->size) * count;
    c->bConverted = 0;
    c->completed = (c->local_size == 0);
    c->prepared = true;
    if (c->local_size == 0)
        return DDT_SUCCESS;
    // accelerator slot: check_addr must report device memory (opal_convertor.c:593-608)
    // probe the first byte the type map touches (buf + true_lb): unlike the reference,
    // which probes pUserBuf itself (opal_convertor.c:624,654), this also classifies
    // MPI_BOTTOM-style buffers whose base lies outside the allocation
    if (classify(static_cast<const char *>(buf) + t->true_lb) != MEM_DEVICE)
        return fail(DDT_ERR_NOT_DEVICE, "user buffer is not device memory: the HIP engine is the "
                                        "accelerator slot of the convertor");
    // a convertor prepared again with the type it holds keeps its plan when the device is the
    // same (the bridge re-prepares its per-thread convertor on every fAdvance: no shared plan
    // table lock or reference count per call, r6 thread scaling)
    int dev = -1;
    if (same_type && hipGetDevice(&dev) == hipSuccess && c->plan->device == dev)
        return DDT_SUCCESS;
    (void) hipGetLastError();
    try {
        c->plan = get_plan(dt);
    } catch (const std::exception &ex) {
        return fail(DDT_ERR_OUT_OF_RESOURCE, ex.what());
    }
    return DDT_SUCCESS;
}

// OPAL_CONVERTOR_PREPARE leaves CONVERTOR_NO_OP set, and fPosition NULL, for a type without
// gaps or one contiguous instance (opal_convertor.c:562-567)
bool is_no_op(const ddt_convertor *c)
{
    return (c->dt->flags & F_NO_GAPS) || ((c->dt->flags & F_CONTIGUOUS) && c->count == 1);
}

int32_t advance(ddt_convertor *c, struct iovec *iov, uint32_t *out_size, size_t *max_data, int dir)
{
    if (!c || !c->prepared || !out_size || !max_data || (*out_size && !iov))
        return fail(DDT_ERR_BAD_PARAM, "convertor not prepared or bad iovec");
    if (c->completed) {   // opal_convertor_pack/unpack: nothing left (opal_convertor.c:258-261)
        if (*out_size)
            iov[0].iov_len = 0;
        *out_size = 0;
        *max_data = 0;
        return 1;
    }
    std::vector<Window> dev;
    std::vector<std::pair<Window, void *>> host;
    uint64_t pos = c->bConverted, total = 0;
    uint32_t used = 0;
    bool pcie = false;
    // A NO_OP convertor (OPAL_CONVERTOR_PREPARE, opal_convertor.c:562-567: a type without
    // gaps, or one contiguous instance) is moved by opal_convertor_pack's memcpy loop
    // (:262-302), which fills every iovec to the byte; other types go through the movers,
    // which never split a predefined element (_pack_accelerator.c:52-58).
    const bool no_op = is_no_op(c);
    for (uint32_t i = 0; i < *out_size; ++i) {
        if (pos >= c->local_size)
            break;
        uint64_t w1 = std::min<uint64_t>(pos + iov[i].iov_len, c->local_size);
        if (dir == 0 && w1 < c->local_size && !no_op) {   // pack never splits a predefined element
            uint64_t s = snap_down_to_element(c->dt, w1);
            w1 = std::max(s, pos);
        }
        uint64_t n = w1 - pos;
        iov[i].iov_len = n;
        used = i + 1;
        if (n) {
            if (!iov[i].iov_base)
                return fail(DDT_ERR_BAD_PARAM, "null iov_base");
            uint64_t hd = 0;
            if (classify(iov[i].iov_base) == MEM_DEVICE)
                dev.push_back({pos, w1, uint64_t(uintptr_t(iov[i].iov_base))});
            else if ((tuning().hostdirect & (dir == 0 ? 2 : 1)) && (hd = pinned_device_range(iov[i].iov_base, n)) != 0) {
                dev.push_back({pos, w1, hd});   // the kernel reads/writes the pinned pages over PCIe
                pcie = true;
            }
            else
                host.push_back({{pos, w1, 0}, iov[i].iov_base});
        }
        pos = w1;
        total += n;
    }
    int rc = execute(c, dev, host, dir, pcie);
    if (rc != DDT_SUCCESS)
        return rc;
    c->bConverted = pos;
    *out_size = used;
    *max_data = total;
    if (c->bConverted == c->local_size) {
        c->completed = true;
        return 1;
    }
    return 0;
}

}  // namespace

extern "C" {

ddt_convertor_t *ddt_convertor_create(void) { return new (std::nothrow) ddt_convertor(); }

void ddt_convertor_destroy(ddt_convertor_t *c) { delete c; }

int ddt_convertor_prepare_for_send(ddt_convertor_t *c, const ddt_datatype_t *t, size_t count,
                                   const void *buf)
{
    return prepare(c, t, count, buf, true);
}

int ddt_convertor_prepare_for_recv(ddt_convertor_t *c, const ddt_datatype_t *t, size_t count,
                                   void *buf)
{
    return prepare(c, t, count, buf, false);
}

int32_t ddt_convertor_pack(ddt_convertor_t *c, struct iovec *iov, uint32_t *out_size, size_t *max_data)
{
    return advance(c, iov, out_size, max_data, 0);
}

int32_t ddt_convertor_unpack(ddt_convertor_t *c, struct iovec *iov, uint32_t *out_size,
                             size_t *max_data)
{
    return advance(c, iov, out_size, max_data, 1);
}

int ddt_convertor_set_position(ddt_convertor_t *c, size_t *position)
{
    // opal_convertor_set_position (opal_convertor.h:357-394)
    if (!c || !position || !c->prepared)
        return fail(DDT_ERR_BAD_PARAM, "bad convertor");
    if (c->local_size <= *position) {
        c->completed = true;
        c->bConverted = c->local_size;
        *position = size_t(c->bConverted);
        return DDT_SUCCESS;
    }
    c->completed = false;
    // A send convertor never stops inside a predefined element: opal_convertor_position_generic
    // (opal_convertor.c:458-470) walks to the position (opal_datatype_position.c:167-367), then
    // drops the partial element (bConverted -= partial_length) and hands back the snapped
    // position.  A NO_OP convertor has no fPosition and lands on the byte (opal_convertor.h:389-392);
    // a receive convertor accepts split elements.
    uint64_t p = *position;
    if (c->send && !is_no_op(c))
        p = snap_down_to_element(c->dt, p);
    c->bConverted = p;
    *position = size_t(p);
    return DDT_SUCCESS;
}

int ddt_type_snap_position(const ddt_datatype_t *t, size_t position, size_t *snapped)
{
    if (!t || !snapped)
        return fail(DDT_ERR_BAD_PARAM, "null datatype or result");
    if (!(t->flags & F_COMMITTED))
        return fail(DDT_ERR_NOT_COMMITTED, "datatype not committed");
    *snapped = size_t(snap_down_to_element(t, position));
    return DDT_SUCCESS;
}

namespace {

// opal_convertor_merge_iov (opal_convertor_raw.c:41-58): extend the current iovec when the
// piece starts where it ends, otherwise open the next one; a piece that needs an iovec
// beyond the caller's array is not consumed.
struct RawOut {
    struct iovec *iov;
    uint32_t cap;
    uint32_t idx = 0;
    uint64_t total = 0;
    bool piece(uint64_t addr, uint64_t len)
    {
        if (len == 0)
            return true;
        struct iovec &cur = iov[idx];
        if (cur.iov_len != 0) {
            if (addr == uint64_t(uintptr_t(cur.iov_base)) + cur.iov_len) {
                cur.iov_len += len;
                total += len;
                return true;
            }
            if (++idx == cap)
                return false;
        }
        iov[idx].iov_base = reinterpret_cast<void *>(uintptr_t(addr));
        iov[idx].iov_len = len;
        total += len;
        return true;
    }
};

// Emit the user-memory pieces of `nodes` (one type-map level at `base`) in type-map order,
// starting `skip` packed bytes in.  Returns false once the iovec array is full.
bool raw_walk(const std::vector<Node> &nodes, uint64_t base, uint64_t skip, RawOut &o)
{
    for (const Node &n : nodes) {
        const uint64_t sz = n.packed_bytes();
        if (skip >= sz) {
            skip -= sz;
            continue;
        }
        switch (n.kind) {
        case Node::DATA: {
            uint64_t k = skip / n.blen, off = skip % n.blen;
            for (; k < n.count; ++k, off = 0)
                if (!o.piece(base + uint64_t(n.disp + int64_t(k) * n.extent) + off, n.blen - off))
                    return false;
            break;
        }
        case Node::LOOP: {
            uint64_t k = skip / n.body_size, rem = skip % n.body_size;
            for (; k < n.count; ++k, rem = 0)
                if (!raw_walk(n.body, base + uint64_t(int64_t(k) * n.extent), rem, o))
                    return false;
            break;
        }
        case Node::LIST: {
            const IndexList &X = *n.list;
            const size_t nb = X.nblk();
            size_t b;
            uint64_t off;
            if (X.len.empty()) {
                b = size_t(skip / X.ulen);
                off = skip % X.ulen;
            } else {
                b = size_t(std::upper_bound(X.poff.begin(), X.poff.begin() + long(nb), skip) - X.poff.begin()) - 1;
                off = skip - X.poff[b];
            }
            for (; b < nb; ++b, off = 0) {
                const uint64_t len = X.len.empty() ? X.ulen : X.len[b];
                if (off >= len)
                    continue;
                if (!o.piece(base + uint64_t(n.disp + X.disp[b]) + off, len - off))
                    return false;
            }
            break;
        }
        }
        skip = 0;
    }
    return true;
}

}  // namespace

int ddt_convertor_prepare_for_raw(ddt_convertor_t *c, const ddt_datatype_t *t, size_t count,
                                  const void *buf)
{
    // the reference prepares a send convertor on a NULL or host base for raw export
    // (ddt_raw2.c:45, common_ompio_file_open.c:860-873): address arithmetic only, so no
    // device check and no plan
    if (!c || !t)
        return fail(DDT_ERR_BAD_PARAM, "null convertor or datatype");
    if (!(t->flags & F_COMMITTED))
        return fail(DDT_ERR_NOT_COMMITTED, "datatype not committed");
    c->dt = const_cast<ddt_datatype *>(t);
    c->count = count;
    c->base = uint64_t(uintptr_t(buf));
    c->send = true;
    c->local_size = uint64_t(t->size) * count;
    c->bConverted = 0;
    c->completed = (c->local_size == 0);
    c->prepared = true;
    return DDT_SUCCESS;
}

int32_t ddt_convertor_raw(ddt_convertor_t *c, struct iovec *iov, uint32_t *iov_count, size_t *length)
{
    // opal_convertor_raw (opal_convertor_raw.c:65-283)
    if (!c || !c->prepared || !iov_count || !length || (*iov_count && !iov))
        return fail(DDT_ERR_BAD_PARAM, "convertor not prepared or bad iovec");
    if (c->completed || *iov_count == 0) {
        if (*iov_count) {
            iov[0].iov_base = nullptr;
            iov[0].iov_len = 0;
        }
        *iov_count = 0;
        *length = 0;
        return c->completed ? 1 : 0;
    }
    const ddt_datatype *t = c->dt;
    RawOut o{iov, *iov_count};
    iov[0].iov_len = 0;
    const uint64_t size = uint64_t(t->size);
    const int64_t ext = t->extent();
    bool room = true;
    for (uint64_t i = c->bConverted / size; room && i < c->count; ++i) {
        const uint64_t skip = i == c->bConverted / size ? c->bConverted % size : 0;
        room = raw_walk(t->opt, c->base + uint64_t(int64_t(i) * ext), skip, o);
    }
    c->bConverted += o.total;
    *length = size_t(o.total);
    *iov_count = room ? (iov[o.idx].iov_len ? o.idx + 1 : o.idx) : o.cap;
    if (c->bConverted == c->local_size) {
        c->completed = true;
        return 1;
    }
    return 0;
}

int ddt_convertor_get_packed_size(const ddt_convertor_t *c, size_t *size)
{
    if (!c || !size)
        return DDT_ERR_BAD_PARAM;
    *size = size_t(c->local_size);
    return DDT_SUCCESS;
}

int ddt_convertor_get_position(const ddt_convertor_t *c, size_t *position)
{
    if (!c || !position)
        return DDT_ERR_BAD_PARAM;
    *position = size_t(c->bConverted);
    return DDT_SUCCESS;
}

int ddt_convertor_is_completed(const ddt_convertor_t *c) { return c && c->completed ? 1 : 0; }

int ddt_convertor_clone(const ddt_convertor_t *src, ddt_convertor_t *dst, int copy_stack)
{
    // opal_convertor_clone (opal_convertor.c:708-756): the resume state is bConverted only
    if (!src || !dst || src == dst)
        return fail(DDT_ERR_BAD_PARAM, "bad convertor");
    dst->dt = src->dt;
    dst->plan = src->plan;
    dst->count = src->count;
    dst->base = src->base;
    dst->send = src->send;
    dst->prepared = src->prepared;
    dst->local_size = src->local_size;
    dst->stream = src->stream;
    dst->async = src->async;
    dst->bConverted = copy_stack ? src->bConverted : 0;
    dst->completed = copy_stack ? src->completed : (src->local_size == 0);
    return DDT_SUCCESS;
}

int ddt_convertor_clone_with_position(const ddt_convertor_t *src, ddt_convertor_t *dst, int copy_stack,
                                      size_t *position)
{
    int rc = ddt_convertor_clone(src, dst, copy_stack);
    if (rc != DDT_SUCCESS)
        return rc;
    return ddt_convertor_set_position(dst, position);
}

int ddt_convertor_need_buffers(const ddt_convertor_t *c)
{
    // opal_convertor_need_buffers (opal_convertor.h:231-240), homogeneous
    if (!c || !c->dt)
        return 1;
    if (c->dt->flags & F_NO_GAPS)
        return 0;
    if (c->count == 1 && (c->dt->flags & F_CONTIGUOUS))
        return 0;
    return 1;
}

int ddt_convertor_get_current_pointer(const ddt_convertor_t *c, void **position)
{
    if (!c || !c->dt || !position)
        return DDT_ERR_BAD_PARAM;
    *position = reinterpret_cast<void *>(c->base + c->bConverted + uint64_t(c->dt->true_lb));
    return DDT_SUCCESS;
}

int ddt_convertor_get_offset_pointer(const ddt_convertor_t *c, size_t offset, void **position)
{
    if (!c || !c->dt || !position)
        return DDT_ERR_BAD_PARAM;
    *position = reinterpret_cast<void *>(c->base + uint64_t(offset) + uint64_t(c->dt->true_lb));
    return DDT_SUCCESS;
}

int ddt_convertor_get_unpacked_size(const ddt_convertor_t *c, size_t *size)
{
    if (!c || !size)
        return DDT_ERR_BAD_PARAM;
    *size = size_t(c->local_size);
    return DDT_SUCCESS;
}

int ddt_convertor_cleanup(ddt_convertor_t *c)
{
    // opal_convertor_cleanup (opal_convertor.h:208-219)
    if (!c)
        return DDT_ERR_BAD_PARAM;
    c->dt = nullptr;
    c->plan.reset();
    c->count = 0;
    c->base = 0;
    c->prepared = false;
    c->completed = true;
    c->local_size = 0;
    c->bConverted = 0;
    return DDT_SUCCESS;
}

int ddt_convertor_set_stream(ddt_convertor_t *c, void *s, int async)
{
    if (!c)
        return DDT_ERR_BAD_PARAM;
    c->stream = static_cast<hipStream_t>(s);
    c->async = async != 0;
    return DDT_SUCCESS;
}

int ddt_pack_size(size_t incount, const ddt_datatype_t *t, size_t *size)
{
    if (!t || !size)
        return DDT_ERR_BAD_PARAM;
    *size = incount * size_t(t->size);
    return DDT_SUCCESS;
}

int ddt_pack(const void *inbuf, size_t incount, const ddt_datatype_t *t, void *outbuf,
             size_t outsize, size_t *position)
{
    // MPI_Pack (ompi/mpi/c/pack.c.in:41-164)
    if (!t || !position || (!outbuf && outsize))
        return fail(DDT_ERR_BAD_PARAM, "bad argument");
    size_t need = incount * size_t(t->size);
    if (*position > outsize || outsize - *position < need)
        return fail(DDT_ERR_TRUNCATE, "output buffer too small");
    if (need == 0)
        return DDT_SUCCESS;
    ddt_convertor c;
    int rc = prepare(&c, t, incount, inbuf, true);
    if (rc != DDT_SUCCESS)
        return rc;
    struct iovec iov{static_cast<char *>(outbuf) + *position, need};
    uint32_t n = 1;
    size_t max_data = 0;
    int32_t r = advance(&c, &iov, &n, &max_data, 0);
    if (r < 0)
        return r;
    *position += max_data;
    return DDT_SUCCESS;
}

int ddt_unpack(const void *inbuf, size_t insize, size_t *position, void *outbuf, size_t outcount,
               const ddt_datatype_t *t)
{
    // MPI_Unpack (ompi/mpi/c/unpack.c.in:38-171)
    if (!t || !position || (!inbuf && insize))
        return fail(DDT_ERR_BAD_PARAM, "bad argument");
    size_t need = outcount * size_t(t->size);
    if (*position > insize || insize - *position < need)
        return fail(DDT_ERR_TRUNCATE, "input buffer too small");
    if (need == 0)
        return DDT_SUCCESS;
    ddt_convertor c;
    int rc = prepare(&c, t, outcount, outbuf, false);
    if (rc != DDT_SUCCESS)
        return rc;
    struct iovec iov{const_cast<char *>(static_cast<const char *>(inbuf)) + *position, need};
    uint32_t n = 1;
    size_t max_data = 0;
    int32_t r = advance(&c, &iov, &n, &max_data, 1);
    if (r < 0)
        return r;
    *position += max_data;
    return DDT_SUCCESS;
}

namespace {

// HBM scratch of the synchronous calls (external32, two-type sndrcv): per thread, per device and per slot,
// grown on demand and reused (each call ends with a stream synchronisation, so the next
// call of the thread finds it free).  Round 1 allocated per call, round 2 first with
// stream-ordered allocations, whose pool returns the memory at every synchronisation: a
// 16 MiB MPI_Pack_external spent ~300 us of its 357 in allocation (profiles/r2_ext_bench.jsonl).
// Only buffers up to kKeepBytes are kept by the thread: a larger request (a multi-GiB message)
// gets a block of its own for the call, handed back to HIP when the call ends (the call has
// synchronised its stream; ADVICE r3: not parked in the engine's pool, where co-resident
// allocators could not have it); ddt_trim() returns pooled memory to HIP.
// A call that returns early on an error may leave work queued on `stream` that still reads or
// writes the buffer: the destructor then waits for that stream before the memory can be
// reused by another thread (settled() marks the call's own final synchronisation).
constexpr size_t kKeepBytes = size_t(256) << 20;
struct DevBuf {
    void *p = nullptr;
    void *own = nullptr;
    int slot = 0;
    hipStream_t stream = nullptr;
    bool queued = false;
    explicit DevBuf(int s, hipStream_t st = nullptr) : slot(s), stream(st) {}
    DevBuf(const DevBuf &) = delete;
    DevBuf &operator=(const DevBuf &) = delete;
    ~DevBuf()
    {
        if (queued)
            (void) hipStreamSynchronize(stream);
        pool_free_now(own);
    }
    void settled() { queued = false; }
    hipError_t alloc(size_t n)
    {
        queued = true;
        if (n > kKeepBytes) {
            own = pool_alloc(n);
            p = own;
            return own ? hipSuccess : hipErrorOutOfMemory;
        }
        struct Cache {
            std::map<std::pair<int, int>, std::pair<void *, size_t>> bufs;   // (device, slot)
            ~Cache()
            {
                for (auto &kv : bufs)
                    pool_free(kv.second.first);
            }
        };
        thread_local Cache cache;
        int dev = 0;
        hipError_t e = hipGetDevice(&dev);
        if (e != hipSuccess)
            return e;
        auto &b = cache.bufs[{dev, slot}];
        if (b.second < n || !b.first) {
            pool_free(b.first);   // the thread's previous call synchronised its stream
            b = {nullptr, 0};
            const size_t want = std::max<size_t>(n, 1u << 20);
            if (!(b.first = pool_alloc(want)))
                return hipErrorOutOfMemory;
            b.second = want;
        }
        p = b.first;
        return hipSuccess;
    }
};

}  // namespace

int ddt_sndrcv(const void *sbuf, size_t scount, const ddt_datatype_t *st, void *rbuf, size_t rcount,
               const ddt_datatype_t *rt, void *stream)
{
    // ompi_datatype_sndrcv (ompi/datatype/ompi_datatype_sndrcv.c:46-126): a local send/recv
    // between two typed device buffers.  A null type means that side is MPI_PACKED bytes.
    hipStream_t s = static_cast<hipStream_t>(stream);
    const size_t ssz = st ? size_t(st->size) : 1, rsz = rt ? size_t(rt->size) : 1;
    if (!st && !rt)
        return fail(DDT_ERR_BAD_PARAM, "both sides packed");
    if (rcount == 0 || rsz == 0)
        return (scount == 0 || ssz == 0) ? DDT_SUCCESS : fail(DDT_ERR_TRUNCATE, "receive is empty");
    auto one_side = [&](const ddt_datatype_t *t, size_t count, const void *ubuf, void *pbuf, size_t n,
                        int dir, size_t *moved) -> int {
        ddt_convertor c;
        int rc = prepare(&c, t, count, ubuf, dir == 0);
        if (rc != DDT_SUCCESS)
            return rc;
        c.stream = s;
        struct iovec iov{pbuf, n};
        uint32_t k = 1;
        int32_t r = advance(&c, &iov, &k, moved, dir);
        return r < 0 ? r : DDT_SUCCESS;
    };
    size_t moved = 0;
    int rc;
    if (st && rt && st == rt) {   // same datatype: typed copy of min(scount, rcount) instances
        if ((rc = ddt_copy_content_same_ddt(rt, std::min(scount, rcount), rbuf, sbuf, stream)) != DDT_SUCCESS)
            return rc;
        return scount > rcount ? fail(DDT_ERR_TRUNCATE, "send larger than receive") : DDT_SUCCESS;
    }
    if (!rt) {                    // receive packed: rcount bytes
        const size_t n = std::min(scount * ssz, rcount);
        if ((rc = one_side(st, scount, sbuf, rbuf, n, 0, &moved)) != DDT_SUCCESS)
            return rc;
        // the reference reports MPI_ERR_TRUNCATE whenever fewer than rcount bytes arrive
        return moved < rcount ? fail(DDT_ERR_TRUNCATE, "packed receive not filled") : DDT_SUCCESS;
    }
    if (!st) {                    // send packed: scount bytes
        const size_t n = std::min(rcount * rsz, scount);
        if ((rc = one_side(rt, rcount, rbuf, const_cast<void *>(sbuf), n, 1, &moved)) != DDT_SUCCESS)
            return rc;
        return scount > moved ? fail(DDT_ERR_TRUNCATE, "packed send larger than receive") : DDT_SUCCESS;
    }
    // two datatypes: pack into HBM scratch, unpack from it (the reference pipelines 64 KiB
    // host chunks; here it is one launch per side, stream-ordered)
    const size_t n = std::min(scount * ssz, rcount * rsz);
    DevBuf tmp(2, s);   // an early return waits for `s` (the scratch is this thread's next call's)
    HIPCHK(tmp.alloc(n));
    rc = one_side(st, scount, sbuf, tmp.p, n, 0, &moved);
    if (rc == DDT_SUCCESS && moved)
        rc = one_side(rt, rcount, rbuf, tmp.p, moved, 1, &moved);
    if (rc != DDT_SUCCESS)
        return rc;
    HIPCHK(hipStreamSynchronize(s));
    tmp.settled();
    return scount * ssz <= rcount * rsz ? DDT_SUCCESS : fail(DDT_ERR_TRUNCATE, "send larger than receive");
}

// ---------------------------------------------------------------- external32
namespace {

int ext_plan_for(const ddt_datatype_t *t, std::shared_ptr<ExtPlan> &X)
{
    if (!t)
        return fail(DDT_ERR_BAD_PARAM, "null datatype");
    if (!(t->flags & F_COMMITTED))
        return fail(DDT_ERR_NOT_COMMITTED, "datatype not committed");
    X = get_ext_plan(const_cast<ddt_datatype *>(t));
    if (X->error)
        return fail(X->error, X->what);
    return DDT_SUCCESS;
}

}  // namespace

int ddt_pack_external_size(const char *datarep, size_t incount, const ddt_datatype_t *t,
                           ptrdiff_t *size)
{
    // ompi_datatype_pack_external_size (ompi_datatype_external.c:115-135)
    (void) datarep;
    if (!size)
        return fail(DDT_ERR_BAD_PARAM, "null size");
    std::shared_ptr<ExtPlan> X;
    int rc = ext_plan_for(t, X);
    if (rc != DDT_SUCCESS)
        return rc;
    *size = ptrdiff_t(incount * X->Se);
    return DDT_SUCCESS;
}

int ddt_pack_external(const char *datarep, const void *inbuf, size_t incount,
                      const ddt_datatype_t *t, void *outbuf, ptrdiff_t outsize, ptrdiff_t *position)
{
    // ompi_datatype_pack_external (ompi_datatype_external.c:33-70): native pack into HBM,
    // then one conversion launch into the external32 stream
    (void) datarep;
    if (!position || *position < 0 || outsize < 0 || (!outbuf && outsize))
        return fail(DDT_ERR_BAD_PARAM, "bad argument");
    std::shared_ptr<ExtPlan> X;
    int rc = ext_plan_for(t, X);
    if (rc != DDT_SUCCESS)
        return rc;
    const uint64_t need = incount * X->Se, native = incount * uint64_t(t->size);
    if (uint64_t(*position) + need > uint64_t(outsize))
        return fail(DDT_ERR_TRUNCATE, "output buffer too small");
    if (need == 0)
        return DDT_SUCCESS;
    if ((rc = ext_upload(*X)) != DDT_SUCCESS)
        return fail(rc, "external32 table upload");
    DevBuf tn(0), te(1);
    HIPCHK(tn.alloc(native));
    ddt_convertor c;
    if ((rc = prepare(&c, t, incount, inbuf, true)) != DDT_SUCCESS)
        return rc;
    struct iovec iov{tn.p, native};
    uint32_t n = 1;
    size_t md = 0;
    if ((rc = advance(&c, &iov, &n, &md, 0)) < 0)
        return rc;
    char *dst = static_cast<char *>(outbuf) + *position;
    const bool dev_out = classify(dst) == MEM_DEVICE;
    if (!dev_out)
        HIPCHK(te.alloc(need));
    HIPCHK(launch_ext(X->d_segs, uint32_t(X->segs.size()), X->d_runs, uint32_t(X->runs.size()), X->E,
                      incount, uint64_t(t->size), X->Se, tn.p, dev_out ? dst : te.p, 0, X->uniform, nullptr));
    if (!dev_out)
        HIPCHK(hipMemcpy(dst, te.p, need, hipMemcpyDeviceToHost));
    HIPCHK(hipStreamSynchronize(nullptr));
    tn.settled();
    te.settled();
    *position += ptrdiff_t(need);
    return DDT_SUCCESS;
}

int ddt_unpack_external(const char *datarep, const void *inbuf, ptrdiff_t insize,
                        ptrdiff_t *position, void *outbuf, size_t outcount, const ddt_datatype_t *t)
{
    // ompi_datatype_unpack_external (ompi_datatype_external.c:72-113)
    (void) datarep;
    if (!position || *position < 0 || insize < 0 || (!inbuf && insize))
        return fail(DDT_ERR_BAD_PARAM, "bad argument");
    std::shared_ptr<ExtPlan> X;
    int rc = ext_plan_for(t, X);
    if (rc != DDT_SUCCESS)
        return rc;
    const uint64_t need = outcount * X->Se, native = outcount * uint64_t(t->size);
    if (uint64_t(*position) + need > uint64_t(insize))
        return fail(DDT_ERR_TRUNCATE, "input buffer too small");
    if (need == 0)
        return DDT_SUCCESS;
    if ((rc = ext_upload(*X)) != DDT_SUCCESS)
        return fail(rc, "external32 table upload");
    ddt_convertor c;
    if ((rc = prepare(&c, t, outcount, outbuf, false)) != DDT_SUCCESS)
        return rc;
    const char *src = static_cast<const char *>(inbuf) + *position;
    DevBuf tn(0), te(1);
    const bool dev_in = classify(src) == MEM_DEVICE;
    if (!dev_in) {
        HIPCHK(te.alloc(need));
        HIPCHK(hipMemcpy(te.p, src, need, hipMemcpyHostToDevice));
    }
    HIPCHK(tn.alloc(native));
    HIPCHK(launch_ext(X->d_segs, uint32_t(X->segs.size()), X->d_runs, uint32_t(X->runs.size()), X->E,
                      outcount, uint64_t(t->size), X->Se, tn.p, dev_in ? const_cast<char *>(src) : te.p, 1,
                      X->uniform, nullptr));
    HIPCHK(hipStreamSynchronize(nullptr));
    struct iovec iov{tn.p, native};
    uint32_t n = 1;
    size_t md = 0;
    if ((rc = advance(&c, &iov, &n, &md, 1)) < 0)
        return rc;
    tn.settled();   // a synchronous advance ends with its stream synchronised
    te.settled();
    *position += ptrdiff_t(need);
    return DDT_SUCCESS;
}

static int window_common(const ddt_datatype_t *t, size_t count, const void *buf, size_t offset,
                         void *packed, size_t len, size_t *out_len, void *stream, int dir)
{
    if (!t || (!packed && len))
        return fail(DDT_ERR_BAD_PARAM, "bad argument");
    ddt_convertor c;
    int rc = prepare(&c, t, count, buf, dir == 0);
    if (rc != DDT_SUCCESS)
        return rc;
    c.stream = static_cast<hipStream_t>(stream);
    c.async = true;
    uint64_t w0 = std::min<uint64_t>(offset, c.local_size);
    uint64_t w1 = std::min<uint64_t>(w0 + len, c.local_size);
    std::vector<Window> dev;
    std::vector<std::pair<Window, void *>> host;
    bool pcie = false;
    if (w1 > w0) {
        uint64_t hd = 0;
        if (classify(packed) == MEM_DEVICE)
            dev.push_back({w0, w1, uint64_t(uintptr_t(packed))});
        else if ((tuning().hostdirect & (dir == 0 ? 2 : 1)) && (hd = pinned_device_range(packed, w1 - w0)) != 0) {
            dev.push_back({w0, w1, hd});   // pinned host window: the kernel moves it over PCIe
            pcie = true;
        } else {
            host.push_back({{w0, w1, 0}, packed});
        }
    }
    rc = execute(&c, dev, host, dir, pcie);
    if (rc == DDT_SUCCESS && !host.empty())
        HIPCHK(hipStreamSynchronize(c.stream));   // staging slots die with `c`
    c.stream = nullptr;
    if (out_len)
        *out_len = size_t(w1 - w0);
    return rc;
}

int ddt_pack_window(const ddt_datatype_t *t, size_t count, const void *buf, size_t offset,
                    void *dst, size_t max_len, size_t *len, void *stream)
{
    return window_common(t, count, buf, offset, dst, max_len, len, stream, 0);
}

int ddt_unpack_window(const ddt_datatype_t *t, size_t count, void *buf, size_t offset,
                      const void *src, size_t len, void *stream)
{
    return window_common(t, count, buf, offset, const_cast<void *>(src), len, nullptr, stream, 1);
}

int ddt_copy_content_same_ddt(const ddt_datatype_t *t, size_t count, void *dst, const void *src,
                              void *stream)
{
    // opal_datatype_copy_content_same_ddt (opal_datatype_copy.c:141-178): device to device,
    // one launch, user layout on both sides.
    if (!t || ((!dst || !src) && count))
        return fail(DDT_ERR_BAD_PARAM, "bad argument");
    if (!(t->flags & F_COMMITTED))
        return fail(DDT_ERR_NOT_COMMITTED, "datatype not committed");
    if (count == 0 || t->size == 0)
        return DDT_SUCCESS;
    if (classify(static_cast<const char *>(dst) + t->true_lb) != MEM_DEVICE
        || classify(static_cast<const char *>(src) + t->true_lb) != MEM_DEVICE)
        return fail(DDT_ERR_NOT_DEVICE, "typed copy needs device buffers");
    ddt_datatype *dt = const_cast<ddt_datatype *>(t);
    std::shared_ptr<Plan> P;
    try {
        P = get_plan(dt);
    } catch (const std::exception &ex) {
        return fail(DDT_ERR_OUT_OF_RESOURCE, ex.what());
    }
    std::vector<Window> w{{0, uint64_t(t->size) * count, uint64_t(uintptr_t(dst))}};
    hipStream_t s = static_cast<hipStream_t>(stream);
    int rc = run_windows(dt, *P, count, uint64_t(uintptr_t(src)), w, true, 0, s);
    if (rc != DDT_SUCCESS)
        return rc;
    HIPCHK(complete_sync(s, true));   // both sides in HBM: the signal kernel's word
    return DDT_SUCCESS;
}

int ddt_type_engine_info(const ddt_datatype_t *t, int64_t *out4)
{
    if (!t || !out4)
        return DDT_ERR_BAD_PARAM;
    if (!(t->flags & F_COMMITTED))
        return fail(DDT_ERR_NOT_COMMITTED, "datatype not committed");
    std::shared_ptr<Plan> P;
    try {
        P = get_plan(const_cast<ddt_datatype *>(t));
    } catch (const std::exception &ex) {
        return fail(DDT_ERR_OUT_OF_RESOURCE, ex.what());
    }
    std::lock_guard<SpinMutex> g(P->mu);
    out4[0] = P->sorted_state;
    out4[1] = P->sorted ? int64_t(P->sorted->dev_bytes) : 0;
    out4[2] = P->sorted ? int64_t(P->sorted->nc) : 0;
    out4[3] = P->sorted ? int64_t(P->sorted->slots) : 0;
    return DDT_SUCCESS;
}

int ddt_type_cache_info(const ddt_datatype_t *t, int64_t *out4)
{
    if (!t || !out4)
        return DDT_ERR_BAD_PARAM;
    if (!(t->flags & F_COMMITTED))
        return fail(DDT_ERR_NOT_COMMITTED, "datatype not committed");
    std::shared_ptr<Plan> P;
    try {
        P = get_plan(const_cast<ddt_datatype *>(t));
    } catch (const std::exception &ex) {
        return fail(DDT_ERR_OUT_OF_RESOURCE, ex.what());
    }
    std::lock_guard<SpinMutex> g(P->mu);
    reap(*P, false);
    out4[0] = int64_t(P->cache.size());
    out4[1] = int64_t(P->graveyard.size());
    out4[2] = int64_t(P->pinned.size());
    out4[3] = P->device;
    return DDT_SUCCESS;
}

int ddt_type_plan_info(const ddt_datatype_t *t, int64_t *out4)
{
    if (!t || !out4)
        return DDT_ERR_BAD_PARAM;
    if (!(t->flags & F_COMMITTED))
        return fail(DDT_ERR_NOT_COMMITTED, "datatype not committed");
    std::shared_ptr<Plan> P;
    try {
        P = get_plan(const_cast<ddt_datatype *>(t));
    } catch (const std::exception &ex) {
        return fail(DDT_ERR_OUT_OF_RESOURCE, ex.what());
    }
    int64_t nl = 0, maxd = 0;
    for (const Leaf &L : P->leaves) {
        nl += L.kind == LEAF_LIST;
        maxd = std::max<int64_t>(maxd, int64_t(L.dims.size()) + 1);
    }
    out4[0] = int64_t(P->leaves.size());
    out4[1] = int64_t(P->dev_bytes);
    out4[2] = nl;
    out4[3] = maxd;
    return DDT_SUCCESS;
}

int64_t ddt_type_plan_leaves(const ddt_datatype_t *t, int64_t *out, size_t cap)
{
    if (!t || !(t->flags & F_COMMITTED))
        return fail(DDT_ERR_NOT_COMMITTED, "datatype not committed");
    std::shared_ptr<Plan> P;
    try {
        P = get_plan(const_cast<ddt_datatype *>(t));
    } catch (const std::exception &ex) {
        return fail(DDT_ERR_OUT_OF_RESOURCE, ex.what());
    }
    std::vector<int64_t> v;
    for (size_t i = 0; i < P->leaves.size(); ++i) {
        const Leaf &L = P->leaves[i];
        v.push_back(L.kind);
        v.push_back(int64_t(L.kind == LEAF_AFFINE ? L.blen : L.list->total));
        v.push_back(L.kind == LEAF_AFFINE ? L.src_off : L.list_shift);
        v.push_back(L.dst_off);
        v.push_back(int64_t(L.dims.size()));
        v.push_back(int64_t(i));
        for (const LeafDim &d : L.dims) {
            v.push_back(int64_t(d.cnt));
            v.push_back(d.sstr);
            v.push_back(d.dstr);
        }
    }
    if (v.size() > cap)
        return -int64_t(v.size());
    if (out)
        std::memcpy(out, v.data(), v.size() * sizeof(int64_t));
    return int64_t(v.size());
}

int64_t ddt_type_plan_list(const ddt_datatype_t *t, size_t leaf, int64_t *disp, uint64_t *len,
                           size_t cap)
{
    if (!t || !(t->flags & F_COMMITTED))
        return fail(DDT_ERR_NOT_COMMITTED, "datatype not committed");
    std::shared_ptr<Plan> P = get_plan(const_cast<ddt_datatype *>(t));
    if (leaf >= P->leaves.size() || P->leaves[leaf].kind != LEAF_LIST)
        return fail(DDT_ERR_BAD_PARAM, "not a list leaf");
    const IndexList &X = *P->leaves[leaf].list;
    size_t n = X.nblk();
    if (n > cap)
        return -int64_t(n);
    for (size_t k = 0; k < n; ++k) {
        disp[k] = X.disp[k];
        len[k] = X.len.empty() ? X.ulen : X.len[k];
    }
    return int64_t(n);
}

int ddt_debug_host_window(const void *p, size_t n, uint64_t *device_addr)
{
    if (!device_addr)
        return DDT_ERR_BAD_PARAM;
    *device_addr = pinned_device_range(p, n);
    return *device_addr ? 1 : 0;
}

int ddt_debug_items(const ddt_datatype_t *t, size_t count, uint64_t user, uint64_t pk, uint64_t w0,
                    uint64_t w1, int same_layout, void *out, size_t cap_bytes, size_t *nitems,
                    size_t *item_size)
{
    if (!t || !(t->flags & F_COMMITTED))
        return fail(DDT_ERR_NOT_COMMITTED, "datatype not committed");
    std::shared_ptr<Plan> P = get_plan(const_cast<ddt_datatype *>(t));
    std::vector<Item> items;
    try {
        build_items(t, *P, count, user, pk, w0, w1, same_layout != 0, items);
    } catch (const std::exception &ex) {
        return fail(DDT_ERR_NOT_SUPPORTED, ex.what());
    }
    assign_tasks(items);
    stream_policy(items);
    if (item_size)
        *item_size = sizeof(Item);
    if (nitems)
        *nitems = items.size();
    if (items.size() * sizeof(Item) > cap_bytes)
        return DDT_ERR_OUT_OF_RESOURCE;
    if (out && !items.empty())
        std::memcpy(out, items.data(), items.size() * sizeof(Item));
    return DDT_SUCCESS;
}

int ddt_selftest(void)
{
    // exhaustive over small divisors, random over large ones
    uint64_t x = 0x9E3779B97F4A7C15ull;
    for (uint32_t d = 1; d < 5000; ++d) {
        FastDiv f = make_fastdiv(d);
        for (int k = 0; k < 200; ++k) {
            x ^= x << 13;
            x ^= x >> 7;
            x ^= x << 17;
            uint32_t n = uint32_t(x);
            if (k < 4)
                n = k == 0 ? 0 : (k == 1 ? 0xffffffffu : (k == 2 ? d : d - 1));
            if (fastdiv(n, f) != n / d)
                return 1;
        }
    }
    for (int k = 0; k < 200000; ++k) {
        x ^= x << 13;
        x ^= x >> 7;
        x ^= x << 17;
        uint32_t d = uint32_t(x >> 32) | 1u, n = uint32_t(x);
        if (k & 1)
            d >>= (k % 31);
        if (d == 0)
            d = 1;
        FastDiv f = make_fastdiv(d);
        if (fastdiv(n, f) != n / d || fastdiv(0xffffffffu, f) != 0xffffffffu / d)
            return 2;
    }
    return 0;
}

int ddt_trim(void)
{
    slot_trim();   // every launch-slot binding ends (its set launches with arguments until it binds again)
    return pool_trim();
}

int ddt_pool_info(int64_t *out6)
{
    if (!out6)
        return DDT_ERR_BAD_PARAM;
    pool_stats(out6);
    return DDT_SUCCESS;
}

int ddt_slot_info(int64_t *out4)
{
    if (!out4)
        return DDT_ERR_BAD_PARAM;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) {
        (void) hipGetLastError();
        dev = -1;
    }
    slot_stats(dev, out4);
    return DDT_SUCCESS;
}

int ddt_sync_info(int64_t *out3)
{
    if (!out3)
        return DDT_ERR_BAD_PARAM;
    out3[0] = g_sig_fast.load();
    out3[1] = g_sig_fallback.load();
    out3[2] = g_sig_plain.load();
    return DDT_SUCCESS;
}

int ddt_slot_state(int dir, int k)
{
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) {
        (void) hipGetLastError();
        return -1;
    }
    return (dir == 0 || dir == 1) ? slot_debug_state(dev, dir, k) : -1;
}

int ddt_tune(const char *key, long value)
{
    if (!key)
        return DDT_ERR_BAD_PARAM;
    std::string k(key);
    if (k == "nt")
        tuning().nt = value < 0 ? -1 : (value ? 1 : 0);
    else if (k == "task_kb")
        tuning().task_kb = value;
    else if (k == "interleave")
        tuning().interleave = value;
    else if (k == "uinterleave")
        tuning().uinterleave = value < 0 ? -1 : value;
    else if (k == "slots")
        tuning().slots = value ? 1 : 0;
    else if (k == "sfloor")
        tuning().sfloor = value;
    else if (k == "slot_max_kb")
        tuning().slot_max_kb = value < 0 ? 0 : value;
    else if (k == "policy")
        tuning().policy = int(value);
    else if (k == "ptr")
        tuning().ptr = value ? 1 : 0;
    else if (k == "xchunk")
        tuning().xchunk = value < 0 ? 0 : value;
    else if (k == "xcd")
        tuning().xcd = value < 0 ? -1 : (value ? 1 : 0);
    else if (k == "spol")
        tuning().spol = value;
    else if (k == "sorted")
        tuning().sorted = value;
    else if (k == "wt")
        tuning().wt = value < 0 ? -1 : int(value > 3 ? 3 : value);
    else if (k == "hostdirect")
        tuning().hostdirect = int(value & 3);
    else if (k == "hd_grid")
        tuning().hd_grid = value < 0 ? 0 : value;
    else if (k == "hd_grid_pack")
        tuning().hd_grid_pack = value < 0 ? 0 : value;
    else if (k == "s2unroll")
        tuning().s2unroll = value >= 16 ? 16 : (value >= 8 ? 8 : 4);
    else if (k == "dsplit")
        tuning().dsplit = value ? 1 : 0;
    else if (k == "sigsync")
        tuning().sigsync = value ? 1 : 0;
    else if (k == "sigspin_us")
        tuning().sigspin_us = value < 0 ? 0 : value;
    else if (k == "slayout")
        tuning().slayout = value & 3;
    else if (k == "s2vec")
        tuning().s2vec = value ? 1 : 0;
    else if (k == "sskew")
        tuning().sskew = value < 0 ? 0 : (value > (1 << 20) ? (1 << 20) : value);
    else if (k == "sstagger")
        tuning().sstagger = value < 0 ? 0 : (value > 255 ? 255 : value);
    else if (k == "sunroll")
        tuning().sunroll = value >= 32 ? 32 : (value >= 16 ? 16 : (value >= 8 ? 8 : 4));
    else if (k == "sseg")
        tuning().sseg = (value == 128 || value == 64 || value == 32) ? value : 1;
    else if (k == "schunk")
        tuning().schunk = value == 2 ? 2 : 1;
    else if (k == "sorted_commit")
        tuning().sorted_commit = value ? 1 : 0;
    else if (k == "stage_mb")
        tuning().stage_mb = value < 1 ? 1 : value;
    else if (k == "snt")
        tuning().snt = value < -2 ? -3 : (value < 0 ? int(value) : (value >= 3 && value <= 5 ? int(value) : (value ? 1 : 0)));
    else if (k == "dfast")
        tuning().dfast = int(value & 3);
    else if (k == "dense")
        tuning().dense = value < 0 ? -1 : int(value);
    else if (k == "stask")
        tuning().stask = value < 0 ? 0 : value;
    else if (k == "spass")
        tuning().spass = value < 1 ? 1 : value;
    else if (k == "consolidate")
        tuning().consolidate = value;
    else if (k == "opt_growth")
        tuning().opt_growth = value < 0 ? 0 : (value > 1024 ? 1024 : value);
    else if (k == "opt_unroll_items")
        tuning().opt_unroll_items = value < 0 ? 0 : value;
    else if (k == "opt_unroll_bytes")
        tuning().opt_unroll_bytes = value < 0 ? 0 : value;
    else if (k == "opt_preserve")
        tuning().opt_preserve = value ? 1 : 0;
    else if (k == "reset")
        tuning() = tuning_defaults();
    else
        return fail(DDT_ERR_BAD_PARAM, "unknown tuning key " + k);
    return DDT_SUCCESS;
}

const char *ddt_version(void) { return "ddt-hip 0.1 (gfx950)"; }

const char *ddt_last_error(void) { return g_last_error.c_str(); }

}  // extern "C"
