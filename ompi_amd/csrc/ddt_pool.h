// ddt_pool.h -- device memory of the engine's own metadata (descriptor sets, index lists,
// address-ordered tables, staging and scratch buffers).
//
// hipFree synchronises the whole device (the ROCm header says so) and fails -- invalidating
// the capture -- while another thread captures a stream in global mode.  The reference frees
// a datatype's description at once in opal_datatype_destruct (opal_datatype_create.c:61-91),
// host memory no queued work reads.  Here queued kernels may still read a plan's device
// memory, so a destroyed plan hands its blocks to this pool behind fence events recorded on
// the streams that launched it, and the pool reuses them once the fences have passed.
// Memory goes back to HIP only in ddt_trim() (a synchronising call, like torch's
// empty_cache).  Blocks a captured graph may read are never reused.
#pragma once

#include <cstddef>
#include <cstdint>
#include <vector>

#include <hip/hip_runtime.h>

namespace ddt {

// `bytes` of device memory on the current device: a cached block of at least that size (at
// most twice it; released blocks whose fences have passed count as cached), else hipMalloc; when that fails, the device's cached blocks go back to HIP and hipMalloc is tried
// once more.  nullptr when HIP is out of memory.
void *pool_alloc(size_t bytes);
// A block no queued work reads any more: reusable at once.
void pool_free(void *p);
// A block no queued work reads any more, handed straight back to HIP (hipFree waits for the
// device): the end of a synchronous call's multi-GiB scratch, which the pool should not keep.
void pool_free_now(void *p);
// Blocks that queued work may still read: reusable once every event in `fences` has passed.
// `unknown` (a launching stream that could take no event) keeps them until the next pool_alloc
// that has to call hipMalloc settles them with one device synchronisation (or ddt_trim()).  The
// cache of free blocks is capped at 1 GiB per device at that same point.  A stream that launched
// a datatype's work must stay valid until the datatype (and a convertor using it) is destroyed:
// the fences are recorded on it, and HIP does not detect a destroyed stream handle (using one
// crashes the runtime, round 4), as CUDA leaves it undefined.
// The pool owns and destroys the events.
void pool_release(const std::vector<void *> &blocks, const std::vector<hipEvent_t> &fences, bool unknown);
// A block a captured graph holds: never reused, never freed.
void pool_keep(void *p);
// Fence events for work queued on `streams` so far: one event per stream that is not being
// captured.  Returns false when a stream is capturing (a graph may hold the memory) -- the
// caller keeps the blocks for good -- and sets `unknown` for a stream that took no event.
bool pool_fences(const std::vector<hipStream_t> &streams, std::vector<hipEvent_t> &fences, bool &unknown);
// ddt_trim: synchronise the device, hand every reusable and fenced block back to HIP.
int pool_trim();
// While one lives on a thread, that thread's allocations never settle unknown releases by a
// device synchronisation (the one call a relaxed-mode thread still may not make during another
// thread's capture, profiles/r5_probe_capture.log): table builds at commit / import run under it.
// `on` false: no effect (the hot path enables it only while a capture is seen, ADVICE r5, so its
// allocations still settle such releases otherwise).
struct PoolNoDeviceSync {
    explicit PoolNoDeviceSync(bool on = true);
    ~PoolNoDeviceSync();
    bool on;
    PoolNoDeviceSync(const PoolNoDeviceSync &) = delete;
    PoolNoDeviceSync &operator=(const PoolNoDeviceSync &) = delete;
};
// out[0..5] = blocks cached free, bytes cached free, blocks waiting on fences, bytes waiting,
// blocks kept for captured graphs, blocks in use.  Fences are checked only by pool_alloc (an
// event query invalidates another thread's global-mode capture; so does any allocation).
void pool_stats(int64_t *out6);

}  // namespace ddt
