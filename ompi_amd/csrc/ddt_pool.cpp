// ddt_pool.cpp -- the engine's device-memory cache (see ddt_pool.h).
#include "ddt_pool.h"

#include <map>
#include <mutex>
#include <unordered_map>

#include "ddt_hip.h"

namespace ddt {

namespace {

constexpr size_t kAlign = 256;
// Free blocks a device's cache may hold before a new hipMalloc hands the largest back to HIP
// (staging and scratch blocks of different sizes must not pile up for good).
constexpr size_t kCacheCap = size_t(1) << 30;

struct Block {
    size_t bytes = 0;
    int device = 0;
    int state = 0;   // 0 in use, 1 free, 2 waiting on fences, 3 kept for a captured graph
};

struct Pending {
    std::vector<void *> blocks;
    std::vector<hipEvent_t> fences;
    bool unknown = false;
};

struct Pool {
    std::mutex mu;
    std::unordered_map<void *, Block> blocks;
    std::map<int, std::multimap<size_t, void *>> free;   // device -> size -> block
    std::vector<Pending> pending;
};

thread_local int t_no_device_sync = 0;

Pool &pool()
{
    static Pool *p = new Pool();   // never destroyed: blocks may be released at exit
    return *p;
}

bool passed(const std::vector<hipEvent_t> &evs)
{
    for (hipEvent_t e : evs) {
        const hipError_t r = hipEventQuery(e);
        if (r != hipSuccess) {
            (void) hipGetLastError();   // hipErrorNotReady is not a launch error
            return false;
        }
    }
    return true;
}

void to_free(Pool &P, void *p)   // P.mu held
{
    Block &b = P.blocks[p];
    b.state = 1;
    P.free[b.device].emplace(b.bytes, p);
}

// Move released blocks whose fences have all passed to the free lists.
void reap(Pool &P)   // P.mu held
{
    for (size_t i = 0; i < P.pending.size();) {
        Pending &r = P.pending[i];
        if (r.unknown || !passed(r.fences)) {
            ++i;
            continue;
        }
        for (hipEvent_t e : r.fences)
            (void) hipEventDestroy(e);
        for (void *p : r.blocks)
            to_free(P, p);
        P.pending.erase(P.pending.begin() + long(i));
    }
}

// Before a new hipMalloc -- a call that already waits for the device and breaks a foreign
// global-mode capture, so nothing is lost by freeing here too: blocks released behind a stream
// that could take no fence (destroyed before the plan or convertor) are settled by one device
// synchronisation, and the largest cached blocks go back to HIP until the cache is within
// kCacheCap.
// A device synchronisation settles only the current device's work, so only releases whose
// blocks all live on `dev` settle here; another device's settle at its own next
// hipMalloc.
bool on_device(const Pool &P, const Pending &r, int dev)   // P.mu held
{
    for (void *p : r.blocks) {
        auto it = P.blocks.find(p);
        if (it == P.blocks.end() || it->second.device != dev)
            return false;
    }
    return true;
}

void settle_and_cap(Pool &P, int dev)   // P.mu held
{
    bool unknown = false;
    for (const Pending &r : P.pending)
        unknown |= r.unknown && on_device(P, r, dev) && !t_no_device_sync;
    if (unknown && hipDeviceSynchronize() == hipSuccess) {
        for (size_t i = 0; i < P.pending.size();) {
            Pending &r = P.pending[i];
            if (!r.unknown || !on_device(P, r, dev)) {
                ++i;
                continue;
            }
            for (hipEvent_t e : r.fences)
                (void) hipEventDestroy(e);
            for (void *p : r.blocks)
                to_free(P, p);
            P.pending.erase(P.pending.begin() + long(i));
        }
    }
    (void) hipGetLastError();
    auto &fl = P.free[dev];
    size_t cached = 0;
    for (auto &sb : fl)
        cached += sb.first;
    while (cached > kCacheCap && !fl.empty()) {
        auto last = std::prev(fl.end());
        cached -= last->first;
        (void) hipFree(last->second);
        P.blocks.erase(last->second);
        fl.erase(last);
    }
}

void *take_free(Pool &P, int dev, size_t bytes)   // P.mu held
{
    auto &fl = P.free[dev];
    auto it = fl.lower_bound(bytes);
    if (it == fl.end() || it->first > 2 * bytes + kAlign)
        return nullptr;
    void *p = it->second;
    fl.erase(it);
    P.blocks[p].state = 0;
    return p;
}

}  // namespace

PoolNoDeviceSync::PoolNoDeviceSync(bool on_) : on(on_)
{
    if (on)
        ++t_no_device_sync;
}
PoolNoDeviceSync::~PoolNoDeviceSync()
{
    if (on)
        --t_no_device_sync;
}

void *pool_alloc(size_t bytes)
{
    Pool &P = pool();
    bytes = (std::max<size_t>(bytes, 1) + kAlign - 1) / kAlign * kAlign;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) {
        (void) hipGetLastError();
        return nullptr;
    }
    std::lock_guard<std::mutex> g(P.mu);
    reap(P);
    if (void *p = take_free(P, dev, bytes))
        return p;
    settle_and_cap(P, dev);
    if (void *p = take_free(P, dev, bytes))
        return p;
    void *p = nullptr;
    if (hipMalloc(&p, bytes) != hipSuccess) {
        (void) hipGetLastError();
        // out of device memory: hand this device's cached blocks of other sizes back to HIP
        // (hipFree waits for the device: the exceptional path only) and try once more
        auto &fl = P.free[dev];
        if (fl.empty())
            return nullptr;
        for (auto &sb : fl) {
            (void) hipFree(sb.second);
            P.blocks.erase(sb.second);
        }
        fl.clear();
        if (hipMalloc(&p, bytes) != hipSuccess) {
            (void) hipGetLastError();
            return nullptr;
        }
    }
    P.blocks[p] = Block{bytes, dev, 0};
    return p;
}

void pool_free(void *p)
{
    if (!p)
        return;
    Pool &P = pool();
    std::lock_guard<std::mutex> g(P.mu);
    auto it = P.blocks.find(p);
    if (it == P.blocks.end() || it->second.state != 0)
        return;
    to_free(P, p);
}

void pool_free_now(void *p)
{
    if (!p)
        return;
    Pool &P = pool();
    std::lock_guard<std::mutex> g(P.mu);
    auto it = P.blocks.find(p);
    if (it == P.blocks.end() || it->second.state != 0)
        return;
    P.blocks.erase(it);
    (void) hipFree(p);
    (void) hipGetLastError();
}

void pool_release(const std::vector<void *> &blocks, const std::vector<hipEvent_t> &fences, bool unknown)
{
    Pool &P = pool();
    std::lock_guard<std::mutex> g(P.mu);
    Pending r;
    r.fences = fences;
    r.unknown = unknown;
    for (void *p : blocks) {
        auto it = p ? P.blocks.find(p) : P.blocks.end();
        if (it == P.blocks.end() || it->second.state != 0)
            continue;
        it->second.state = 2;
        r.blocks.push_back(p);
    }
    if (r.blocks.empty() && !r.unknown) {
        for (hipEvent_t e : r.fences)
            (void) hipEventDestroy(e);
        return;
    }
    P.pending.push_back(std::move(r));
}

void pool_keep(void *p)
{
    if (!p)
        return;
    Pool &P = pool();
    std::lock_guard<std::mutex> g(P.mu);
    auto it = P.blocks.find(p);
    if (it != P.blocks.end() && it->second.state == 0)
        it->second.state = 3;
}

bool pool_fences(const std::vector<hipStream_t> &streams, std::vector<hipEvent_t> &fences, bool &unknown)
{
    for (hipStream_t s : streams) {
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        if (hipStreamIsCapturing(s, &cs) != hipSuccess) {
            (void) hipGetLastError();   // a destroyed stream: its work cannot be fenced
            unknown = true;
            continue;
        }
        if (cs != hipStreamCaptureStatusNone)
            return false;
        hipEvent_t e = nullptr;
        if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess || hipEventRecord(e, s) != hipSuccess) {
            (void) hipGetLastError();
            if (e)
                (void) hipEventDestroy(e);
            unknown = true;
            continue;
        }
        fences.push_back(e);
    }
    return true;
}

int pool_trim()
{
    Pool &P = pool();
    std::lock_guard<std::mutex> g(P.mu);
    int cur = 0;
    if (hipGetDevice(&cur) != hipSuccess)
        return DDT_ERR_HIP;
    std::map<int, bool> devs;
    for (auto &kv : P.blocks)
        devs[kv.second.device] = true;
    for (auto &d : devs) {
        if (hipSetDevice(d.first) != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
            (void) hipGetLastError();
            (void) hipSetDevice(cur);
            return DDT_ERR_HIP;
        }
    }
    (void) hipSetDevice(cur);
    for (Pending &r : P.pending) {
        for (hipEvent_t e : r.fences)
            (void) hipEventDestroy(e);
        for (void *p : r.blocks)
            to_free(P, p);
    }
    P.pending.clear();
    for (auto &kv : P.free) {
        for (auto &sb : kv.second) {
            (void) hipFree(sb.second);
            P.blocks.erase(sb.second);
        }
        kv.second.clear();
    }
    return DDT_SUCCESS;
}

void pool_stats(int64_t *out)
{
    // no reap here (no event queries): safe while another thread captures in global mode
    Pool &P = pool();
    std::lock_guard<std::mutex> g(P.mu);
    for (int i = 0; i < 6; ++i)
        out[i] = 0;
    for (auto &kv : P.blocks) {
        const Block &b = kv.second;
        if (b.state == 1) {
            out[0] += 1;
            out[1] += int64_t(b.bytes);
        } else if (b.state == 2) {
            out[2] += 1;
            out[3] += int64_t(b.bytes);
        } else if (b.state == 3) {
            out[4] += 1;
        } else {
            out[5] += 1;
        }
    }
}

}  // namespace ddt
