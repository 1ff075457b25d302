// ddt_external.cpp -- the external32 signature of a committed type.
//
// MPI_Pack_external runs the reference's convertor with the external32 architecture
// (ompi_datatype_external.c:33-135, ompi_datatype_external32.c:35-38: big endian, bool
// 1 byte, long 4 bytes).  The heterogeneous copy functions then convert element by
// element in type-map order (opal_copy_functions_heterogeneous.c:1361-1393):
//   1-byte types are copied (the swap mask skips them, opal_convertor.c:191-203);
//   LONG / UNSIGNED_LONG shrink to 4 bytes on pack and are sign / zero extended on
//     unpack (copy_long_heterogeneous :1094-1223, unsigned :1225-1360);
//   complex types swap each component (COPY_2SAMETYPE_HETEROGENEOUS :776-842);
//   everything else is byte-swapped whole (opal_dt_swap_bytes :49-70).
// Long double types follow the gcc x86-64 build (x87 long double in 16 bytes, _Float128
// available): FLOAT12 (long double, MPI_LONG_DOUBLE) and FLOAT16 (_Float128) swap their 16
// bytes whole (COPY_TYPE_HETEROGENEOUS without the long-double flag, :1033-1034, :1058-1059);
// LONG_DOUBLE_COMPLEX converts each component x87 <-> IEEE quad (:779-842 with ldbl_to_f128 /
// f128_to_ldbl, :488-590), CONV_LDBL; FLOAT128_COMPLEX, whose reference copy treats quad
// components as long doubles (:1082-1083), is refused.
//
// The engine keeps the type map's element ids on the uncommitted description (Node::tid).
// This file compresses that sequence into segments: `reps` repetitions of a short body of
// same-type runs.  ddt_ext_kernel walks them with one thread per element.
// hvector(128 Mi, 1, 32 B) of struct{double, int[3]} is ONE segment of two runs.
#include <stdexcept>

#include <hip/hip_runtime.h>

#include "ddt_core.h"
#include "ddt_hip.h"
#include "ddt_plan.h"
#include "ddt_pool.h"

namespace ddt {

namespace {

constexpr size_t kBodyMax = 1024;      // runs kept in one repeated body
constexpr size_t kSegMax = 1u << 16;   // segments per instance before refusing
constexpr size_t kRunMax = 1u << 22;   // runs (all segments) before refusing

thread_local size_t g_runs = 0;        // runs appended while flattening one type

// external32 element bytes per OPAL id (-1: no portable form), opal_convertor.c:146-172
const int kExtSize[29] = {0, 0, 0, 0, 1, 2, 4, 8, 16, 1, 2, 4, 8, 16, 2,
                          4, 8, 16, 16, 4, 8, 16, 32, 1, 4, 4, 4, -1, 0};
const int kNatSize[29] = {0, 0, 0, 0, 1, 2, 4, 8, 16, 1, 2, 4, 8, 16, 2,
                          4, 8, 16, 16, 4, 8, 16, 32, 1, 4, 8, 8, 32, 0};

struct SigRun {
    uint16_t tid;
    uint64_t n;
};
struct Seg {
    uint64_t reps;
    std::vector<SigRun> runs;
};
using Flat = std::vector<Seg>;

void append_run(Flat &f, uint16_t tid, uint64_t n)
{
    if (n == 0)
        return;
    if (f.empty() || f.back().reps != 1)
        f.push_back({1, {}});
    auto &r = f.back().runs;
    if (!r.empty() && r.back().tid == tid) {
        r.back().n += n;
        return;
    }
    if (++g_runs > kRunMax)
        throw std::length_error("external32 signature too irregular");
    r.push_back({tid, n});
}

void append_seg(Flat &f, const Seg &s)
{
    if (s.reps == 1) {
        for (const SigRun &r : s.runs)
            append_run(f, r.tid, r.n);
    } else if (s.runs.size() == 1) {
        append_run(f, s.runs[0].tid, s.runs[0].n * s.reps);
    } else {
        g_runs += s.runs.size();
        if (g_runs > kRunMax)
            throw std::length_error("external32 signature too irregular");
        f.push_back(s);
    }
}

uint64_t elem_count(const Node &n, uint64_t bytes)
{
    if (n.tid < 4 || n.tid > 27 || n.esize <= 0)
        throw std::runtime_error("type map element without a basic type id");
    return bytes / uint64_t(n.esize);
}

Flat flatten(const std::vector<Node> &nodes)
{
    Flat f;
    for (const Node &n : nodes) {
        switch (n.kind) {
        case Node::DATA:
            append_run(f, n.tid, elem_count(n, n.count * n.blen));
            break;
        case Node::LIST:
            if (n.list)
                append_run(f, n.tid, elem_count(n, n.list->total));
            break;
        case Node::LOOP: {
            if (n.count == 0)
                break;
            Flat b = flatten(n.body);
            if (b.empty())
                break;
            if (b.size() == 1 && b[0].runs.size() <= kBodyMax) {
                append_seg(f, {b[0].reps * n.count, b[0].runs});
                break;
            }
            if (n.count * b.size() > kSegMax)
                throw std::length_error("external32 signature too irregular");
            for (uint64_t c = 0; c < n.count; ++c)
                for (const Seg &s : b)
                    append_seg(f, s);
            break;
        }
        }
        if (f.size() > kSegMax)
            throw std::length_error("external32 signature too irregular");
    }
    return f;
}

}  // namespace

ExtPlan::~ExtPlan()
{
    // external32 calls run on the default stream and synchronise it before returning; the
    // tables still go to the pool behind a fence on that stream (no device-wide wait, no
    // hipFree: see ddt_pool.h)
    if (!d_segs && !d_runs)
        return;
    std::vector<void *> blocks{d_segs, d_runs};
    std::vector<hipEvent_t> fences;
    bool unknown = false;
    if (pool_fences({hipStream_t(nullptr)}, fences, unknown)) {
        pool_release(blocks, fences, unknown);
    } else {
        for (hipEvent_t e : fences)
            (void) hipEventDestroy(e);
        for (void *p : blocks)
            pool_keep(p);
    }
}

std::shared_ptr<ExtPlan> get_ext_plan(ddt_datatype *t)
{
    std::lock_guard<ddt::SpinMutex> g(t->plan_mu);
    if (t->ext)
        return t->ext;
    auto X = std::make_shared<ExtPlan>();
    try {
        g_runs = 0;
        Flat f = flatten(t->desc);
        uint64_t e0 = 0, nb = 0, eb = 0;
        for (const Seg &s : f) {
            ConvSeg cs{};
            cs.e0 = e0;
            cs.reps = s.reps;
            cs.nbase = nb;
            cs.ebase = eb;
            cs.run0 = uint32_t(X->runs.size());
            cs.nruns = uint32_t(s.runs.size());
            uint64_t be = 0, bn = 0, bx = 0;
            for (const SigRun &r : s.runs) {
                const int xs = kExtSize[r.tid], ns = kNatSize[r.tid];
                if (xs < 0) {
                    X->error = DDT_ERR_NOT_SUPPORTED;
                    X->what = "external32: FLOAT128_COMPLEX is not converted (the reference passes its "
                              "quad components through ldbl_to_f128, opal_copy_functions_heterogeneous.c:1082)";
                    break;
                }
                ConvRun cr{};
                cr.e0 = be;
                cr.noff = bn;
                cr.eoff = bx;
                cr.nsz = uint32_t(ns);
                cr.esz = uint32_t(xs);
                if (r.tid == 25)
                    cr.kind = CONV_LONG;
                else if (r.tid == 26)
                    cr.kind = CONV_ULONG;
                else if (r.tid == 22)
                    cr.kind = CONV_LDBL;
                else
                    cr.kind = ns == 1 ? CONV_COPY : CONV_SWAP;
                cr.comp = r.tid == 19 ? 2 : r.tid == 20 ? 4 : r.tid == 21 ? 8 : uint32_t(ns);
                X->runs.push_back(cr);
                be += r.n;
                bn += r.n * uint64_t(ns);
                bx += r.n * uint64_t(xs);
            }
            if (X->error)
                break;
            cs.body_elems = be;
            cs.nbody = bn;
            cs.ebody = bx;
            X->segs.push_back(cs);
            e0 += be * s.reps;
            nb += bn * s.reps;
            eb += bx * s.reps;
        }
        if (!X->error) {
            if (nb != uint64_t(t->size))
                throw std::logic_error("external32 signature does not cover the type size");
            X->E = e0;
            X->Se = eb;
            uint32_t c = X->runs.empty() ? 0 : X->runs[0].comp;
            for (const ConvRun &r : X->runs)
                if ((r.kind != CONV_COPY && r.kind != CONV_SWAP) || r.nsz != r.esz || r.comp != c)
                    c = 0;
            X->uniform = (c == 1 || c == 2 || c == 4 || c == 8 || c == 16) ? c : 0;
        }
    } catch (const std::length_error &ex) {
        X->error = DDT_ERR_NOT_SUPPORTED;
        X->what = ex.what();
    } catch (const std::exception &ex) {
        X->error = DDT_ERR_BAD_PARAM;
        X->what = ex.what();
    }
    t->ext = X;
    return X;
}

// Upload the segment tables (first conversion only; caller holds no lock).
int ext_upload(ExtPlan &X)
{
    static std::mutex mu;
    std::lock_guard<std::mutex> g(mu);
    if (X.d_segs || X.segs.empty())
        return DDT_SUCCESS;
    const size_t sb = X.segs.size() * sizeof(ConvSeg), rb = X.runs.size() * sizeof(ConvRun);
    ConvSeg *ds = nullptr;
    ConvRun *dr = nullptr;
    if (!(ds = static_cast<ConvSeg *>(pool_alloc(sb))) || !(dr = static_cast<ConvRun *>(pool_alloc(rb)))
        || upload(ds, X.segs.data(), sb) != hipSuccess
        || upload(dr, X.runs.data(), rb) != hipSuccess) {
        pool_free(ds);
        pool_free(dr);
        return DDT_ERR_HIP;
    }
    X.d_runs = dr;
    X.d_segs = ds;
    return DDT_SUCCESS;
}

}  // namespace ddt
