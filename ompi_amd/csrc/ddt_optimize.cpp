// ddt_optimize.cpp -- Open MPI's commit optimizer, restated for the engine's type maps.
//
// The engine's constructors build a Node tree (ddt_core.h) that mirrors opal_datatype_add's
// `desc`.  At commit the tree is written out as that description (build_opal_desc), run through
// a restatement of opal_datatype_commit's optimizer (optimize_desc), and the result is read back
// into Nodes exactly as the bridge reads a real Open MPI opt_desc (nodes_from_desc).  So the
// elements a pack fragment keeps whole and a send position snaps to -- the carriers of fused
// mixed-type regions included -- are the reference's, for every type, however it was built.
//
// Reference: opal/datatype/opal_datatype_optimize.c
//   optimize_short (:890-1295)  one pass: merge / fuse DATA, compress contiguous loops, expand
//                               short innermost loops, loop-boundary fusion, unrolling
//   short_restart (:1347-1478)  passes to a fixed point; boundary expansion kept only when it
//                               lowers the copy-range count (:406-435), growth <= 10x
//   promoted_type (:581-611)    carrier of a mixed region: widest UINT8/4/2 that tiles it and
//                               is aligned at disp (and extent when count > 1), else UINT1
// with the reference's run-time parameters (opal_datatype_module.c:85-90, registered :347-383),
// read at commit: defaults max_desc_growth 10, unroll 8 items of <= 128 bytes, preserve_type on;
// set by ddt_tune("opt_growth" / "opt_unroll_items" / "opt_unroll_bytes" / "opt_preserve") or
// their MCA environment form OMPI_MCA_opal_datatype_optimize_*.  COUNT_OPTIMIZABLE (:385-401) is a hint no mover reads and
// is not computed.
//
// Sealed lists (engine extension): an index list of more than kSealBlocks blocks (64 Mi for
// BASELINE config 4) is not expanded into one entry per block.  It enters the optimizer as one
// entry standing for its blocks [sb, se): a pass runs the pending element against its first
// blocks as it would against separate DATA entries, then the rest of the list is the greedy
// merge of its blocks from a fresh start (sealed_opt_entries, O(blocks), cached), whose last
// pending element stays pending so the next element can merge into it.  Only that greedy's
// result is kept as a block range, never expanded.  Loops holding a list are neither unrolled,
// expanded nor compressed (none of the reference's limits lets a loop of more than 2^20 items
// take those paths); a loop-boundary fusion with the list as the body's first or last item takes
// its first or last block and splits the range around it, as the reference's separate entries.
#include "ddt_optimize.h"
#include "ddt_plan.h"

#include <algorithm>
#include <cstring>
#include <map>
#include <tuple>

namespace ddt {
namespace {

constexpr uint32_t kData = F_DATA;
constexpr uint32_t kContig = F_CONTIGUOUS;
constexpr uint32_t kElemMask = 0x01FFu;                                  // OPAL_DATATYPE_FLAG_ELEM_MASK
constexpr uint32_t kBasic = F_PREDEFINED | F_CONTIGUOUS | F_NO_GAPS | F_DATA | F_COMMITTED;
constexpr uint64_t kInlineBlocklen = 8;   // OPAL_DATATYPE_PREDEFINED_MAX_INLINE_BLOCKLEN
// opal_datatype_config.optimize (opal_datatype_module.c:85-90), read at commit (ddt_plan.h Tuning)
inline uint64_t unroll_items() { return uint64_t(tuning().opt_unroll_items); }
inline uint64_t unroll_bytes() { return uint64_t(tuning().opt_unroll_bytes); }
constexpr uint16_t kNoType = 0xFFFF;

inline int64_t esz(uint16_t t) { return kOpalSize[t]; }
inline int64_t bytes_of(const DescEntry &e) { return int64_t(e.blen) * esz(e.type); }
inline uint32_t kept(uint32_t f) { return kBasic | (f & kTypeChanged); }
inline bool is_data(const DescEntry &e) { return (e.flags & kData) != 0; }

DescEntry loop_entry(uint32_t loops, uint32_t items, int64_t extent, uint32_t flags)
{
    DescEntry e;
    e.flags = uint16_t(flags & ~kData);
    e.type = kDescLoop;
    e.count = items;
    e.loops = loops;
    e.blen = ~uint64_t(0);
    e.extent = extent;
    return e;
}

DescEntry end_entry(uint32_t items, int64_t first, uint64_t size, uint32_t flags)
{
    DescEntry e;
    e.flags = uint16_t(flags & ~kData);
    e.type = kDescEndLoop;
    e.count = items;
    e.loops = ~uint32_t(0);
    e.blen = size;
    e.disp = first;
    return e;
}

// The optimized entries of blocks [k0, k1) of a sealed list from a fresh start: Pass::run's DATA
// path (:1146-1278) over them, streamed -- one element type, so no mixed regions; count-1 blocks,
// so never an inline pair -- each entry emitted as elem() writes it (CREATE_ELEM's contiguous
// collapse).  With `pend`, the final pending element is returned there instead of emitted, with
// the first block it covers in *pend_start; *merged tells whether any two blocks merged or fused.
struct SealedTail {
    DescEntry pend;
    size_t start = 0;
    bool merged = false;
};

template <class Emit>
void sealed_opt_entries(const IndexList &X, uint16_t type, uint16_t flags, int64_t disp, size_t k0, size_t k1,
                        Emit &&out, SealedTail *tail = nullptr)
{
    const uint64_t es = uint64_t(esz(type));
    auto emit = [&](DescEntry x) {
        if (x.extent == int64_t(x.blen * es)) {
            x.blen *= x.count;
            x.extent *= int64_t(x.count);
            x.count = 1;
        }
        x.flags = uint16_t(x.flags | kData);
        out(x);
    };
    DescEntry last;
    last.count = 0;
    size_t ls = k0, les = k0;   // first block of the pending entry / of its last element
    bool merged = false;
    for (size_t k = k0; k < k1; ++k) {
        const uint64_t len = X.len.empty() ? X.ulen : X.len[k];
        DescEntry cur;
        cur.flags = flags;
        cur.type = type;
        cur.count = 1;
        cur.blen = len / es;
        cur.extent = int64_t(len);
        cur.disp = disp + X.disp[k];
        if (last.count == 0) {
            last = cur;
            ls = les = k;
            continue;
        }
        if (bytes_of(last) == last.extent) {
            last.extent *= last.count;
            last.blen *= last.count;
            last.count = 1;
        }
        const int64_t lbs = bytes_of(last), cbs = bytes_of(cur);
        if (lbs == cbs) {
            if (last.extent * int64_t(last.count) + last.disp == cur.disp) {
                last.count += 1;
                les = k;
                merged = true;
                continue;
            }
            if (last.count == 1) {
                last.extent = cur.disp - last.disp;
                last.count = 2;
                les = k;
                merged = true;
                continue;
            }
        }
        if (last.disp + int64_t(last.count - 1) * last.extent + lbs == cur.disp) {   // adjacent: fuse
            const int64_t fext = last.extent + cur.extent;
            if (last.count != 1) {
                DescEntry head = last;
                head.count -= 1;
                emit(head);
                last.disp += int64_t(last.count - 1) * last.extent;
                last.count = 1;
                ls = les;
            }
            last.blen += cur.blen;
            last.extent = fext;
            merged = true;
            continue;
        }
        emit(last);
        last = cur;
        ls = les = k;
    }
    if (tail) {
        tail->pend = last;
        tail->start = ls;
        tail->merged = merged;
    } else if (last.count) {
        emit(last);
    }
}

// Fresh-start tails of sealed lists, computed once per (list, range) for all passes of a commit.
struct SealedCache {
    std::map<std::tuple<int32_t, uint32_t, uint32_t>, SealedTail> tails;
    std::map<std::tuple<int32_t, uint32_t, uint32_t>, int64_t> counts;
};

// ------------------------------------------------------------------ the optimizer
using Lists = std::vector<std::shared_ptr<const IndexList>>;

class Pass {
public:
    Pass(const std::vector<DescEntry> &d, uint32_t *flags, const Lists &lists, SealedCache &cache,
         uint32_t mask = kOptimizeAll, bool top_only = false)
        : d_(d), flags_(flags), lists_(lists), cache_(cache), mask_(mask), top_only_(top_only)
    {
    }

    // one optimize_short pass; the output keeps the END_LOOP sentinel at [used]
    void run(std::vector<DescEntry> &o, size_t &used, bool boundary, bool *expanded, bool *reevaluate);

private:
    const std::vector<DescEntry> &d_;
    uint32_t *flags_;
    const Lists &lists_;
    SealedCache &cache_;
    const uint32_t mask_;   // optimization_mask (opal_datatype.h:148-151)
    const bool top_only_;   // top_loop_boundary_only: boundary expansion of top-level loops only
    std::vector<DescEntry> *o_ = nullptr;
    bool *reeval_ = nullptr;
    // the pending element is the fresh-start tail of the sealed entry at o_[tail_at_] (blocks up
    // to tail_end_): emitted unchanged, it goes back into that entry's range instead
    bool tail_on_ = false;
    size_t tail_at_ = 0;
    uint32_t tail_end_ = 0;
    DescEntry tail_;

    bool absorb(DescEntry &last, const DescEntry &cur, bool inner);
    void emit_pending(DescEntry &last);
    void take_sealed(const DescEntry &cur, DescEntry &last, bool inner);

    // CREATE_ELEM (opal_datatype_internal.h:195-209)
    void elem(uint16_t type, uint32_t flags, uint64_t blen, uint32_t count, int64_t disp, int64_t extent)
    {
        DescEntry e;
        e.flags = uint16_t(flags | kData);
        e.type = type;
        e.count = count;
        e.blen = blen;
        e.extent = extent;
        e.disp = disp;
        if (extent == int64_t(blen * uint64_t(esz(type)))) {
            e.blen *= count;
            e.extent *= count;
            e.count = 1;
        }
        o_->push_back(e);
    }
    void put(const DescEntry &e) { o_->push_back(e); }

    uint32_t next_item(size_t pos, uint32_t item) const
    {
        const DescEntry &e = d_[pos + item];
        return e.type == kDescLoop && !is_data(e) ? item + e.count + 1 : item + 1;
    }
    bool innermost(size_t pos) const
    {
        for (uint32_t k = 1; k < d_[pos].count; ++k)
            if (d_[pos + k].type == kDescLoop && !is_data(d_[pos + k]))
                return false;
        return true;
    }
    bool holds_sealed(size_t pos) const
    {
        for (uint32_t k = 1; k < d_[pos].count; ++k)
            if (d_[pos + k].sealed >= 0)
                return true;
        return false;
    }
    uint32_t unroll_factor(size_t pos) const;
    bool as_elem(size_t pos, uint32_t item, DescEntry &out) const;
    bool compress(size_t pos, DescEntry &out) const;
    bool fuse_tail_head(const DescEntry &tail, const DescEntry &head, int64_t delta, uint32_t rcount,
                        int64_t rextent, DescEntry &fused) const;
    void copy_range(size_t pos, uint32_t from, uint32_t to, int64_t delta);
    DescEntry sealed_block(const DescEntry &s, uint32_t k) const;
    void put_sealed(const DescEntry &s, uint32_t b0, uint32_t b1, int64_t delta);
    bool loop_boundary(size_t pos);
    void unrolled(size_t pos, uint32_t f);
};

// opal_datatype_opt_collapse_elem (:539-549)
void collapse(DescEntry &e)
{
    if (e.count > 1 && e.extent == bytes_of(e)) {
        e.blen *= e.count;
        e.extent *= e.count;
        e.count = 1;
    }
}

// opal_datatype_opt_promoted_type + set_mixed_region (:581-630)
void mixed_region(DescEntry &e, int64_t bytes, uint32_t count, int64_t disp, int64_t extent)
{
    uint16_t type = 9;   // UINT1 (always when preserve_type is off, :586-588)
    for (uint16_t c : {uint16_t(12), uint16_t(11), uint16_t(10)}) {   // UINT8, UINT4, UINT2
        if (!tuning().opt_preserve)
            break;
        const uint64_t sz = uint64_t(esz(c)), al = uint64_t(kOpalAlign[c]);
        if (uint64_t(bytes) % sz || (uint64_t(disp) & (al - 1)) || (count > 1 && (uint64_t(extent) & (al - 1))))
            continue;
        type = c;
        break;
    }
    e.type = type;
    e.flags = uint16_t(kBasic | kTypeChanged);
    e.blen = uint64_t(bytes / esz(type));
    e.count = count;
    e.disp = disp;
    e.extent = extent;
    e.sealed = -1;
}

uint32_t Pass::unroll_factor(size_t pos) const   // :72-110
{
    const DescEntry &L = d_[pos], &E = d_[pos + L.count];
    if (L.loops < 4 || L.count < 2 || (L.flags & kContig) || E.type != kDescEndLoop || is_data(E))
        return 1;
    const uint32_t body = L.count - 1;
    if (unroll_items() < body)
        return 1;
    for (uint32_t k = 0; k < body; ++k) {
        const DescEntry &e = d_[pos + k + 1];
        if (!is_data(e) || e.sealed >= 0)
            return 1;
        const uint64_t ts = uint64_t(esz(e.type));
        if (!ts || !e.blen || e.blen > unroll_bytes() / ts || e.count > unroll_bytes() / (e.blen * ts))
            return 1;
    }
    const uint32_t f = std::min<uint32_t>(uint32_t(std::min<uint64_t>(unroll_items() / body, UINT32_MAX)), L.loops / 2);
    return f > 1 ? f : 1;
}

void Pass::unrolled(size_t pos, uint32_t f)   // :165-215
{
    const DescEntry &L = d_[pos], &E = d_[pos + L.count];
    const uint32_t body = L.count - 1, iters = L.loops / f, tail = L.loops % f, items = body * f;
    put(loop_entry(iters, items + 1, L.extent * f, L.flags));
    auto body_at = [&](int64_t shift) {
        for (uint32_t k = 0; k < body; ++k) {
            const DescEntry &e = d_[pos + k + 1];
            elem(e.type, kept(e.flags), e.blen, e.count, e.disp + shift, e.extent);
        }
    };
    for (uint32_t it = 0; it < f; ++it)
        body_at(int64_t(it) * L.extent);
    put(end_entry(items + 1, E.disp, E.blen * f, E.flags));
    for (uint32_t it = 0; it < tail; ++it)
        body_at(int64_t(iters * f + it) * L.extent);
}

bool Pass::as_elem(size_t pos, uint32_t item, DescEntry &out) const   // :716-734
{
    const DescEntry &e = d_[pos + item];
    if (is_data(e)) {
        if (e.sealed >= 0)
            return false;
        out = e;
        out.flags = uint16_t(kept(out.flags));
        collapse(out);
        return out.count == 1;
    }
    if (e.type == kDescLoop)
        return compress(pos + item, out) && out.count == 1;
    return false;
}

bool Pass::compress(size_t pos, DescEntry &out) const   // :641-709
{
    const DescEntry &L = d_[pos], &E = d_[pos + L.count];
    if (!(L.flags & kContig) || holds_sealed(pos))
        return false;
    uint16_t ctype = kNoType;
    uint32_t cflags = kBasic;
    uint64_t cblen = 0;
    bool homog = true, any = false;
    for (uint32_t i = 1; i < L.count; i = next_item(pos, i)) {
        DescEntry cur;
        any = true;
        if (!as_elem(pos, i, cur)) {
            homog = false;
            break;
        }
        if (ctype == kNoType) {
            ctype = cur.type;
            cblen = cur.blen;
            cflags |= cur.flags & kTypeChanged;
            continue;
        }
        if (ctype != cur.type) {
            homog = false;
            break;
        }
        cblen += cur.blen;
        cflags |= cur.flags & kTypeChanged;
    }
    if (!any)
        return false;
    if (homog) {
        const uint64_t ts = uint64_t(esz(ctype));
        if (!ts || E.blen % ts || E.blen != cblen * ts) {
            homog = false;
        } else {
            out = DescEntry{};
            out.type = ctype;
            out.flags = uint16_t(cflags);
            out.blen = E.blen / ts;
            out.count = L.loops;
            out.extent = L.extent;
            out.disp = E.disp;
        }
    }
    if (!homog)
        mixed_region(out, int64_t(E.blen), L.loops, E.disp, L.extent);
    collapse(out);
    return true;
}

bool Pass::fuse_tail_head(const DescEntry &tail, const DescEntry &head, int64_t delta, uint32_t rcount,
                          int64_t rextent, DescEntry &fused) const   // :741-786
{
    if (tail.count != 1 || head.count != 1)
        return false;
    const int64_t ts = bytes_of(tail), hs = bytes_of(head);
    if (tail.disp + ts != head.disp + delta)
        return false;
    fused = tail;
    if (tail.type == head.type) {
        fused.flags = uint16_t(kBasic | ((tail.flags | head.flags) & kTypeChanged));
        fused.blen += head.blen;
    } else {
        mixed_region(fused, ts + hs, rcount, tail.disp, rextent);
    }
    fused.count = 1;
    fused.extent = ts + hs;
    if (fused.flags & kTypeChanged)
        *flags_ |= kRestricted;
    return true;
}

void Pass::copy_range(size_t pos, uint32_t from, uint32_t to, int64_t delta)   // :515-533
{
    for (uint32_t i = from; i < to; ++i) {
        DescEntry e = d_[pos + i];
        if (is_data(e)) {
            e.flags = uint16_t(kept(e.flags));
            e.disp += delta;
        } else if (e.type == kDescEndLoop) {
            e.disp += delta;
        }
        put(e);
    }
}

// Block k of a sealed entry as the DATA element the reference holds for it (count 1).
DescEntry Pass::sealed_block(const DescEntry &s, uint32_t k) const
{
    const IndexList &X = *lists_[size_t(s.sealed)];
    const uint64_t len = X.len.empty() ? X.ulen : X.len[k];
    DescEntry b;
    b.flags = uint16_t(kept(s.flags));
    b.type = s.type;
    b.count = 1;
    b.blen = len / uint64_t(esz(s.type));
    b.extent = int64_t(len);
    b.disp = s.disp + X.disp[k];
    return b;
}

// A sealed entry restricted to blocks [b0, b1), shifted by delta (nothing when empty).
void Pass::put_sealed(const DescEntry &s, uint32_t b0, uint32_t b1, int64_t delta)
{
    if (b0 >= b1)
        return;
    DescEntry e = s;
    e.flags = uint16_t(kept(e.flags));
    e.sb = b0;
    e.se = b1;
    e.disp += delta;
    put(e);
}

bool Pass::loop_boundary(size_t pos)   // :799-888
{
    const DescEntry &L = d_[pos], &E = d_[pos + L.count];
    if (L.loops < 2)
        return false;
    // the body's top-level items; a sealed list is se - sb items of the reference's
    std::vector<uint32_t> items;
    uint64_t ref_items = L.count, nitems = 0;
    for (uint32_t i = 1; i < L.count; i = next_item(pos, i)) {
        const DescEntry &e = d_[pos + i];
        if (!(e.type == kDescLoop && !is_data(e)) && !is_data(e))
            return false;
        items.push_back(i);
        nitems += (is_data(e) && e.sealed >= 0) ? uint64_t(e.se - e.sb) : 1;
    }
    for (uint32_t i = 1; i < L.count; ++i)
        if (d_[pos + i].sealed >= 0)
            ref_items += uint64_t(d_[pos + i].se - d_[pos + i].sb) - 1;
    if (ref_items <= 2 || nitems < 2 || items.empty())
        return false;
    const uint32_t fi = items.front(), li = items.back();
    const DescEntry &F = d_[pos + fi], &T = d_[pos + li];
    const bool fs = is_data(F) && F.sealed >= 0, ls = is_data(T) && T.sealed >= 0;
    DescEntry first, last, fused;
    if (fs)
        first = sealed_block(F, F.sb);
    else if (!as_elem(pos, fi, first))
        return false;
    if (ls)
        last = sealed_block(T, T.se - 1);
    else if (!as_elem(pos, li, last))
        return false;
    if (!fuse_tail_head(last, first, L.extent, L.loops - 1, L.extent, fused))
        return false;
    // the first iteration without its last item
    if (fi == li) {
        put_sealed(F, F.sb, F.se - 1, 0);
    } else {
        copy_range(pos, fi, li, 0);
        if (ls)
            put_sealed(T, T.sb, T.se - 1, 0);
    }
    if (nitems == 2) {
        elem(fused.type, fused.flags, fused.blen, L.loops - 1, fused.disp, L.extent);
    } else {
        const size_t at = o_->size();
        put(loop_entry(L.loops - 1, 0, L.extent, L.flags));
        elem(fused.type, fused.flags, fused.blen, 1, fused.disp, fused.extent);
        if (fs)
            put_sealed(F, F.sb + 1, fi == li ? F.se - 1 : F.se, L.extent);
        if (fi != li) {
            copy_range(pos, next_item(pos, fi), li, L.extent);
            if (ls)
                put_sealed(T, T.sb, T.se - 1, L.extent);
        }
        const uint32_t steady = uint32_t(o_->size() - at);   // body entries + the END_LOOP
        (*o_)[at].count = steady;
        put(end_entry(steady, fused.disp, E.blen, L.flags));
    }
    elem(last.type, last.flags, last.blen, last.count, last.disp + int64_t(L.loops - 1) * L.extent,
         last.extent);
    return true;
}

// The DATA path of optimize_short (:1146-1278): `cur` against the pending `last`.  True when cur
// was merged or fused into last (a head of last may have been emitted); false when the caller
// emits last and makes cur the pending element.
bool Pass::absorb(DescEntry &last, const DescEntry &cur, bool inner)
{
    if (bytes_of(last) == last.extent) {
        last.extent *= last.count;
        last.blen *= last.count;
        last.count = 1;
    }
    const int64_t lbs = bytes_of(last), cbs = bytes_of(cur);
    if (lbs == cbs) {   // one entry of count last + cur
        const bool mixed = last.type != cur.type;
        int64_t mext = last.extent;
        const uint32_t mcount = last.count + cur.count;
        bool can = false;
        if (last.extent * int64_t(last.count) + last.disp == cur.disp
            && (cur.count == 1 || last.extent == cur.extent)) {
            can = true;
        } else if (last.count == 1 && (cur.count == 1 || last.disp + cur.extent == cur.disp)) {
            mext = cur.count == 1 ? cur.disp - last.disp : cur.extent;
            can = true;
        }
        if (can) {
            if (reeval_ && inner)
                *reeval_ = true;
            if (mixed) {
                mixed_region(last, lbs, mcount, last.disp, mext);
                *flags_ |= kRestricted;
            } else {
                last.flags |= cur.flags & kTypeChanged;
                last.extent = mext;
                last.count = mcount;
            }
            tail_on_ = false;
            return true;
        }
    }
    const bool inline_pair = last.count > 1 && cur.count > 1 && last.blen <= kInlineBlocklen
                             && cur.blen <= kInlineBlocklen;
    if (!inline_pair && (mask_ & kOptimizeFusion)   // (:1220-1223)
        && last.disp + int64_t(last.count - 1) * last.extent + lbs == cur.disp) {
        // fuse the last block of `last` with the first block of `cur`
        const bool shrinks = last.count == 1 && cur.count == 1;
        const int64_t fext = last.extent + cur.extent;
        if (shrinks && reeval_ && inner)
            *reeval_ = true;
        tail_on_ = false;
        if (last.count != 1) {
            elem(last.type, kept(last.flags), last.blen, last.count - 1, last.disp, last.extent);
            last.disp += int64_t(last.count - 1) * last.extent;
            last.count = 1;
        }
        if (last.type == cur.type) {
            last.flags |= cur.flags & kTypeChanged;
            last.blen += cur.blen;
        } else {
            mixed_region(last, lbs + cbs, 1, last.disp, fext);
            *flags_ |= kRestricted;
        }
        last.extent = fext;
        if (cur.count != 1) {
            elem(last.type, kept(last.flags), last.blen, last.count, last.disp, last.extent);
            last = cur;
            last.count -= 1;
            last.disp += last.extent;
        }
        return true;
    }
    return false;
}

void Pass::emit_pending(DescEntry &last)
{
    if (last.count) {
        const DescEntry &t = tail_;
        if (tail_on_ && last.flags == t.flags && last.type == t.type && last.count == t.count
            && last.blen == t.blen && last.extent == t.extent && last.disp == t.disp)
            (*o_)[tail_at_].se = tail_end_;   // the list's own tail, untouched: back into its range
        else
            elem(last.type, kept(last.flags), last.blen, last.count, last.disp, last.extent);
        last.count = 0;
    }
    tail_on_ = false;
}

// A sealed list against the pending element: its first blocks go through the DATA path like
// separate entries until one starts afresh; from there the list is its fresh-start greedy, kept
// as a block range, with that greedy's last pending element as the new pending element.
void Pass::take_sealed(const DescEntry &cur, DescEntry &last, bool inner)
{
    const IndexList &X = *lists_[size_t(cur.sealed)];
    const uint64_t es = uint64_t(esz(cur.type));
    uint32_t k = cur.sb;
    const uint32_t end = cur.se;
    if (last.count) {
        for (; k < end; ++k) {
            const uint64_t len = X.len.empty() ? X.ulen : X.len[k];
            DescEntry b;
            b.flags = cur.flags;
            b.type = cur.type;
            b.count = 1;
            b.blen = len / es;
            b.extent = int64_t(len);
            b.disp = cur.disp + X.disp[k];
            if (!absorb(last, b, inner))
                break;
        }
        if (k == end)
            return;
        emit_pending(last);
    }
    const auto key = std::make_tuple(cur.sealed, k, end);
    auto it = cache_.tails.find(key);
    if (it == cache_.tails.end()) {
        SealedTail t;
        sealed_opt_entries(X, cur.type, cur.flags, 0, k, end, [](const DescEntry &) {}, &t);
        it = cache_.tails.emplace(key, t).first;
    }
    const SealedTail &t = it->second;
    // merges among the list's own blocks happen in the first pass over them (cur.loops == 0);
    // later passes see their result, a fixed point of the same rules
    if (t.merged && cur.loops == 0 && reeval_ && inner)
        *reeval_ = true;
    last = t.pend;
    last.disp += cur.disp;
    if (t.start > k) {
        DescEntry s = cur;
        s.sb = k;
        s.se = uint32_t(t.start);
        s.loops = 1;   // in merged form from here on
        put(s);
        tail_on_ = true;
        tail_at_ = o_->size() - 1;
        tail_end_ = end;
        tail_ = last;
    }
}

void Pass::run(std::vector<DescEntry> &o, size_t &used, bool boundary, bool *expanded, bool *reevaluate)
{
    o.clear();
    o_ = &o;
    reeval_ = reevaluate;
    tail_on_ = false;
    if (expanded)
        *expanded = false;
    if (reevaluate)
        *reevaluate = false;
    // the stack: output index just past each open LOOP, and whether that loop is innermost
    std::vector<int64_t> open{-1};
    std::vector<char> inner{0};
    DescEntry last, cur;
    last.flags = 0xFFFF;
    size_t pos = 0;
    auto flush_last = [&]() { emit_pending(last); };
    while (!open.empty()) {
        const DescEntry &e = d_[pos];
        if (!is_data(e) && e.type == kDescEndLoop) {
            flush_last();
            const uint32_t items = uint32_t(int64_t(o.size()) - open.back() + 1);
            put(end_entry(items, e.disp, e.blen, e.flags));
            const int64_t at = open.back();
            open.pop_back();
            inner.pop_back();
            if (!open.empty())
                o[size_t(at - 1)].count = items;
            ++pos;
            continue;
        }
        if (!is_data(e) && e.type == kDescLoop) {
            const DescEntry L = e;
            DescEntry cmp;
            if ((L.flags & kContig) && compress(pos, cmp)) {
                if (reevaluate)
                    *reevaluate = true;
                if (cmp.flags & kTypeChanged)
                    *flags_ |= kRestricted;
                pos += L.count + 1;
                cur = cmp;
            } else {
                flush_last();
                last.type = kDescLoop;
                if (L.count <= 4 && L.loops <= 2 && innermost(pos) && !holds_sealed(pos)) {
                    // fully expand a short innermost loop (:1054-1082)
                    if (reevaluate)
                        *reevaluate = true;
                    int64_t shift = 0;
                    for (uint32_t i = 0; i < L.loops; ++i, shift += L.extent)
                        for (uint32_t j = 0; j + 1 < L.count; ++j) {
                            const DescEntry &c = d_[pos + 1 + j];
                            elem(c.type, kept(c.flags), c.blen, c.count, c.disp + shift, c.extent);
                        }
                    pos += L.count + 1;
                    continue;
                }
                if (boundary && (mask_ & kOptimizeBoundary) && (!top_only_ || open.size() == 1)
                    && loop_boundary(pos)) {   // (:1091-1101)
                    if (expanded)
                        *expanded = true;
                    pos += L.count + 1;
                    continue;
                }
                const uint32_t f = (mask_ & kOptimizeUnroll) ? unroll_factor(pos) : 1;   // (:1112-1115)
                if (f > 1) {
                    unrolled(pos, f);
                    pos += L.count + 1;
                    continue;
                }
                put(loop_entry(L.loops, L.count, L.extent, L.flags));
                open.push_back(int64_t(o.size()));
                inner.push_back(char(innermost(pos)));
                ++pos;
                continue;
            }
        } else {
            cur = e;
            cur.flags = uint16_t(kept(cur.flags));
            ++pos;
            if (cur.sealed >= 0) {
                take_sealed(cur, last, inner.back());
                continue;
            }
        }
        // DATA (or a compressed loop) against the pending element (:1146-1278)
        if (last.count == 0) {
            last = cur;
            tail_on_ = false;
            continue;
        }
        if (absorb(last, cur, inner.back()))
            continue;
        emit_pending(last);
        last = cur;
    }
    flush_last();
    used = o.size() - 1;   // the top-level END_LOOP is the sentinel
}

// opal_datatype_opt_count_range_groups_desc (:406-435); a sealed list counts its blocks
uint64_t ranges(const std::vector<DescEntry> &d, const std::vector<std::shared_ptr<const IndexList>> &lists,
                size_t from, size_t to)
{
    uint64_t r = 0;
    for (size_t pos = from; pos < to;) {
        const DescEntry &e = d[pos];
        if (is_data(e)) {
            r += e.sealed >= 0 ? uint64_t(e.se - e.sb) : e.count;
            ++pos;
        } else if (e.type == kDescLoop) {
            const uint64_t lr = (e.flags & kContig) ? 1 : ranges(d, lists, pos + 1, pos + e.count);
            r += lr * e.loops;
            pos += e.count + 1;
        } else {
            ++pos;
        }
    }
    return r;
}

}  // namespace

// ompi_datatype_desc_has_small_blocks (ompi_datatype_create_contiguous.c:52-70): a DATA entry of
// blocklen < 9 (with count > 1 when `counted`); a sealed list stands for its optimized entries
bool desc_has_small_blocks(const DescForm &d, bool counted)
{
    for (size_t i = 0; i < d.used; ++i) {
        const DescEntry &e = d.e[i];
        if (!is_data(e))
            continue;
        if (e.sealed >= 0) {
            bool hit = false;
            sealed_opt_entries(*d.lists[size_t(e.sealed)], e.type, e.flags, 0, e.sb, e.se,
                               [&](const DescEntry &x) { hit |= x.blen < 9 && (!counted || x.count > 1); });
            if (hit)
                return true;
        } else if (e.blen < 9 && (!counted || e.count > 1)) {
            return true;
        }
    }
    return false;
}

DescEntry loop_desc_entry(uint32_t loops, uint32_t items, int64_t extent, uint32_t flags)
{
    return loop_entry(loops, items, extent, flags);
}

DescEntry end_desc_entry(uint32_t items, int64_t first, uint64_t size, uint32_t flags)
{
    return end_entry(items, first, size, flags);
}

void optimize_desc(const DescForm &in, int64_t size, DescForm &out, uint32_t *flags, uint32_t mask, bool top_only)
{
    // opal_datatype_optimize_short_restart (:1347-1478) from opal_datatype_commit (:1765-1777)
    const int64_t growth = tuning().opt_growth;   // clamped to 1024 (opal_datatype_module.c:370-372)
    const int64_t limit = int64_t(in.used) * growth;
    const uint32_t init = *flags;
    // The growth cap counts entries as the reference holds them: a sealed list is nblk entries in
    // `desc` and its optimized entries (sealed_opt_entries) after a pass.  In sealed-as-one units a
    // form within `limit` is within the reference's cap too (a list never gains entries), so the
    // O(blocks) count runs only when that cheaper check fails.
    SealedCache cache;
    int64_t in_extra = 0;
    for (size_t i = 0; i < in.used; ++i)
        if (in.e[i].sealed >= 0)
            in_extra += int64_t(in.e[i].se - in.e[i].sb) - 1;
    auto over = [&](const DescForm &f) {
        if (int64_t(f.used) <= limit)
            return false;
        if (!in_extra)
            return true;
        int64_t extra = 0;
        for (size_t i = 0; i < f.used; ++i) {
            const DescEntry &x = f.e[i];
            if (x.sealed < 0)
                continue;
            const auto key = std::make_tuple(x.sealed, x.sb, x.se);
            auto it = cache.counts.find(key);
            if (it == cache.counts.end()) {
                int64_t m = 0;
                sealed_opt_entries(*in.lists[size_t(x.sealed)], x.type, x.flags, 0, x.sb, x.se,
                                   [&](const DescEntry &) { ++m; });
                it = cache.counts.emplace(key, m).first;
            }
            extra += it->second - 1;
        }
        return int64_t(f.used) + extra > (int64_t(in.used) + in_extra) * growth;
    };
    auto short_pass = [&](const std::vector<DescEntry> &src, DescForm &dst, bool boundary, bool *expanded,
                          bool *reevaluate) {
        Pass p(src, flags, in.lists, cache, mask, top_only);
        p.run(dst.e, dst.used, boundary, expanded, reevaluate);
        dst.lists = in.lists;
    };
    auto count_ranges = [&](const DescForm &f) { return ranges(f.e, in.lists, 0, f.used); };
    out = DescForm{};
    if (in.used == 0) {
        out.lists = in.lists;
        return;
    }
    DescForm cand, next, base;
    bool expanded = false, reeval = false;
    *flags = init;
    short_pass(in.e, cand, true, &expanded, &reeval);
    uint32_t cand_flags = *flags;
    bool any_expanded = expanded;
    if (expanded || reeval) {
        uint64_t cand_ranges = count_ranges(cand);
        while (expanded || reeval) {
            if (over(cand))
                break;
            bool nexp = false, nre = false;
            *flags = init | (cand_flags & kRestricted);
            short_pass(cand.e, next, true, &nexp, &nre);
            const uint64_t nr = count_ranges(next);
            if (over(next) || (nexp && nr >= cand_ranges))
                break;
            any_expanded |= nexp;
            cand_flags = *flags;
            cand = std::move(next);
            cand_ranges = nr;
            expanded = nexp;
            reeval = nre;
        }
        if (any_expanded) {
            // the non-expanding baseline, converged the same way (:1427-1474)
            *flags = init;
            reeval = false;
            short_pass(in.e, base, false, nullptr, &reeval);
            uint32_t base_flags = *flags;
            while (reeval) {
                bool nre = false;
                *flags = init | (base_flags & kRestricted);
                short_pass(base.e, next, false, nullptr, &nre);
                if (over(next))
                    break;
                base_flags = *flags;
                base = std::move(next);
                reeval = nre;
            }
            if (!(!over(cand) && cand_ranges < count_ranges(base))) {
                cand = std::move(base);
                cand_flags = base_flags;
            }
        }
    }
    *flags = init | (cand_flags & kRestricted);
    out = std::move(cand);
    // opal_datatype_opt_set_fake_end_loop (:454-465) over the optimized description
    const DescEntry &s = in.e[in.used];
    out.e.resize(out.used + 1);
    out.e[out.used] = end_entry(uint32_t(out.used), s.disp, uint64_t(size), 0);
    out.e[out.used].flags = 0;
}

// ------------------------------------------------------------------ Node tree -> desc
namespace {

struct Writer {
    DescForm &f;
    bool ok = true;

    void data(uint32_t flags, uint16_t tid, uint64_t count, uint64_t bytes, int64_t extent, int64_t disp)
    {
        const int64_t es = (tid >= 4 && tid <= 27) ? esz(tid) : 0;
        if (es <= 0 || bytes % uint64_t(es) || count > 0xffffffffull) {
            ok = false;
            return;
        }
        DescEntry e;
        e.flags = uint16_t(flags | kData);
        e.type = tid;
        e.count = uint32_t(count);
        e.blen = bytes / uint64_t(es);
        e.extent = extent;
        e.disp = disp;
        f.e.push_back(e);
    }

    static bool first_disp(const std::vector<Node> &nodes, int64_t &out)
    {
        for (const Node &n : nodes) {
            switch (n.kind) {
            case Node::DATA: out = n.disp; return true;
            case Node::LIST:
                if (n.list && n.list->nblk()) {
                    out = n.disp + n.list->disp[0];
                    return true;
                }
                break;
            case Node::LOOP:
                if (first_disp(n.body, out))
                    return true;
                break;
            }
        }
        return false;
    }

    void nodes(const std::vector<Node> &ns)
    {
        for (const Node &n : ns) {
            if (!ok)
                return;
            switch (n.kind) {
            case Node::DATA:
                data(n.flags, n.tid, n.count, n.blen, n.extent, n.disp);
                break;
            case Node::LIST: {
                const IndexList &X = *n.list;
                if (X.nblk() > kSealBlocks) {
                    DescEntry e;
                    e.flags = uint16_t(n.flags | kData);
                    e.type = n.tid;
                    e.count = 1;
                    e.blen = X.total / uint64_t(esz(n.tid));
                    e.extent = int64_t(X.total);
                    e.disp = n.disp;
                    e.sealed = int32_t(f.lists.size());
                    e.sb = 0;
                    e.se = uint32_t(X.nblk());
                    f.lists.push_back(n.list);
                    f.e.push_back(e);
                    break;
                }
                for (size_t k = 0; k < X.nblk() && ok; ++k) {
                    const uint64_t len = X.len.empty() ? X.ulen : X.len[k];
                    data(n.flags, n.tid, 1, len, int64_t(len), n.disp + X.disp[k]);
                }
                break;
            }
            case Node::LOOP: {
                if (n.count > 0xffffffffull) {
                    ok = false;
                    return;
                }
                const uint32_t lflags = n.flags & (kElemMask & ~F_COMMITTED);
                const size_t at = f.e.size();
                f.e.push_back(loop_entry(uint32_t(n.count), 0, n.extent, lflags));
                nodes(n.body);
                const uint32_t items = uint32_t(f.e.size() - at);
                f.e[at].count = items;
                int64_t first = 0;
                first_disp(n.body, first);
                f.e.push_back(end_entry(items, first, n.body_size, lflags));
                break;
            }
            }
        }
    }
};

}  // namespace

bool build_opal_desc(const std::vector<Node> &nodes, int64_t size, DescForm &out)
{
    out = DescForm{};
    Writer w{out};
    w.nodes(nodes);
    if (!w.ok)
        return false;
    out.used = out.e.size();
    int64_t first = 0;
    if (size != 0)
        Writer::first_disp(nodes, first);
    DescEntry s = end_entry(uint32_t(out.used), first, uint64_t(size), 0);
    s.flags = 0;
    out.e.push_back(s);
    return true;
}

void encode_desc(const DescForm &d, std::vector<unsigned char> &out, bool optimized)
{
    out.clear();
    auto put = [&](uint16_t flags, uint16_t type, uint32_t a, uint32_t b, uint64_t c, int64_t x, int64_t y) {
        unsigned char p[32] = {0};
        std::memcpy(p, &flags, 2);
        std::memcpy(p + 2, &type, 2);
        std::memcpy(p + 4, &a, 4);
        if (!(flags & kData) && (type == kDescLoop || type == kDescEndLoop)) {
            std::memcpy(p + 8, &b, 4);
            std::memcpy(p + 16, &c, 8);
            std::memcpy(p + 24, type == kDescLoop ? &x : &y, 8);
        } else {
            std::memcpy(p + 8, &c, 8);
            std::memcpy(p + 16, &x, 8);
            std::memcpy(p + 24, &y, 8);
        }
        out.insert(out.end(), p, p + 32);
    };
    // a sealed list expands into many entries: the LOOP / END_LOOP pairs around it count the
    // entries actually written (CREATE_LOOP_START / _END items, opal_datatype_internal.h:171-189)
    std::vector<size_t> open;
    for (size_t i = 0; i < d.used; ++i) {
        const DescEntry &e = d.e[i];
        if (!(e.flags & kData) && e.type == kDescLoop) {
            open.push_back(out.size() / 32);
        } else if (!(e.flags & kData) && e.type == kDescEndLoop && !open.empty()) {
            const size_t at = open.back();
            open.pop_back();
            const uint32_t items = uint32_t(out.size() / 32 - at);
            std::memcpy(out.data() + 32 * at + 4, &items, 4);
            put(e.flags, e.type, items, e.loops, e.blen, e.extent, e.disp);
            continue;
        }
        if (e.sealed >= 0) {
            const IndexList &X = *d.lists[size_t(e.sealed)];
            const uint64_t es = uint64_t(esz(e.type));
            if (!optimized) {
                for (size_t k = e.sb; k < e.se; ++k) {
                    const uint64_t len = X.len.empty() ? X.ulen : X.len[k];
                    put(e.flags, e.type, 1, 0, len / es, int64_t(len), e.disp + X.disp[k]);
                }
                continue;
            }
            sealed_opt_entries(X, e.type, e.flags, e.disp, e.sb, e.se, [&](const DescEntry &x) {
                put(x.flags, x.type, x.count, 0, x.blen, x.extent, x.disp);
            });
            continue;
        }
        put(e.flags, e.type, e.count, e.loops, e.blen, e.extent, e.disp);
    }
}

}  // namespace ddt
