// ddt_typemap.cpp -- MPI derived-datatype construction and commit for the MI355X engine.
//
// Bounds, size and flag bookkeeping follow opal_datatype_add
// (opal/datatype/opal_datatype_add.c:133-460); the constructors issue the same
// sequence of adds as ompi/datatype/ompi_datatype_create_*.c, so lb/ub/extent,
// true bounds and the type-map order are those of the reference.  The type-map
// representation itself is the engine's own (ddt_core.h).
#include <algorithm>
#include <cstring>
#include <numeric>

#include "ddt_core.h"
#include "ddt_hip.h"
#include "ddt_optimize.h"
#include "ddt_plan.h"

using namespace ddt;

namespace {

constexpr const int64_t *kSize = kOpalSize;
constexpr const int64_t *kAlign = kOpalAlign;
constexpr uint32_t kElemFlags = 0x01FFu & ~F_COMMITTED;   // OPAL_DATATYPE_FLAG_ELEM_MASK w/o COMMITTED

constexpr size_t kListMin = 8;       // indexed runs longer than this become LIST nodes
constexpr size_t kPatternMax = 256;  // max element starts kept for a merged mixed block

ddt_datatype g_predef[29];
std::once_flag g_predef_once;

void init_predefined()
{
    // OPAL_DATATYPE_LB / _UB (opal_datatype_constructors.h:77-85, 169-172): size 0, no
    // description, bounds markers only (MPI_LB / MPI_UB, ompi_datatype_module.c:92-93)
    for (int id = 2; id <= 3; ++id) {
        ddt_datatype &t = g_predef[id];
        t.id = uint16_t(id);
        t.lb = t.ub = t.true_lb = t.true_ub = 0;
        t.align = 0;
        t.nbElems = 1;
        t.flags = F_PREDEFINED;
        t.bdt_used = 1u << id;   // OPAL_DATATYPE_INIT_BASIC_TYPE (opal_datatype_constructors.h:77-85)
    }
    for (int id = 4; id <= 27; ++id) {
        ddt_datatype &t = g_predef[id];
        t.id = uint16_t(id);
        t.size = kSize[id];
        t.lb = 0;
        t.ub = kSize[id];
        t.true_lb = 0;
        t.true_ub = kSize[id];
        t.align = kAlign[id];
        t.nbElems = 1;
        t.bdt_used = 1u << id;   // OPAL_DATATYPE_INIT_BASIC_DATATYPE (:87-96)
        t.flags = F_PREDEFINED | F_CONTIGUOUS | F_NO_GAPS | F_DATA | F_COMMITTED;
        Node n;
        n.kind = Node::DATA;
        n.esize = kSize[id];
        n.tid = uint16_t(id);
        n.count = 1;
        n.blen = uint64_t(kSize[id]);
        n.extent = kSize[id];
        n.disp = 0;
        // desc[0] of a predefined type (opal_datatype_module.c:418-426)
        n.flags = F_PREDEFINED | F_DATA | F_CONTIGUOUS | F_NO_GAPS;
        t.desc.push_back(n);
        t.opt = t.desc;
        t.opt_prefix = {0, uint64_t(kSize[id])};
    }
}

void shift_nodes(std::vector<Node> &nodes, int64_t d)
{
    for (Node &n : nodes) {
        if (n.kind == Node::LOOP)
            shift_nodes(n.body, d);
        else
            n.disp += d;
    }
}

bool is_predefined(const ddt_datatype *t) { return (t->flags & F_PREDEFINED) && t->id != 0; }

// Bounds / size / flags of opal_datatype_add (opal_datatype_add.c:133-460).  Returns the
// previous true_ub (for the contiguity test) or sets *skip when nothing is appended.
struct AddState {
    int64_t old_true_ub;
    bool skip;
};

// opal_datatype_add treats an extent of -1 as "use the added type's ub - lb"
// (opal_datatype_add.c:156-161), including when a constructor computed -1 from a
// negative stride; reproduced so bounds and type map match the reference.
inline int64_t effective_extent(const ddt_datatype *add, int64_t extent)
{
    return extent == -1 ? add->ub - add->lb : extent;
}

AddState add_bounds(ddt_datatype *base, const ddt_datatype *add, uint64_t count, int64_t disp,
                    int64_t extent)
{
    AddState st{0, true};
    if (count == 0)
        return st;
    extent = effective_extent(add, extent);
    if (add->id == 2 || add->id == 3) {
        // the LB / UB markers (:158-186): move the bound to disp, nothing is appended; the id
        // survives a dup (opal_datatype_clone.c:74), so a duplicated marker is one too
        base->bdt_used |= 1u << add->id;   // (:163, :175)
        if (add->id == 2) {
            base->lb = (base->flags & F_USER_LB) ? std::min(base->lb, disp) : disp;
            base->flags |= F_USER_LB;
        } else {
            base->ub = (base->flags & F_USER_UB) ? std::max(base->ub, disp) : disp;
            base->flags |= F_USER_UB;
        }
        // (wrapping: the other bound may still be the constructor's INT64_MIN / MAX)
        if (int64_t(uint64_t(base->ub) - uint64_t(base->lb)) != base->size)
            base->flags &= ~F_NO_GAPS;
        return st;
    }
    int64_t lb, ub;
    {   // OPAL_DATATYPE_LB_UB_CONT (:98-116)
        int64_t upper = disp + extent * int64_t(count - 1), lower = disp;
        if (lower < upper) {
            lb = lower;
            ub = upper;
        } else {
            lb = upper;
            ub = lower;
        }
        lb += add->lb;
        ub += add->ub;
    }
    int64_t true_lb = lb - (add->lb - add->true_lb);
    int64_t true_ub = ub - (add->ub - add->true_ub);
    if (true_lb > true_ub)
        std::swap(true_lb, true_ub);
    if ((add->flags ^ base->flags) & F_USER_LB) {
        if (base->flags & F_USER_LB)
            lb = base->lb;
        base->flags |= F_USER_LB;
    } else {
        lb = std::min(base->lb, lb);
    }
    if ((base->flags ^ add->flags) & F_USER_UB) {
        if (base->flags & F_USER_UB)
            ub = base->ub;
        base->flags |= F_USER_UB;
    } else {
        ub = std::max(base->ub, ub);
    }
    base->lb = lb;
    base->ub = ub;
    base->align = std::max(base->align, add->align);
    if (!(base->flags & F_USER_UB)) {
        // C remainder, as the reference (a negative extent gives a negative remainder); a
        // power-of-two alignment (every predefined type's) takes it without a division
        const int64_t x = base->ub - base->lb, a = base->align;
        const int64_t eps = (a & (a - 1)) ? x % a
                                          : (x >= 0 ? (x & (a - 1)) : -int64_t(uint64_t(-x) & uint64_t(a - 1)));
        if (eps != 0)
            base->ub += base->align - eps;
    }
    base->flags |= F_DATA;
    if (add->size == 0)
        return st;
    base->size += int64_t(count) * add->size;
    base->bdt_used |= add->bdt_used;   // (:306)
    st.old_true_ub = (base->nbElems == 0) ? disp : base->true_ub;
    base->true_lb = std::min(true_lb, base->true_lb);
    base->true_ub = std::max(true_ub, base->true_ub);
    if (!is_predefined(add)) {
        base->flags |= (add->flags & F_USER_LB);
        base->flags |= (add->flags & F_USER_UB);
    }
    st.skip = false;
    return st;
}

void add_finish(ddt_datatype *base, const ddt_datatype *add, uint64_t count, int64_t disp,
                int64_t extent, const AddState &st)
{
    extent = effective_extent(add, extent);
    uint32_t local = base->flags & add->flags;
    base->flags &= ~(F_CONTIGUOUS | F_NO_GAPS);
    if ((local & F_CONTIGUOUS) && (disp + add->true_lb) == st.old_true_ub
        && (add->size == extent || count < 2)) {
        base->flags |= F_CONTIGUOUS;
        if (base->size == base->ub - base->lb)
            base->flags |= F_NO_GAPS;
    }
    base->nbElems += count * add->nbElems;
}

// opal_datatype_add: bounds + append of `count` replicas of `add` at disp + i*extent.
void type_add(ddt_datatype *base, const ddt_datatype *add, uint64_t count, int64_t disp,
              int64_t extent)
{
    extent = effective_extent(add, extent);
    AddState st = add_bounds(base, add, count, disp, extent);
    if (st.skip)
        return;
    if (is_predefined(add)) {   // predefined branch (:319-345)
        Node n;
        n.kind = Node::DATA;
        n.esize = add->size;
        n.tid = add->id;
        n.disp = disp;
        n.flags = add->flags & kElemFlags;
        if (extent == add->size) {
            n.count = 1;
            n.blen = count * uint64_t(add->size);
            n.extent = int64_t(n.blen);
        } else {
            n.count = count;
            n.blen = uint64_t(add->size);
            n.extent = extent;
            if (count > 1)
                n.flags &= ~(F_CONTIGUOUS | F_NO_GAPS);
        }
        base->desc.push_back(std::move(n));
    } else {
        std::vector<Node> sub = add->desc;
        shift_nodes(sub, disp);
        bool done = false;
        if (sub.size() == 1 && sub[0].kind == Node::DATA) {   // single DATA entry (:361-397)
            Node e = sub[0];
            if (count == 1) {
                base->desc.push_back(e);
                done = true;
            } else if (e.count == 1) {
                if (int64_t(e.blen) == extent) {
                    e.blen *= count;
                    e.extent = int64_t(e.blen);
                } else {
                    e.count = count;
                    e.extent = extent;
                }
                base->desc.push_back(e);
                done = true;
            } else if (extent == int64_t(e.count) * e.extent && e.count * count <= 0xffffffffull) {
                // the reference's element count is 32 bits; beyond it a loop is built (:379-390)
                e.count *= count;
                base->desc.push_back(e);
                done = true;
            }
        }
        if (!done) {   // build_loop (:400-431)
            if (count == 1) {
                for (Node &n : sub)
                    base->desc.push_back(std::move(n));
            } else {
                Node l;
                l.kind = Node::LOOP;
                l.count = count;
                l.extent = extent;
                l.flags = add->flags;
                l.body = std::move(sub);
                l.body_size = uint64_t(add->size);
                base->desc.push_back(std::move(l));
            }
        }
    }
    add_finish(base, add, count, disp, extent, st);
}

ddt_datatype *make_empty()
{
    // opal_datatype_empty (opal_datatype_constructors.h:67-75) via ompi_datatype_duplicate
    ddt_datatype *t = new_type();
    t->lb = t->ub = t->true_lb = t->true_ub = 0;
    t->align = 1;
    t->nbElems = 1;
    t->flags = F_CONTIGUOUS | F_NO_GAPS;
    return t;
}

ddt_datatype *clone_type(const ddt_datatype *o)
{
    // opal_datatype_clone (opal_datatype_clone.c:35-80): copy everything, drop PREDEFINED
    ddt_datatype *t = new_type();
    t->id = o->id;   // kept, as the reference does (:74): a dup of MPI_LB / MPI_UB stays a marker
    t->flags = o->flags & ~(F_PREDEFINED | F_COMMITTED);
    t->size = o->size;
    t->lb = o->lb;
    t->ub = o->ub;
    t->true_lb = o->true_lb;
    t->true_ub = o->true_ub;
    t->align = o->align;
    t->nbElems = o->nbElems;
    t->bdt_used = o->bdt_used;
    t->desc = o->desc;
    return t;
}

// Can `old` be replicated as a single contiguous block of its own size (LIST element)?
bool simple_block(const ddt_datatype *old)
{
    return old->size > 0 && old->desc.size() == 1 && old->desc[0].kind == Node::DATA
           && old->desc[0].count == 1 && int64_t(old->desc[0].blen) == old->size
           && old->extent() == old->size && old->desc[0].disp == 0 && !old->desc[0].pat;
}

uint64_t gcd64(uint64_t a, uint64_t b) { return b ? gcd64(b, a % b) : a; }

// gcd(g, x) for the running gcd of a list: once g is a power of two (it is from the first few
// blocks on for any list of aligned displacements) it is min(g, lowest set bit of x), with no
// division -- a 64 Mi-block list no longer spends seconds in 64-bit remainders
inline uint64_t gcd_acc(uint64_t g, uint64_t x)
{
    if (g && !(g & (g - 1)))
        return x ? std::min(g, x & (~x + 1)) : g;
    return gcd64(g, x);
}

std::shared_ptr<IndexList> finish_list(std::shared_ptr<IndexList> L)
{
    size_t n = L->disp.size();
    L->min_disp = INT64_MAX;
    L->max_end = INT64_MIN;
    uint64_t g = 0, gl = 0, acc = 0;
    if (!L->len.empty()) {
        L->poff.resize(n);
        for (size_t i = 0; i < n; ++i) {
            L->poff[i] = acc;
            acc += L->len[i];
            gl = gcd_acc(gl, L->len[i]);
            L->min_disp = std::min(L->min_disp, L->disp[i]);
            L->max_end = std::max(L->max_end, L->disp[i] + int64_t(L->len[i]));
            g = gcd_acc(g, uint64_t(L->disp[i] < 0 ? -L->disp[i] : L->disp[i]));
        }
        // all equal lengths -> uniform list
        if (n > 0 && gl == L->len[0]) {
            bool uni = true;
            for (size_t i = 1; i < n && uni; ++i)
                uni = L->len[i] == L->len[0];
            if (uni) {
                L->ulen = L->len[0];
                L->len.clear();
                L->poff.clear();
            }
        }
    } else {
        acc = L->ulen * n;
        gl = L->ulen;
        for (size_t i = 0; i < n; ++i) {
            L->min_disp = std::min(L->min_disp, L->disp[i]);
            L->max_end = std::max(L->max_end, L->disp[i] + int64_t(L->ulen));
            g = gcd_acc(g, uint64_t(L->disp[i] < 0 ? -L->disp[i] : L->disp[i]));
        }
    }
    L->total = acc;
    L->disp_gcd = g ? g : 0;
    L->len_gcd = gl;
    return L;
}

// Shared driver of the four indexed constructors (ompi_datatype_create_indexed.c:35-183):
// the caller merges blocks that abut in type-map order and feeds them here one at a time; the
// first kListMin are held back, and the type becomes either per-block adds or, for a longer run
// of a simple element type, one LIST node with the identical bounds.  Streaming, with the block
// lengths kept only once two differ: a 64 Mi-block list is built in one pass over its
// displacements, with no intermediate block array.
struct Block {
    int64_t disp_bytes;
    uint64_t nelem;
};

class IndexedBuilder {
public:
    IndexedBuilder(const ddt_datatype *old, size_t hint)
        : old_(old), t_(new_type()), extent_(old->extent()), hint_(hint), simple_(simple_block(old))
    {
        held_.reserve(kListMin + 1);
    }

    void add(int64_t disp_bytes, uint64_t nelem)
    {
        if (!L_) {
            held_.push_back({disp_bytes, nelem});
            if (held_.size() > kListMin && simple_) {   // a list: replay the held blocks into it
                L_ = std::make_shared<IndexList>();
                L_->esize = old_->desc[0].esize;
                L_->disp.reserve(hint_);
                for (const Block &b : held_)
                    to_list(b.disp_bytes, b.nelem);
                held_.clear();
            }
            return;
        }
        to_list(disp_bytes, nelem);
    }

    ddt_datatype *finish()
    {
        if (!L_) {
            for (const Block &b : held_)
                type_add(t_, old_, b.nelem, b.disp_bytes, extent_);
            return t_;
        }
        if (L_->len.empty())
            L_->ulen = ulen_;   // every block the same length (finish_list: no poff)
        else
            L_->len.shrink_to_fit();
        Node n;
        n.kind = Node::LIST;
        n.esize = L_->esize;
        n.tid = old_->desc[0].tid;
        // the flags of each block's DATA entry: the predefined type's own, or the copied
        // entry of a one-entry derived type (opal_datatype_add.c:328-329, :359)
        n.flags = is_predefined(old_) ? (old_->flags & kElemFlags) : old_->desc[0].flags;
        n.list = finish_list(L_);
        t_->desc.push_back(std::move(n));
        return t_;
    }

private:
    void to_list(int64_t disp_bytes, uint64_t nelem)
    {
        AddState st = add_bounds(t_, old_, nelem, disp_bytes, extent_);
        if (st.skip)
            return;
        const uint64_t bytes = nelem * uint64_t(old_->size);
        if (L_->disp.empty())
            ulen_ = bytes;
        else if (L_->len.empty() && bytes != ulen_) {   // the first differing length
            L_->len.reserve(hint_);
            L_->len.assign(L_->disp.size(), ulen_);
        }
        L_->disp.push_back(disp_bytes);
        if (!L_->len.empty())
            L_->len.push_back(bytes);
        add_finish(t_, old_, nelem, disp_bytes, extent_, st);
    }

    const ddt_datatype *old_;
    ddt_datatype *t_;
    int64_t extent_;
    size_t hint_;
    bool simple_;
    std::vector<Block> held_;
    std::shared_ptr<IndexList> L_;
    uint64_t ulen_ = 0;
};

}  // namespace

namespace ddt {

uint64_t Node::packed_bytes() const
{
    switch (kind) {
    case DATA: return count * blen;
    case LOOP: return count * body_size;
    case LIST: return list ? list->total : 0;
    }
    return 0;
}

ddt_datatype *new_type() { return new ddt_datatype(); }

// ---------------------------------------------------------------- commit normalisation
namespace {

bool element_starts(const Node &n, std::vector<uint32_t> &out)
{
    // element start offsets of one block of DATA node n
    if (n.blen > 0xffffffffull)
        return false;
    if (n.pat) {
        uint64_t P = n.pat->period;
        for (uint64_t k = 0; k < n.blen; k += P)
            for (uint32_t s : n.pat->starts) {
                if (out.size() >= kPatternMax)
                    return false;
                out.push_back(uint32_t(k + s));
            }
    } else {
        for (uint64_t s = 0; s < n.blen; s += uint64_t(n.esize)) {
            if (out.size() >= kPatternMax)
                return false;
            out.push_back(uint32_t(s));
        }
    }
    return true;
}

// Try to merge DATA b (count 1) onto the end of DATA a (count 1): contiguous in memory and
// therefore in the packed stream.
bool try_merge(Node &a, const Node &b)
{
    if (a.kind != Node::DATA || b.kind != Node::DATA || a.count != 1 || b.count != 1)
        return false;
    if (a.disp + int64_t(a.blen) != b.disp)
        return false;
    const uint16_t tid = a.tid == b.tid ? a.tid : 0;
    if (!a.pat && !b.pat && a.esize == b.esize) {
        a.blen += b.blen;
        a.extent = int64_t(a.blen);
        a.tid = tid;
        return true;
    }
    std::vector<uint32_t> sa, sb;
    if (!element_starts(a, sa) || !element_starts(b, sb) || sa.size() + sb.size() > kPatternMax)
        return false;
    auto p = std::make_shared<Pattern>();
    p->period = a.blen + b.blen;
    p->starts = sa;
    for (uint32_t s : sb)
        p->starts.push_back(uint32_t(s + a.blen));
    a.blen += b.blen;
    a.extent = int64_t(a.blen);
    a.esize = std::min(a.esize, b.esize);
    a.tid = tid;
    a.pat = p;
    return true;
}

void push_merge(std::vector<Node> &out, Node &&n)
{
    if (n.kind == Node::DATA && n.count > 1 && n.extent == int64_t(n.blen)) {
        n.blen *= n.count;
        n.count = 1;
        n.extent = int64_t(n.blen);
    }
    if (n.kind == Node::DATA && n.count * n.blen == 0)
        return;
    if (!out.empty() && try_merge(out.back(), n))
        return;
    out.push_back(std::move(n));
}

}  // namespace

void normalize(std::vector<Node> &nodes)
{
    std::vector<Node> out;
    out.reserve(nodes.size());
    for (Node &n : nodes) {
        if (n.kind == Node::LOOP) {
            normalize(n.body);
            if (n.body.empty() || n.count == 0 || n.body_size == 0)
                continue;
            if (n.count == 1) {
                for (Node &c : n.body)
                    push_merge(out, std::move(c));
                continue;
            }
            if (n.body.size() == 1 && n.body[0].kind == Node::DATA) {
                Node e = n.body[0];
                if (e.count == 1) {
                    if (int64_t(e.blen) == n.extent) {
                        // contiguous iterations: one block; a pattern keeps its period
                        e.blen *= n.count;
                        e.extent = int64_t(e.blen);
                    } else {
                        e.count = n.count;
                        e.extent = n.extent;
                    }
                    push_merge(out, std::move(e));
                    continue;
                } else if (n.extent == int64_t(e.count) * e.extent) {
                    e.count *= n.count;
                    push_merge(out, std::move(e));
                    continue;
                }
            }
            out.push_back(std::move(n));
        } else if (n.kind == Node::DATA) {
            push_merge(out, std::move(n));
        } else {
            if (n.list && n.list->total > 0)
                out.push_back(std::move(n));
        }
    }
    nodes.swap(out);
}

bool opt_desc_of(const ddt_datatype *t, DescForm &out)
{
    DescForm in;
    if (!build_opal_desc(t->desc, t->size, in))
        return false;
    uint32_t flags = 0;
    optimize_desc(in, t->size, out, &flags);
    return true;
}

// opal_datatype_commit (opal_datatype_optimize.c:1739-1782): the type map's Open MPI description
// goes through the restated optimizer (ddt_optimize.cpp) and comes back as the committed tree, so
// fragments and send positions stop on the reference's opt_desc elements.  An imported
// description already is an opt_desc; a type map whose description the 32-byte form cannot hold
// (a count beyond 32 bits) keeps its own elements.
// opal_datatype_opt_loop_nesting_depth (opal_datatype_optimize.c:222-241): the deepest LOOP
// nesting of a description; sibling loops do not add depth
uint32_t loop_depth(const DescForm &d)
{
    uint32_t depth = 0, mx = 0;
    for (size_t i = 0; i < d.used; ++i) {
        if (d.e[i].type == kDescLoop)
            mx = std::max(mx, ++depth);
        else if (d.e[i].type == kDescEndLoop && depth > 0)
            --depth;
    }
    return mx;
}

// the same on the tree (an imported opt_desc, or a type map the 32-byte form cannot hold)
uint32_t loop_depth(const std::vector<Node> &nodes)
{
    uint32_t mx = 0;
    for (const Node &n : nodes)
        if (n.kind == Node::LOOP)
            mx = std::max(mx, 1 + loop_depth(n.body));
    return mx;
}

int commit(ddt_datatype *t)
{
    if (t->flags & F_COMMITTED)
        return DDT_SUCCESS;
    bool optimized = false;
    t->stack_depth = loop_depth(t->desc);
    if (!t->imported) {
        DescForm in, out;
        std::vector<Node> nodes;
        if (build_opal_desc(t->desc, t->size, in)) {
            uint32_t flags = 0;
            optimize_desc(in, t->size, out, &flags);
            // opal_datatype_opt_update_stack_depth (:248-261): max over desc and opt_desc
            t->stack_depth = std::max(loop_depth(in), loop_depth(out));
            if (nodes_from_desc(out, nodes)) {
                t->opt = std::move(nodes);
                t->opt_flags = flags;
                optimized = true;
                // the committed opt_desc itself, as the reference keeps it: the
                // export and MPI_Pack's consolidation read THIS description, not one rebuilt
                // later under tuning values that may have changed since the commit
                t->opt_form = std::make_shared<const DescForm>(std::move(out));
            }
        }
    }
    if (!optimized)
        t->opt = t->desc;
    normalize(t->opt);
    t->opt_prefix.assign(1, 0);
    for (const Node &n : t->opt)
        t->opt_prefix.push_back(t->opt_prefix.back() + n.packed_bytes());
    t->flags |= F_COMMITTED;
    return DDT_SUCCESS;
}

namespace {
uint64_t snap_in_node(const Node &n, uint64_t off)
{
    switch (n.kind) {
    case Node::DATA: {
        uint64_t blk = off / n.blen, r = off % n.blen;
        uint64_t s;
        if (n.pat) {
            uint64_t P = n.pat->period, k = r / P, rr = r % P;
            auto it = std::upper_bound(n.pat->starts.begin(), n.pat->starts.end(), uint32_t(rr));
            s = k * P + *(it - 1);
        } else {
            s = (r / uint64_t(n.esize)) * uint64_t(n.esize);
        }
        return blk * n.blen + s;
    }
    case Node::LOOP: {
        uint64_t it = off / n.body_size, r = off % n.body_size, acc = 0;
        for (const Node &c : n.body) {
            uint64_t b = c.packed_bytes();
            if (r < acc + b)
                return it * n.body_size + acc + snap_in_node(c, r - acc);
            acc += b;
        }
        return it * n.body_size + acc;
    }
    case Node::LIST: {
        const IndexList &L = *n.list;
        uint64_t e = uint64_t(L.esize);
        if (L.len.empty()) {
            uint64_t blk = off / L.ulen, r = off % L.ulen;
            return blk * L.ulen + (r / e) * e;
        }
        auto it = std::upper_bound(L.poff.begin(), L.poff.end(), off);
        uint64_t start = *(it - 1);
        return start + ((off - start) / e) * e;
    }
    }
    return off;
}
}  // namespace

uint64_t snap_down_to_element(const ddt_datatype *t, uint64_t p)
{
    if (t->size <= 0)
        return p;
    uint64_t size = uint64_t(t->size), inst = p / size, q = p % size;
    if (q == 0)
        return p;
    auto it = std::upper_bound(t->opt_prefix.begin(), t->opt_prefix.end(), q);
    size_t idx = size_t(it - t->opt_prefix.begin()) - 1;
    if (idx >= t->opt.size())
        return p;
    return inst * size + t->opt_prefix[idx] + snap_in_node(t->opt[idx], q - t->opt_prefix[idx]);
}

}  // namespace ddt

uint64_t ddt_next_serial()
{
    static std::atomic<uint64_t> next{1};
    return next.fetch_add(1, std::memory_order_relaxed);
}

// ================================================================ C ABI: construction
namespace ddt {
namespace {
// GET_FIRST_NON_LOOP's displacement (opal_datatype_internal.h:282-294)
int64_t first_elem_disp(const DescForm &d)
{
    for (size_t i = 0; i < d.used; ++i) {
        const DescEntry &e = d.e[i];
        if (e.flags & F_DATA)
            return e.sealed >= 0 ? e.disp + d.lists[size_t(e.sealed)]->disp[e.sb] : e.disp;
    }
    return 0;
}
}  // namespace

void consolidate_into(ddt_datatype *t, const ddt_datatype *old, const DescForm &body, uint64_t count,
                      uint32_t mask);

// ompi_datatype_consolidate_create (ompi_datatype_create_contiguous.c:119-180) and
// opal_datatype_optimize_from_contiguous (opal_datatype_optimize.c:1480-1573)
ddt_datatype *consolidate(const ddt_datatype *old, uint64_t count, int64_t threshold)
{
    if (count == 0 || int64_t(count) < threshold || count > uint64_t(INT64_MAX))
        return nullptr;
    if ((old->flags & F_NO_GAPS) || old->size == 0)
        return nullptr;   // already contiguous across counts / nothing to move
    if ((old->flags & F_CONTIGUOUS) && old->size == old->extent())
        return nullptr;
    // the old type's committed opt_desc (cached at its commit; its desc when imported: that
    // already is one)
    DescForm body;
    if (old->opt_form)
        body = *old->opt_form;
    else if (old->imported ? !build_opal_desc(old->desc, old->size, body) : !opt_desc_of(old, body))
        return nullptr;
    // ompi_datatype_consolidate_optimization_mask (:72-100)
    uint32_t mask = kOptimizeAll;
    if (body.used && desc_has_small_blocks(body, false)) {
        mask &= ~kOptimizeBoundary;
        if (desc_has_small_blocks(body, true))
            mask &= ~kOptimizeFusion;
    }
    // the wrapping loop's count is 32 bits (:1504-1507); an empty body leaves the type as is
    if (count < 2 || count > 0xffffffffull || body.used == 0)
        return nullptr;
    ddt_datatype_t *t = nullptr;
    if (ddt_type_create_contiguous(size_t(count), old, &t) != DDT_SUCCESS || !t)
        return nullptr;
    try {
        consolidate_into(t, old, body, count, mask);
    } catch (...) {
        (void) ddt_type_destroy(&t);   // the new type is the caller's only once complete
        throw;
    }
    return t;
}

void consolidate_into(ddt_datatype *t, const ddt_datatype *old, const DescForm &body, uint64_t count,
                      uint32_t mask)
{
    const uint32_t loop_flags = (old->flags & 0x01FFu) & ~F_COMMITTED;
    DescForm in;
    in.lists = body.lists;
    in.e.reserve(body.used + 3);
    in.e.push_back(loop_desc_entry(uint32_t(count), uint32_t(body.used + 1), old->extent(), loop_flags));
    in.e.insert(in.e.end(), body.e.begin(), body.e.begin() + long(body.used));
    in.used = in.e.size();   // before the END_LOOP below: first_elem_disp skips the LOOP
    const int64_t first = first_elem_disp(in);
    in.e.push_back(end_desc_entry(uint32_t(body.used + 1), first, uint64_t(old->size), loop_flags));
    in.used = in.e.size();
    DescEntry fake = end_desc_entry(uint32_t(in.used), first, uint64_t(t->size), 0);
    fake.flags = 0;
    in.e.push_back(fake);   // opal_datatype_opt_set_fake_end_loop (:454-465)
    auto out = std::make_shared<DescForm>();
    uint32_t flags = 0;
    optimize_desc(in, t->size, *out, &flags, mask, true);
    t->opt_flags = flags | (old->opt_flags & kRestricted);
    std::vector<Node> nodes;
    if (nodes_from_desc(*out, nodes))
        t->opt = std::move(nodes);
    else
        t->opt = t->desc;
    normalize(t->opt);
    t->opt_prefix.assign(1, 0);
    for (const Node &n : t->opt)
        t->opt_prefix.push_back(t->opt_prefix.back() + n.packed_bytes());
    // opal_datatype_commit_description: committed, stack depth over desc and opt_desc
    t->stack_depth = std::max(loop_depth(t->desc), loop_depth(*out));
    t->flags |= F_COMMITTED;
    t->opt_form = std::move(out);
}
}  // namespace ddt

extern "C" {

const ddt_datatype_t *ddt_predefined(int id)
{
    std::call_once(g_predef_once, init_predefined);
    if (id < 2 || id > 27)
        return nullptr;
    return &g_predef[id];
}

int ddt_type_create_contiguous(size_t count, const ddt_datatype_t *old, ddt_datatype_t **out)
{
    if (!old || !out)
        return DDT_ERR_BAD_PARAM;
    if (count == 0 || old->size == 0) {
        *out = make_empty();
        return DDT_SUCCESS;
    }
    ddt_datatype *t = new_type();
    type_add(t, old, count, 0, old->extent());
    *out = t;
    return DDT_SUCCESS;
}

int ddt_type_create_vector(size_t count, size_t blen, ptrdiff_t stride, const ddt_datatype_t *old,
                           ddt_datatype_t **out)
{
    // ompi_datatype_create_vector (ompi_datatype_create_vector.c:32-58)
    if (!old || !out)
        return DDT_ERR_BAD_PARAM;
    int64_t extent = old->extent();
    if (count == 0 || blen == 0) {
        *out = make_empty();
        return DDT_SUCCESS;
    }
    ddt_datatype *t = new_type();
    if (int64_t(blen) == stride || count <= 1) {
        type_add(t, old, count * blen, 0, extent);
    } else if (blen == 1) {
        type_add(t, old, count, 0, extent * stride);
    } else {
        type_add(t, old, blen, 0, extent);
        ddt_datatype *t2 = new_type();
        type_add(t2, t, count, 0, extent * stride);
        delete t;
        t = t2;
    }
    *out = t;
    return DDT_SUCCESS;
}

int ddt_type_create_hvector(size_t count, size_t blen, ptrdiff_t stride, const ddt_datatype_t *old,
                            ddt_datatype_t **out)
{
    // ompi_datatype_create_hvector (ompi_datatype_create_vector.c:61-88)
    if (!old || !out)
        return DDT_ERR_BAD_PARAM;
    int64_t extent = old->extent();
    if (count == 0 || blen == 0) {
        *out = make_empty();
        return DDT_SUCCESS;
    }
    ddt_datatype *t = new_type();
    if (extent * int64_t(blen) == stride || count <= 1) {
        type_add(t, old, count * blen, 0, extent);
    } else if (blen == 1) {
        type_add(t, old, count, 0, stride);
    } else {
        type_add(t, old, blen, 0, extent);
        ddt_datatype *t2 = new_type();
        type_add(t2, t, count, 0, stride);
        delete t;
        t = t2;
    }
    *out = t;
    return DDT_SUCCESS;
}

static int indexed_common(size_t count, const size_t *blens, const ptrdiff_t *disps, size_t ublen,
                          bool uniform, bool bytes, const ddt_datatype_t *old, ddt_datatype_t **out)
{
    if (!old || !out || (count && !disps) || (!uniform && count && !blens))
        return DDT_ERR_BAD_PARAM;
    int64_t extent = old->extent();
    size_t i = 0;
    if (!uniform) {
        for (; i < count && blens[i] == 0; ++i)
            ;
        if (i == count || old->size == 0) {
            *out = make_empty();
            return DDT_SUCCESS;
        }
    } else if (count == 0 || ublen == 0) {
        *out = make_empty();
        return DDT_SUCCESS;
    }
    auto bl = [&](size_t k) { return uniform ? ublen : blens[k]; };
    IndexedBuilder build(old, count - i);
    int64_t disp = disps[i];
    uint64_t dlen = bl(i);
    int64_t endat = bytes ? disp + int64_t(dlen) * extent : disp + int64_t(dlen);
    for (i += 1; i < count; ++i) {
        if (bl(i) == 0)
            continue;
        if (endat == disps[i]) {
            dlen += bl(i);
            endat += bytes ? int64_t(bl(i)) * extent : int64_t(bl(i));
        } else {
            build.add(bytes ? disp : disp * extent, dlen);
            disp = disps[i];
            dlen = bl(i);
            endat = bytes ? disp + int64_t(dlen) * extent : disp + int64_t(dlen);
        }
    }
    build.add(bytes ? disp : disp * extent, dlen);
    *out = build.finish();
    return DDT_SUCCESS;
}

int ddt_type_create_indexed(size_t count, const size_t *blens, const ptrdiff_t *disps,
                            const ddt_datatype_t *old, ddt_datatype_t **out)
{
    return indexed_common(count, blens, disps, 0, false, false, old, out);
}

int ddt_type_create_hindexed(size_t count, const size_t *blens, const ptrdiff_t *disps,
                             const ddt_datatype_t *old, ddt_datatype_t **out)
{
    return indexed_common(count, blens, disps, 0, false, true, old, out);
}

int ddt_type_create_indexed_block(size_t count, size_t blen, const ptrdiff_t *disps,
                                  const ddt_datatype_t *old, ddt_datatype_t **out)
{
    return indexed_common(count, nullptr, disps, blen, true, false, old, out);
}

int ddt_type_create_hindexed_block(size_t count, size_t blen, const ptrdiff_t *disps,
                                   const ddt_datatype_t *old, ddt_datatype_t **out)
{
    return indexed_common(count, nullptr, disps, blen, true, true, old, out);
}

int ddt_type_create_struct(size_t count, const size_t *blens, const ptrdiff_t *disps,
                           const ddt_datatype_t *const *types, ddt_datatype_t **out)
{
    // ompi_datatype_create_struct (ompi_datatype_create_struct.c:32-98)
    if (!out || (count && (!blens || !disps || !types)))
        return DDT_ERR_BAD_PARAM;
    size_t i = 0;
    for (; i < count && blens[i] == 0; ++i)
        ;
    if (i == count) {
        *out = make_empty();
        return DDT_SUCCESS;
    }
    for (size_t k = i; k < count; ++k)
        if (!types[k])
            return DDT_ERR_BAD_PARAM;
    const ddt_datatype *lastType = types[i];
    uint64_t lastBlock = blens[i];
    int64_t lastExtent = lastType->extent();
    int64_t lastDisp = disps[i];
    int64_t endto = lastDisp + lastExtent * int64_t(lastBlock);
    ddt_datatype *t = new_type();
    for (i += 1; i < count; ++i) {
        if (types[i] == lastType && disps[i] == endto) {
            lastBlock += blens[i];
            endto = lastDisp + int64_t(lastBlock) * lastExtent;
        } else {
            type_add(t, lastType, lastBlock, lastDisp, lastExtent);
            lastType = types[i];
            lastExtent = lastType->extent();
            lastBlock = blens[i];
            lastDisp = disps[i];
            endto = lastDisp + lastExtent * int64_t(lastBlock);
        }
    }
    type_add(t, lastType, lastBlock, lastDisp, lastExtent);
    *out = t;
    return DDT_SUCCESS;
}

static void resize_in_place(ddt_datatype *t, int64_t lb, int64_t extent)
{
    // opal_datatype_resize (opal_datatype_resize.c:23-41)
    t->lb = lb;
    t->ub = lb + extent;
    t->flags &= ~F_NO_GAPS;
    t->flags |= F_USER_LB | F_USER_UB;
    if (extent == t->size && (t->flags & F_CONTIGUOUS))
        t->flags |= F_NO_GAPS;
}

int ddt_type_create_resized(const ddt_datatype_t *old, ptrdiff_t lb, ptrdiff_t extent,
                            ddt_datatype_t **out)
{
    if (!old || !out)
        return DDT_ERR_BAD_PARAM;
    ddt_datatype *t = clone_type(old);
    resize_in_place(t, lb, extent);
    *out = t;
    return DDT_SUCCESS;
}

int ddt_type_dup(const ddt_datatype_t *old, ddt_datatype_t **out)
{
    if (!old || !out)
        return DDT_ERR_BAD_PARAM;
    *out = clone_type(old);
    return DDT_SUCCESS;
}

// ---- darray (ompi_datatype_create_darray.c), the same constructor calls in the same order
namespace {

int64_t gsize_prod(const size_t *g, int from, int to)   // product of g[from..to]
{
    int64_t p = 1;
    for (int i = from; i <= to; ++i)
        p *= int64_t(g[i]);
    return p;
}

// block() (ompi_datatype_create_darray.c:34-98)
int darray_block(const size_t *gsizes, int dim, int ndims, int nprocs, int rank, int darg, int order,
                 int64_t orig_extent, const ddt_datatype *old, ddt_datatype **out, int64_t *st_offset)
{
    const int64_t global_size = int64_t(gsizes[dim]);
    const int64_t blksize = darg == DDT_DISTRIBUTE_DFLT_DARG
                                ? global_size / nprocs + (global_size % nprocs != 0)
                                : int64_t(darg);
    const int64_t j = global_size - blksize * rank;
    int64_t mysize = blksize < j ? blksize : j;
    if (mysize < 0)
        mysize = 0;
    const int start_loop = order == DDT_ORDER_C ? ndims - 1 : 0;
    const int step = order == DDT_ORDER_C ? -1 : 1;
    int rc;
    if (dim == start_loop) {
        rc = ddt_type_create_contiguous(size_t(mysize), old, out);
    } else {
        int64_t stride = orig_extent;
        for (int i = start_loop; i != dim; i += step)
            stride *= int64_t(gsizes[i]);
        rc = ddt_type_create_hvector(size_t(mysize), 1, stride, old, out);
    }
    if (rc != DDT_SUCCESS)
        return rc;
    *st_offset = mysize == 0 ? 0 : blksize * rank;
    const int64_t ub = orig_extent * (order == DDT_ORDER_FORTRAN ? gsize_prod(gsizes, 0, dim)
                                                                 : gsize_prod(gsizes, dim, ndims - 1));
    resize_in_place(*out, 0, ub);
    return DDT_SUCCESS;
}

// cyclic() (ompi_datatype_create_darray.c:101-184)
int darray_cyclic(const size_t *gsizes, int dim, int ndims, int nprocs, int rank, int darg, int order,
                  int64_t orig_extent, const ddt_datatype *old, ddt_datatype **out, int64_t *st_offset)
{
    const int64_t blksize = darg == DDT_DISTRIBUTE_DFLT_DARG ? 1 : int64_t(darg);
    const int64_t st_index = int64_t(rank) * blksize;
    const int64_t end_index = int64_t(gsizes[dim]) - 1;
    int64_t local_size = 0;
    if (end_index >= st_index) {
        local_size = ((end_index - st_index + 1) / (int64_t(nprocs) * blksize)) * blksize;
        const int64_t rem = (end_index - st_index + 1) % (int64_t(nprocs) * blksize);
        local_size += rem < blksize ? rem : blksize;
    }
    const int64_t count = local_size / blksize, rem = local_size % blksize;
    int64_t stride = int64_t(nprocs) * blksize * orig_extent;
    if (order == DDT_ORDER_FORTRAN)
        stride *= gsize_prod(gsizes, 0, dim - 1);
    else
        stride *= gsize_prod(gsizes, dim + 1, ndims - 1);
    int rc = ddt_type_create_hvector(size_t(count), size_t(blksize), stride, old, out);
    if (rc != DDT_SUCCESS)
        return rc;
    if (rem) {
        // trailing partial block through a struct (:150-165)
        const ddt_datatype *types[2] = {*out, old};
        const ptrdiff_t disps[2] = {0, ptrdiff_t(count * stride)};
        const size_t blens[2] = {1, size_t(rem)};
        ddt_datatype *tmp = nullptr;
        rc = ddt_type_create_struct(2, blens, disps, types, &tmp);
        delete *out;
        *out = tmp;
        if (rc != DDT_SUCCESS)
            return rc;
    }
    const int64_t ub = orig_extent * (order == DDT_ORDER_FORTRAN ? gsize_prod(gsizes, 0, dim)
                                                                 : gsize_prod(gsizes, dim, ndims - 1));
    resize_in_place(*out, 0, ub);
    *st_offset = local_size == 0 ? 0 : int64_t(rank) * blksize;
    return DDT_SUCCESS;
}

}  // namespace

int ddt_type_create_darray(int size, int rank, int ndims, const size_t *gsizes, const int *distribs,
                           const int *dargs, const int *psizes, int order, const ddt_datatype_t *old,
                           ddt_datatype_t **out)
{
    // ompi_datatype_create_darray (ompi_datatype_create_darray.c:187-312)
    if (!old || !out || (ndims > 0 && (!gsizes || !distribs || !dargs || !psizes)) || size < 1
        || rank < 0 || rank >= size)
        return DDT_ERR_BAD_PARAM;
    if (ndims < 1) {
        *out = make_empty();
        return DDT_SUCCESS;
    }
    for (int i = 0; i < ndims; ++i)
        if (psizes[i] < 1)
            return DDT_ERR_BAD_PARAM;
    const int64_t orig_extent = old->extent();
    std::vector<int> coords(static_cast<size_t>(ndims), 0);
    int64_t ub = orig_extent;
    {
        int tmp_rank = rank, procs = size;
        for (int i = 0; i < ndims; ++i) {
            procs /= psizes[i];
            if (procs < 1)
                return DDT_ERR_BAD_PARAM;
            coords[size_t(i)] = tmp_rank / procs;
            tmp_rank %= procs;
            ub *= int64_t(gsizes[i]);
        }
    }
    std::vector<int64_t> st(static_cast<size_t>(ndims), 0);
    ddt_datatype *last = clone_type(old);
    const int start_loop = order == DDT_ORDER_C ? ndims - 1 : 0;
    const int step = order == DDT_ORDER_C ? -1 : 1;
    const int end_loop = order == DDT_ORDER_C ? -1 : ndims;
    for (int i = start_loop; i != end_loop; i += step) {
        ddt_datatype *nt = nullptr;
        int rc;
        switch (distribs[i]) {
        case DDT_DISTRIBUTE_BLOCK:
            rc = darray_block(gsizes, i, ndims, psizes[i], coords[size_t(i)], dargs[i], order,
                              orig_extent, last, &nt, &st[size_t(i)]);
            break;
        case DDT_DISTRIBUTE_CYCLIC:
            rc = darray_cyclic(gsizes, i, ndims, psizes[i], coords[size_t(i)], dargs[i], order,
                               orig_extent, last, &nt, &st[size_t(i)]);
            break;
        case DDT_DISTRIBUTE_NONE:
            // a block distribution on one process (:264-274)
            rc = darray_block(gsizes, i, ndims, order == DDT_ORDER_C ? psizes[i] : 1,
                              order == DDT_ORDER_C ? coords[size_t(i)] : 0, DDT_DISTRIBUTE_DFLT_DARG,
                              order, orig_extent, last, &nt, &st[size_t(i)]);
            break;
        default:
            rc = DDT_ERR_BAD_PARAM;
        }
        delete last;
        if (rc != DDT_SUCCESS) {
            delete nt;
            return rc;
        }
        last = nt;
    }
    // move the data to its displacement: a fresh type + one add (:288-306)
    int64_t disp = st[size_t(start_loop)], tmp_size = 1;
    for (int i = start_loop + step; i != end_loop; i += step) {
        tmp_size *= int64_t(gsizes[i - step]);
        disp += tmp_size * st[size_t(i)];
    }
    disp *= orig_extent;
    ddt_datatype *nt = new_type();
    type_add(nt, last, 1, disp, ub);
    delete last;
    resize_in_place(nt, 0, ub);
    *out = nt;
    return DDT_SUCCESS;
}

int ddt_type_create_subarray(int ndims, const size_t *sizes, const size_t *subsizes,
                             const size_t *starts, int order, const ddt_datatype_t *old,
                             ddt_datatype_t **out)
{
    // ompi_datatype_create_subarray (ompi_datatype_create_subarray.c:32-112)
    if (!old || !out || ndims < 0 || (ndims > 0 && (!sizes || !subsizes || !starts)))
        return DDT_ERR_BAD_PARAM;
    int64_t extent = old->extent(), size, displ;
    ddt_datatype_t *last = nullptr, *nt = nullptr;
    if (ndims < 2) {
        if (ndims == 0) {
            *out = make_empty();
            return DDT_SUCCESS;
        }
        ddt_type_create_contiguous(subsizes[0], old, &last);
        size = int64_t(sizes[0]);
        displ = int64_t(starts[0]);
    } else {
        int i, step, end_loop;
        if (order == DDT_ORDER_C) {
            i = ndims - 1;
            step = -1;
            end_loop = -1;
        } else {
            i = 0;
            step = 1;
            end_loop = ndims;
        }
        ddt_type_create_vector(subsizes[i + step], subsizes[i], ptrdiff_t(sizes[i]), old, &last);
        size = int64_t(sizes[i]) * int64_t(sizes[i + step]);
        displ = int64_t(starts[i]) + int64_t(starts[i + step]) * int64_t(sizes[i]);
        for (i += 2 * step; i != end_loop; i += step) {
            ddt_type_create_hvector(subsizes[i], 1, size * extent, last, &nt);
            delete last;
            displ += size * int64_t(starts[i]);
            size *= int64_t(sizes[i]);
            last = nt;
        }
    }
    nt = new_type();
    type_add(nt, last, 1, displ * extent, size * extent);
    delete last;
    resize_in_place(nt, 0, size * extent);
    *out = nt;
    return DDT_SUCCESS;
}

int ddt_type_commit(ddt_datatype_t *t)
{
    if (!t)
        return DDT_ERR_BAD_PARAM;
    const int rc = commit(t);
    if (rc == DDT_SUCCESS)
        (void) prebuild_device(t);   // a large index list: its address-ordered tables now, not
                                     // inside the first pack (a failure leaves that to first use)
    return rc;
}

int ddt_type_prepare_device(ddt_datatype_t *t)
{
    if (!t)
        return DDT_ERR_BAD_PARAM;
    if (!(t->flags & F_COMMITTED))
        return DDT_ERR_NOT_COMMITTED;
    return prebuild_device(t);
}

int ddt_type_destroy(ddt_datatype_t **t)
{
    if (!t || !*t)
        return DDT_ERR_BAD_PARAM;
    if (is_predefined(*t)) {
        *t = nullptr;
        return DDT_SUCCESS;
    }
    delete *t;
    *t = nullptr;
    return DDT_SUCCESS;
}

int ddt_type_size(const ddt_datatype_t *t, size_t *size)
{
    if (!t || !size)
        return DDT_ERR_BAD_PARAM;
    *size = size_t(t->size);
    return DDT_SUCCESS;
}

int ddt_type_get_extent(const ddt_datatype_t *t, ptrdiff_t *lb, ptrdiff_t *extent)
{
    if (!t)
        return DDT_ERR_BAD_PARAM;
    if (lb)
        *lb = t->lb;
    if (extent)
        *extent = t->ub - t->lb;
    return DDT_SUCCESS;
}

int ddt_type_get_true_extent(const ddt_datatype_t *t, ptrdiff_t *true_lb, ptrdiff_t *true_extent)
{
    if (!t)
        return DDT_ERR_BAD_PARAM;
    if (true_lb)
        *true_lb = t->true_lb;
    if (true_extent)
        *true_extent = t->true_ub - t->true_lb;
    return DDT_SUCCESS;
}

uint32_t ddt_type_flags(const ddt_datatype_t *t) { return t ? t->flags : 0; }

namespace {
// Basic elements of one instance of a node list (the uncommitted description: every element
// keeps its own type size, like opal_datatype_compute_ptypes over desc).
uint64_t elements_of(const std::vector<Node> &nodes)
{
    uint64_t e = 0;
    for (const Node &n : nodes) {
        if (n.kind == Node::DATA)
            e += n.count * (n.blen / uint64_t(n.esize));
        else if (n.kind == Node::LOOP)
            e += n.count * elements_of(n.body);
        else if (n.list)
            e += n.list->total / uint64_t(n.esize);
    }
    return e;
}

// opal_datatype_get_element_count (opal_datatype_get_count.c:32-92): elements within the first
// `left` packed bytes of one instance, walking the type map in order; -1 when the budget ends
// inside an element.  *done is set once the budget is used up.
int64_t count_within(const std::vector<Node> &nodes, uint64_t &left, bool &done)
{
    int64_t acc = 0;
    for (const Node &n : nodes) {
        if (n.kind == Node::LOOP) {
            if (n.body_size == 0)
                continue;
            const uint64_t total = n.count * n.body_size;
            const uint64_t be = elements_of(n.body);
            if (total < left) {   // whole loop
                acc += int64_t(n.count * be);
                left -= total;
                continue;
            }
            const uint64_t full = left == 0 ? 0 : (left - 1) / n.body_size;   // iterations before the last
            acc += int64_t(full * be);
            left -= full * n.body_size;
            const int64_t r = count_within(n.body, left, done);
            return r < 0 ? -1 : acc + r;
        }
        const uint64_t bytes = n.packed_bytes();
        const uint64_t es = uint64_t(n.esize);
        if (bytes >= left) {   // the budget ends in this entry (opal_datatype_get_count.c:81-86)
            done = true;
            const uint64_t k = left / es;
            const bool whole = left == k * es;
            left = 0;
            return whole ? acc + int64_t(k) : -1;
        }
        acc += int64_t(bytes / es);
        left -= bytes;
    }
    return acc;
}
}  // namespace

int ddt_get_elements(const ddt_datatype_t *t, size_t ucount, size_t *count)
{
    // ompi_datatype_get_elements (ompi/datatype/ompi_datatype_get_elements.c:30-76)
    if (!t || !count)
        return DDT_ERR_BAD_PARAM;
    *count = 0;
    const uint64_t size = uint64_t(t->size);
    if (size == 0)
        return DDT_SUCCESS;
    uint64_t full = ucount / size, left = ucount - full * size;
    if (is_predefined(t)) {
        if (left)
            return DDT_ERR_VALUE_OUT_OF_BOUNDS;
        *count = size_t(full);
        return DDT_SUCCESS;
    }
    uint64_t n = full ? full * elements_of(t->desc) : 0;
    if (left) {
        bool done = false;
        const int64_t r = count_within(t->desc, left, done);
        if (r < 0)
            return DDT_ERR_VALUE_OUT_OF_BOUNDS;
        n += uint64_t(r);
    }
    *count = size_t(n);
    return DDT_SUCCESS;
}

int ddt_type_consolidate(const ddt_datatype_t *old, size_t count, ddt_datatype_t **out)
{
    if (!old || !out)
        return DDT_ERR_BAD_PARAM;
    *out = nullptr;
    if (!(old->flags & F_COMMITTED))
        return DDT_ERR_NOT_COMMITTED;
    try {
        *out = consolidate(old, count, tuning().consolidate);
    } catch (const std::bad_alloc &) {
        return DDT_ERR_OUT_OF_RESOURCE;
    }
    return DDT_SUCCESS;
}

int ddt_type_commit_info(const ddt_datatype_t *t, int64_t *o)
{
    if (!t || !o)
        return DDT_ERR_BAD_PARAM;
    o[0] = int64_t(t->stack_depth);
    o[1] = int64_t(t->bdt_used);
    o[2] = int64_t(t->opt_flags);
    o[3] = (t->flags & F_COMMITTED) ? 1 : 0;
    return DDT_SUCCESS;
}

int ddt_type_info(const ddt_datatype_t *t, int64_t *o)
{
    if (!t || !o)
        return DDT_ERR_BAD_PARAM;
    o[0] = t->size;
    o[1] = t->lb;
    o[2] = t->ub;
    o[3] = t->true_lb;
    o[4] = t->true_ub;
    o[5] = t->align;
    o[6] = int64_t(t->flags);
    o[7] = int64_t(t->nbElems);
    return DDT_SUCCESS;
}

// ---- opal description import (opal_datatype_internal.h:119-160 layout, 32-byte entries)
namespace {
struct RawEntry {
    uint16_t flags, type;
    uint32_t a;   // DATA: count; LOOP/END_LOOP: items
    uint32_t b;   // LOOP: loops
    uint32_t pad;
    uint64_t c;   // DATA: blocklen; END_LOOP: size
    int64_t d;    // DATA: extent; LOOP: extent
    int64_t e;    // DATA: disp; END_LOOP: first_elem_disp
};

// Runs of at least kFoldMin consecutive DATA entries of one basic type, each of at most
// kFoldCount blocks, are imported as ONE index list instead of one node per entry: the
// optimizer leaves an indexed type as one- or two-block DATA entries (the 64 Mi blocks of
// BASELINE config 4 are 32 M entries, opal_datatype_optimize.c:1179-1185), which would
// otherwise become 32 M plan leaves.  Type-map order and bytes are unchanged.
constexpr size_t kFoldMin = 64;
constexpr uint32_t kFoldCount = 16;

struct RawData {
    uint16_t type;
    uint32_t count;
    uint64_t blen;   // bytes
    int64_t extent, disp;
};

// A run of foldable DATA entries of one type, streamed: the first kFoldMin entries wait in
// `head`; from then on blocks go straight into the index list, whose per-block lengths are
// materialised only once two of them differ (cfg4's 33.5 M entries import without a second
// copy of the description or a length array).
struct Fold {
    uint16_t type = 0;
    std::vector<RawData> head;
    std::shared_ptr<IndexList> L;
    bool uni = true;
    uint64_t ulen = 0;

    bool empty() const { return head.empty() && !L; }
    void add_blocks(const RawData &r)
    {
        for (uint32_t k = 0; k < r.count; ++k) {
            L->disp.push_back(r.disp + int64_t(k) * r.extent);
            if (uni && r.blen != ulen) {
                uni = false;
                L->len.assign(L->disp.size() - 1, ulen);
            }
            if (!uni)
                L->len.push_back(r.blen);
        }
    }
    // `left`: entries of this level from r on, so the list can reserve for a run that
    // continues to the level's end (no regrowth copies of a 256 MiB displacement array)
    void push(const RawData &r, size_t left)
    {
        if (empty())
            type = r.type;
        if (L) {
            add_blocks(r);
            return;
        }
        head.push_back(r);
        if (head.size() < kFoldMin)
            return;
        L = std::make_shared<IndexList>();
        L->esize = kSize[type];
        L->disp.reserve(std::min<size_t>(head.size() * kFoldCount + left * size_t(r.count), size_t(1) << 27));
        uni = true;
        ulen = head[0].blen;
        for (const RawData &h : head)
            add_blocks(h);
        head.clear();
    }
    void flush(std::vector<Node> &out)
    {
        if (L) {
            // the reservation assumed the run continues to the level's end; a run that ended
            // early hands the unused part back (other entries after a short run)
            if (L->disp.capacity() > L->disp.size() + L->disp.size() / 4)
                L->disp.shrink_to_fit();
            if (uni) {
                L->ulen = ulen;
                L->len.clear();
            }
            Node n;
            n.kind = Node::LIST;
            n.esize = L->esize;
            n.tid = type;
            n.list = finish_list(L);
            out.push_back(std::move(n));
            L.reset();
        }
        for (const RawData &r : head)
            out.push_back(data_node(r));
        head.clear();
    }
    static Node data_node(const RawData &r)
    {
        Node n;
        n.kind = Node::DATA;
        n.esize = kSize[r.type];
        n.tid = r.type;
        n.count = r.count;
        n.blen = r.blen;
        n.extent = r.extent;
        n.disp = r.disp;
        return n;
    }
};

// `sealed`: the engine's own long index lists, passed through the optimizer whole
// (ddt_optimize.h); a DATA entry of type 0 names one: count = its index, blocklen = the element
// type, disp = the shift of every block.
using SealedLists = std::vector<std::shared_ptr<const IndexList>>;

bool parse_opal(const unsigned char *raw, size_t begin, size_t end, std::vector<Node> &out,
                const SealedLists *sealed = nullptr)
{
    size_t i = begin;
    Fold run;
    while (i < end) {
        const unsigned char *p = raw + 32 * i;
        uint16_t flags, type;
        std::memcpy(&flags, p, 2);
        std::memcpy(&type, p + 2, 2);
        if ((flags & F_DATA) && type == 0 && sealed) {
            uint32_t idx;
            uint64_t tid;
            int64_t shift;
            std::memcpy(&idx, p + 4, 4);
            std::memcpy(&tid, p + 8, 8);
            std::memcpy(&shift, p + 24, 8);
            if (idx >= sealed->size() || tid < 4 || tid > 27)
                return false;
            run.flush(out);
            Node n;
            n.kind = Node::LIST;
            n.tid = uint16_t(tid);
            n.esize = kSize[tid];
            n.list = (*sealed)[idx];
            n.disp = shift;
            out.push_back(std::move(n));
            ++i;
            continue;
        }
        if (flags & F_DATA) {
            uint32_t count;
            uint64_t blocklen;
            int64_t extent, disp;
            std::memcpy(&count, p + 4, 4);
            std::memcpy(&blocklen, p + 8, 8);
            std::memcpy(&extent, p + 16, 8);
            std::memcpy(&disp, p + 24, 8);
            if (type < 4 || type > 27)
                return false;
            const RawData d{type, count, blocklen * uint64_t(kSize[type]), extent, disp};
            const bool foldable = count >= 1 && count <= kFoldCount && d.blen > 0;
            if (!run.empty() && (!foldable || run.type != type))
                run.flush(out);
            if (foldable)
                run.push(d, end - i);
            else
                out.push_back(Fold::data_node(d));
            ++i;
        } else if (type == 0) {   // LOOP
            run.flush(out);
            uint32_t items, loops;
            int64_t extent;
            std::memcpy(&items, p + 4, 4);
            std::memcpy(&loops, p + 8, 4);
            std::memcpy(&extent, p + 24, 8);
            // the matching END_LOOP sits `items` entries on and carries the same item count
            // (CREATE_LOOP_START / CREATE_LOOP_END, opal_datatype_internal.h:171-189); it must
            // lie inside this level, and its size must be the body's packed bytes
            const size_t endi = i + items;
            if (items < 1 || endi >= end)
                return false;
            const unsigned char *q = raw + 32 * endi;
            uint16_t eflags, etype;
            uint32_t eitems;
            uint64_t size;
            std::memcpy(&eflags, q, 2);
            std::memcpy(&etype, q + 2, 2);
            std::memcpy(&eitems, q + 4, 4);
            std::memcpy(&size, q + 16, 8);
            if ((eflags & F_DATA) || etype != 1 || eitems != items)
                return false;
            Node l;
            l.kind = Node::LOOP;
            l.count = loops;
            l.extent = extent;
            l.body_size = size;
            if (!parse_opal(raw, i + 1, endi, l.body, sealed))
                return false;
            uint64_t body = 0;
            for (const Node &n : l.body)
                body += n.packed_bytes();
            if (body != size)
                return false;
            out.push_back(std::move(l));
            i = endi + 1;
        } else {
            return false;   // stray END_LOOP
        }
    }
    run.flush(out);   // a run that ends the description
    return true;
}
}  // namespace


namespace {
// One entry per DATA block run / LOOP marker of the uncommitted type map, in the
// dt_elem_desc_t layout (opal_datatype_internal.h:119-169) the import reads.
void put_entry(std::vector<unsigned char> &out, uint16_t flags, uint16_t type, uint32_t a, uint32_t b,
               uint64_t c, int64_t d, int64_t e)
{
    unsigned char p[32] = {0};
    std::memcpy(p, &flags, 2);
    std::memcpy(p + 2, &type, 2);
    std::memcpy(p + 4, &a, 4);
    if (type == 0 || type == 1) {   // LOOP: items, loops, unused, extent; END_LOOP: items, unused, size, first disp
        std::memcpy(p + 8, &b, 4);
        std::memcpy(p + 16, &c, 8);
        std::memcpy(p + 24, type == 0 ? &d : &e, 8);
    } else {                        // DATA: count, blocklen, extent, disp
        std::memcpy(p + 8, &c, 8);
        std::memcpy(p + 16, &d, 8);
        std::memcpy(p + 24, &e, 8);
    }
    out.insert(out.end(), p, p + 32);
}

bool export_nodes(const std::vector<Node> &nodes, std::vector<unsigned char> &out)
{
    for (const Node &n : nodes) {
        switch (n.kind) {
        case Node::DATA: {
            const uint16_t type = n.tid ? n.tid : 9;   // a mixed run travels as UINT1 bytes
            const uint64_t es = n.tid ? uint64_t(kSize[n.tid]) : 1;
            if (n.count > 0xffffffffull || n.blen % es)
                return false;
            put_entry(out, uint16_t(F_DATA), type, uint32_t(n.count), 0, n.blen / es, n.extent, n.disp);
            break;
        }
        case Node::LIST: {
            const IndexList &X = *n.list;
            const uint16_t type = n.tid ? n.tid : 9;
            const uint64_t es = n.tid ? uint64_t(kSize[n.tid]) : 1;
            for (size_t k = 0; k < X.nblk(); ++k) {
                const uint64_t len = X.len.empty() ? X.ulen : X.len[k];
                if (len % es)
                    return false;
                put_entry(out, uint16_t(F_DATA), type, 1, 0, len / es, int64_t(len), n.disp + X.disp[k]);
            }
            break;
        }
        case Node::LOOP: {
            const size_t at = out.size();
            put_entry(out, 0, 0, 0, uint32_t(n.count), ~uint64_t(0), n.extent, 0);
            if (n.count > 0xffffffffull || !export_nodes(n.body, out))
                return false;
            const uint32_t items = uint32_t((out.size() - at) / 32);   // LOOP + body entries
            std::memcpy(&out[at + 4], &items, 4);
            put_entry(out, 0, 1, items, 0xffffffffu, n.body_size, 0, 0);
            break;
        }
        }
    }
    return true;
}
}  // namespace

int64_t ddt_type_to_opal_desc(const ddt_datatype_t *t, void *out, size_t cap)
{
    if (!t)
        return DDT_ERR_BAD_PARAM;
    std::vector<unsigned char> buf;
    DescForm d;
    if (t->imported) {
        if (!export_nodes(t->desc, buf))
            return DDT_ERR_NOT_SUPPORTED;
    } else {
        if (!build_opal_desc(t->desc, t->size, d))
            return DDT_ERR_NOT_SUPPORTED;
        encode_desc(d, buf);
    }
    const size_t used = buf.size() / 32;
    if (used > cap)
        return -int64_t(used);
    if (out && used)
        std::memcpy(out, buf.data(), buf.size());
    return int64_t(used);
}

int64_t ddt_type_to_opal_opt_desc(const ddt_datatype_t *t, void *out, size_t cap, uint32_t *flags)
{
    if (!t)
        return DDT_ERR_BAD_PARAM;
    std::vector<unsigned char> buf;
    uint32_t fl = t->opt_flags;
    if (t->opt_form) {
        encode_desc(*t->opt_form, buf, true);
    } else if (t->imported) {
        if (!export_nodes(t->desc, buf))
            return DDT_ERR_NOT_SUPPORTED;
    } else {
        DescForm in, o;
        if (!build_opal_desc(t->desc, t->size, in))
            return DDT_ERR_NOT_SUPPORTED;
        fl = 0;
        optimize_desc(in, t->size, o, &fl);
        encode_desc(o, buf, true);
    }
    if (flags)
        *flags = fl;
    const size_t used = buf.size() / 32;
    if (used > cap)
        return -int64_t(used);
    if (out && used)
        std::memcpy(out, buf.data(), buf.size());
    return int64_t(used);
}

namespace {
// bdt_used of an imported description: its DATA entries' predefined ids
uint32_t bdt_of(const std::vector<Node> &nodes)
{
    uint32_t m = 0;
    for (const Node &n : nodes)
        m |= n.kind == Node::LOOP ? bdt_of(n.body) : (n.tid ? 1u << n.tid : 0u);
    return m;
}
}  // namespace

int ddt_type_from_opal_desc(const void *desc, size_t used, size_t size, ptrdiff_t lb, ptrdiff_t ub,
                            ptrdiff_t true_lb, ptrdiff_t true_ub, ddt_datatype_t **out)
{
    if (!desc || !out)
        return DDT_ERR_BAD_PARAM;
    ddt_datatype *t = new_type();
    if (!parse_opal(static_cast<const unsigned char *>(desc), 0, used, t->desc)) {
        delete t;
        return DDT_ERR_BAD_PARAM;
    }
    t->size = int64_t(size);
    t->lb = lb;
    t->ub = ub;
    t->true_lb = true_lb;
    t->true_ub = true_ub;
    t->flags = F_DATA;
    t->nbElems = 0;
    t->imported = true;
    t->bdt_used = bdt_of(t->desc);
    uint64_t s = 0;
    for (const Node &n : t->desc)
        s += n.packed_bytes();
    if (s != size) {
        delete t;
        return DDT_ERR_BAD_PARAM;
    }
    commit(t);
    *out = t;
    return DDT_SUCCESS;
}

}  // extern "C"

namespace ddt {
// The committed tree of an optimized description: the bridge's own import (parse_opal), with
// sealed lists carried through as LIST nodes.
bool nodes_from_desc(const DescForm &d, std::vector<Node> &out)
{
    std::vector<unsigned char> raw(32 * d.used, 0);
    SealedLists lists = d.lists;   // + the slices of lists whose ends merged with a neighbour
    for (size_t i = 0; i < d.used; ++i) {
        const DescEntry &e = d.e[i];
        unsigned char *p = raw.data() + 32 * i;
        std::memcpy(p, &e.flags, 2);
        if (e.sealed >= 0) {
            const uint16_t zero = 0;
            uint32_t idx = uint32_t(e.sealed);
            const IndexList &X = *d.lists[idx];
            if (e.sb != 0 || e.se != X.nblk()) {
                auto S = std::make_shared<IndexList>();
                S->esize = X.esize;
                S->disp.assign(X.disp.begin() + e.sb, X.disp.begin() + e.se);
                if (X.len.empty())
                    S->ulen = X.ulen;
                else
                    S->len.assign(X.len.begin() + e.sb, X.len.begin() + e.se);
                idx = uint32_t(lists.size());
                lists.push_back(finish_list(S));
            }
            const uint64_t tid = e.type;
            std::memcpy(p + 2, &zero, 2);
            std::memcpy(p + 4, &idx, 4);
            std::memcpy(p + 8, &tid, 8);
            std::memcpy(p + 24, &e.disp, 8);
            continue;
        }
        std::memcpy(p + 2, &e.type, 2);
        std::memcpy(p + 4, &e.count, 4);
        if (!(e.flags & F_DATA)) {
            std::memcpy(p + 8, &e.loops, 4);
            std::memcpy(p + 16, &e.blen, 8);
            std::memcpy(p + 24, e.type == kDescLoop ? &e.extent : &e.disp, 8);
        } else {
            std::memcpy(p + 8, &e.blen, 8);
            std::memcpy(p + 16, &e.extent, 8);
            std::memcpy(p + 24, &e.disp, 8);
        }
    }
    out.clear();
    return parse_opal(raw.data(), 0, d.used, out, &lists);
}
}  // namespace ddt
