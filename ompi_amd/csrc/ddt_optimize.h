// ddt_optimize.h -- Open MPI's description form and commit optimizer for the engine's type maps.
//
// A committed Open MPI datatype carries two descriptions (opal_datatype.h:172-212): `desc`,
// appended to by opal_datatype_add, and `opt_desc`, which opal_datatype_commit derives from it
// (opal_datatype_optimize.c:1739-1782).  The accelerator movers walk opt_desc and never split one
// of its predefined elements (opal_datatype_pack_accelerator.c:52-58); a send convertor's position
// lands on one of them (opal_datatype_position.c:167-367).  The optimizer re-types every fused
// mixed-type region to an unsigned carrier (UINT8/4/2, else UINT1, :581-630), so those elements are
// not the type map's own.  The engine restates the optimizer (ddt_optimize.cpp) so that a type built
// with its own constructors fragments and positions exactly like the reference's.
#pragma once

#include <cstdint>
#include <memory>
#include <vector>

#include "ddt_core.h"

namespace ddt {

// One dt_elem_desc_t (opal_datatype_internal.h:119-169), fields by role:
//   DATA      {flags, type >= 4, count, -, blocklen (elements), extent, disp}
//   LOOP      {flags, 0, items, loops, -, extent, -}
//   END_LOOP  {flags, 1, items, -, size, -, first_elem_disp}
// `sealed` >= 0 marks an engine index list too long to expand entry by entry (DescForm::lists),
// its blocks [sb, se) standing for the entries the optimizer makes of them (ddt_optimize.cpp,
// "sealed lists").
struct DescEntry {
    uint16_t flags = 0, type = 0;
    uint32_t count = 0;
    uint32_t loops = 0;
    uint64_t blen = 0;
    int64_t extent = 0;
    int64_t disp = 0;
    int32_t sealed = -1;
    uint32_t sb = 0, se = 0;
};

struct DescForm {
    std::vector<DescEntry> e;                               // entries (+ END_LOOP sentinel at [used])
    size_t used = 0;
    std::vector<std::shared_ptr<const IndexList>> lists;   // sealed lists by index
};

constexpr uint16_t kDescLoop = 0, kDescEndLoop = 1;
constexpr uint32_t kTypeChanged = 0x0200u;       // OPAL_DATATYPE_OPTIMIZED_TYPE_CHANGED
constexpr uint32_t kRestricted = 0x00010000u;    // OPAL_DATATYPE_OPTIMIZED_RESTRICTED
constexpr size_t kSealBlocks = size_t(1) << 20;  // lists longer than this stay sealed

// desc of a type map as opal_datatype_add builds it (opal_datatype_add.c:307-431), with the
// END_LOOP sentinel of opal_datatype_commit_description (opal_datatype_optimize.c:467-492).
// False when an entry does not fit the 32-byte form (a count beyond 32 bits).
bool build_opal_desc(const std::vector<Node> &nodes, int64_t size, DescForm &out);

// opal_datatype_commit's optimizer (opal_datatype_optimize_short_restart with
// OPAL_DATATYPE_OPTIMIZE_ALL and the default tunables); *flags gets kRestricted when a region
// was re-typed.  `out` shares `in`'s sealed lists.
// optimization_mask bits (opal_datatype.h:148-151)
constexpr uint32_t kOptimizeFusion = 0x1u, kOptimizeBoundary = 0x2u, kOptimizeUnroll = 0x4u;
constexpr uint32_t kOptimizeAll = 0xFFFFFFFFu;
// opal_datatype_optimize_short_restart (opal_datatype_optimize.c:1347-1478): `mask` removes
// transforms, `top_only` limits loop-boundary expansion to top-level loops (the consolidation
// path, opal_datatype_optimize_from_contiguous :1480-1573)
void optimize_desc(const DescForm &in, int64_t size, DescForm &out, uint32_t *flags, uint32_t mask = kOptimizeAll,
                   bool top_only = false);
// ompi_datatype_consolidate_create (ompi_datatype_create_contiguous.c:119-180) -- see ddt_hip.h
ddt_datatype *consolidate(const ddt_datatype *old, uint64_t count, int64_t threshold);
bool desc_has_small_blocks(const DescForm &d, bool counted);
DescEntry loop_desc_entry(uint32_t loops, uint32_t items, int64_t extent, uint32_t flags);
DescEntry end_desc_entry(uint32_t items, int64_t first, uint64_t size, uint32_t flags);

// Node tree of a committed description (the bridge's import, sealed lists passed through).
bool nodes_from_desc(const DescForm &d, std::vector<Node> &out);

// 32-byte entries of a description.  Sealed lists expand one DATA entry per block, or, with
// `optimized` (the output of optimize_desc), with the optimizer's DATA merges applied along the
// list (count-2 pairs at their distance, arithmetic runs extended: opal_datatype_optimize.c
// :1146-1278), so the export of a committed 64 Mi-block list is the reference's opt_desc.
void encode_desc(const DescForm &d, std::vector<unsigned char> &out, bool optimized = false);

}  // namespace ddt
