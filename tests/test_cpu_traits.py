"""The corpus' trait tags pin the engine's commit metadata (flags, bounds, stack_depth, bdt_used).

The reference tags every corpus datatype with shape traits (datatype_corpus.c:2143-2236, enum at
datatype_corpus.h:54-65), and opt_desc_equiv.c recomputes them from the COMMITTED type --
MPI_Type_get_extent / get_true_extent and opal_datatype_t::{flags, size, bdt_used, stack_depth}
(`observed_traits`, opt_desc_equiv.c:223-276) -- failing on any mismatch (:278-290, :458).
`observed` below restates that function; TRAITS holds the reference's tags as data.  Both the
engine (ddt_type_commit_info) and the oracle (ort_commit_info) must reproduce every tag, so a
misreading of the committed depth or of the predefined-type set shared by the two restatements
cannot hide behind their agreement with each other.
"""
from __future__ import annotations

import random

import pytest

from . import corpus
from . import recipes as R

# datatype_corpus.h:54-65
CONTIGUOUS, HAS_GAPS, NESTED_LOOP, RESIZED, MIXED_TYPES = 1, 2, 4, 8, 16
SINGLE_ITER, NEG_EXTENT, ZERO_EXTENT, OVERLAP, PAIR = 32, 64, 128, 256, 512
NAMES = {CONTIGUOUS: "CONTIGUOUS", HAS_GAPS: "HAS_GAPS", NESTED_LOOP: "NESTED_LOOP", RESIZED: "RESIZED",
         MIXED_TYPES: "MIXED_TYPES", SINGLE_ITER: "SINGLE_ITER", NEG_EXTENT: "NEG_EXTENT",
         ZERO_EXTENT: "ZERO_EXTENT", OVERLAP: "OVERLAP", PAIR: "PAIR"}

# the `traits` column of corpus_desc[] (datatype_corpus.c:2143-2236), entry by entry
TRAITS = {
    "contig": CONTIGUOUS,
    "indexed_gap": HAS_GAPS | NESTED_LOOP | MIXED_TYPES,
    "optimized_indexed_gap": HAS_GAPS | RESIZED,
    "constant_gap": HAS_GAPS,
    "optimized_constant_gap": HAS_GAPS,
    "struct_constant_gap": HAS_GAPS,
    "struct_constant_gap_resized": CONTIGUOUS | RESIZED | MIXED_TYPES,
    "struct_merged_with_gap_resized": CONTIGUOUS | RESIZED | MIXED_TYPES,
    "ddtbench_fft2d_scatter": HAS_GAPS | RESIZED | OVERLAP,
    "ddtbench_fft2d_gather": HAS_GAPS | RESIZED | OVERLAP,
    "ddtbench_milc_su3_zdown": HAS_GAPS,
    "ddtbench_nas_lu_y": HAS_GAPS,
    "ddtbench_nas_lu_x": CONTIGUOUS,
    "ddtbench_nas_mg_x": HAS_GAPS,
    "ddtbench_nas_mg_y": HAS_GAPS,
    "ddtbench_nas_mg_z": HAS_GAPS,
    "ddtbench_lammps_full": HAS_GAPS | PAIR | RESIZED,
    "ddtbench_lammps_atomic": HAS_GAPS | PAIR | RESIZED,
    "ddtbench_specfem3d_oc": HAS_GAPS | RESIZED,
    "ddtbench_specfem3d_cm": HAS_GAPS | RESIZED,
    "ddtbench_specfem3d_mt": HAS_GAPS | PAIR,
    "ddtbench_wrf_vec": HAS_GAPS | RESIZED,
    "ddtbench_wrf_subarray": HAS_GAPS | RESIZED,
    "complex_hvector": HAS_GAPS,
    "adv_single_iter_gap": CONTIGUOUS | SINGLE_ITER | RESIZED,
    "adv_zero_extent_overlap": CONTIGUOUS | ZERO_EXTENT | OVERLAP | RESIZED,
    "adv_neg_extent": CONTIGUOUS | NEG_EXTENT | RESIZED,
    "adv_mixed_promote": CONTIGUOUS | MIXED_TYPES | RESIZED,
}

F_OVERLAP, F_CONTIGUOUS, F_USER_LB, F_USER_UB = 0x0008, 0x0010, 0x0040, 0x0080
NON_PAYLOAD = (1 << 0) | (1 << 1) | (1 << 2) | (1 << 3)   # LOOP, END_LOOP, LB, UB ids


def observed(info: dict, stack_depth: int, bdt_used: int, pair: bool) -> int:
    """observed_traits (opt_desc_equiv.c:223-276) on a committed type's metadata."""
    lb, extent = info["lb"], info["ub"] - info["lb"]
    true_lb, true_extent = info["true_lb"], info["true_ub"] - info["true_lb"]
    flags, size = info["flags"], info["size"]
    t = PAIR if pair else 0
    if extent < 0:
        t |= NEG_EXTENT
    if extent == 0:
        t |= ZERO_EXTENT
    if flags & F_OVERLAP:
        t |= OVERLAP
    elif true_extent > 0 and true_extent > abs(extent):
        t |= OVERLAP
    if flags & F_CONTIGUOUS:
        t |= CONTIGUOUS
    if true_extent > size:
        t |= HAS_GAPS
    if (flags & (F_USER_LB | F_USER_UB)) or extent != true_extent or lb != true_lb:
        t |= RESIZED
    if stack_depth >= 2:
        t |= NESTED_LOOP
    payload = bdt_used & ~NON_PAYLOAD
    if payload & (payload - 1):
        t |= MIXED_TYPES
    if ((flags & F_CONTIGUOUS) and extent > true_extent and extent > 0 and stack_depth < 2
            and not (t & (OVERLAP | MIXED_TYPES))):
        t |= SINGLE_ITER
    return t


def spell(t: int) -> str:
    return "|".join(n for b, n in NAMES.items() if t & b) or "(none)"


def test_traits_cover_the_corpus():
    assert set(TRAITS) == set(corpus.CORPUS)
    assert set(corpus.PAIR_RECV) == {n for n, t in TRAITS.items() if t & PAIR}


@pytest.mark.parametrize("name", sorted(corpus.CORPUS))
def test_corpus_traits_engine_and_oracle(name):
    rec, _ = corpus.CORPUS[name]()
    pair = name in corpus.PAIR_RECV
    b = R.Built(rec)
    oi, oc = b.o.info(), b.o.commit_info()
    o_traits = observed(oi, oc["stack_depth"], oc["bdt_used"], pair)
    e = b.engine()
    ei, ec = e.info(), e.commit_info()
    assert ec["committed"] == 1
    e_traits = observed(ei, ec["stack_depth"], ec["bdt_used"], pair)
    want = TRAITS[name]
    assert o_traits == want, f"oracle {spell(o_traits)} != declared {spell(want)}"
    assert e_traits == want, f"engine {spell(e_traits)} != declared {spell(want)}"
    assert (ec["stack_depth"], ec["bdt_used"]) == (oc["stack_depth"], oc["bdt_used"])


@pytest.mark.parametrize("name", sorted(corpus.PAIR_RECV))
def test_pair_receive_types_hold_the_send_stream(name):
    """The PAIR entries' receive types (datatype_corpus.c:626-789) take the send type's packed
    stream (equal sizes), and their commit metadata agrees between engine and oracle."""
    srec, _ = corpus.CORPUS[name]()
    rrec = corpus.PAIR_RECV[name]
    s, r = R.Built(srec), R.Built(rrec)
    assert s.o.info()["size"] == r.o.info()["size"] == s.engine().info()["size"] == r.engine().info()["size"]
    rc = r.engine().commit_info()
    assert (rc["stack_depth"], rc["bdt_used"]) == (r.o.commit_info()["stack_depth"],
                                                   r.o.commit_info()["bdt_used"])


def test_commit_metadata_engine_equals_oracle_on_fuzzed_recipes():
    """stack_depth and bdt_used of 600 random recipes (half mixed-type structs in loops, LB/UB
    markers included through the random constructors): engine == oracle."""
    rng = random.Random(0x7A17)
    for i in range(600):
        rec = R.random_mixed_recipe(rng) if i % 2 else R.random_recipe(rng)
        b = R.Built(rec)
        oc = b.o.commit_info()
        ec = b.engine().commit_info()
        assert (ec["stack_depth"], ec["bdt_used"]) == (oc["stack_depth"], oc["bdt_used"]), rec


def test_stack_depth_and_bdt_known_answers():
    """Small known answers from the reference's own rules: a predefined type has depth 0 and its
    own bit (opal_datatype_constructors.h:87-96); vector(3,2,4) of double is ONE DATA entry
    (count 3, blen 2: the one-entry merge of opal_datatype_add.c:358-397), so depth 0; repeating
    it at another stride builds a LOOP (:400-431), and repeating that a LOOP around the LOOP;
    a struct{double,int} ORs the two bits (:306); MPI_LB / MPI_UB set their bits (:163,175)."""
    DOUBLE, INT = corpus.DOUBLE, corpus.INT
    cases = [
        (("basic", DOUBLE), 0, 1 << DOUBLE),
        (("vector", 3, 2, 4, ("basic", DOUBLE)), 0, 1 << DOUBLE),
        (("vector", 3, 1, 4, ("basic", DOUBLE)), 0, 1 << DOUBLE),
        (("contig", 3, ("vector", 3, 2, 4, ("basic", DOUBLE))), 1, 1 << DOUBLE),
        (("contig", 2, ("contig", 3, ("vector", 3, 2, 4, ("basic", DOUBLE)))), 2, 1 << DOUBLE),
        (("struct", [1, 1], [0, 8], [("basic", DOUBLE), ("basic", INT)]), 0, (1 << DOUBLE) | (1 << INT)),
        (("struct", [1, 1, 1], [0, 0, 24], [("basic", 2), ("basic", DOUBLE), ("basic", 3)]), 0,
         (1 << 2) | (1 << 3) | (1 << DOUBLE)),
    ]
    for rec, depth, bdt in cases:
        b = R.Built(rec)
        for got in (b.o.commit_info(), b.engine().commit_info()):
            assert (got["stack_depth"], got["bdt_used"]) == (depth, bdt), rec
