"""The commit optimizer on CPU: opal_datatype_commit
(opal/datatype/opal_datatype_optimize.c:1739-1782) restated twice -- by the oracle
(oracle/ddt_oracle.c, test infrastructure) and by the engine (ompi_amd/csrc/ddt_optimize.cpp,
the product's commit) -- and pinned to what the reference itself produced:

* SURVEY.md Appendix A, the `opal_datatype_dump` output of the real reference for the BASELINE
  shapes (cfg1, the cfg2 faces, cfg3's dim-2 face, cfg5's struct{double,int[3]} and its hvector,
  cfg4's two-block FLOAT4 pairs);
* `position.c` on MPI_LONG_DOUBLE_INT (365 x 112-byte segments + 80, recorded from the
  reference): the 20 fused bytes of {long double, int} are one UINT4 x 5 carrier;
* datatype_corpus.c's merged struct{double,long,char} (17 contiguous bytes of three types:
  one UINT1 carrier, opal_datatype_optimize.c:581-611).

Then the two restatements are held to each other entry for entry (desc, opt_desc and the
OPTIMIZED_RESTRICTED flag) on thousands of fuzzed recipes, half of them mixed-type structs in
loops, and every opt_desc must describe exactly the bytes of its desc in the same order.
"""
from __future__ import annotations

import random

import pytest

from tests import corpus as C
from tests import opal_shapes as S
from tests import oracle as O
from tests import recipes as R
from tests.positioning import create_segments

INT4, UINT1, UINT4, FLOAT4, FLOAT8, FLOAT12, LONG, CHAR = 6, 9, 11, 15, 16, 17, 25, 4
F_DATA = 0x100
BASIC = 0x136   # OPAL_DATATYPE_FLAG_BASIC
CHANGED = 0x200  # OPAL_DATATYPE_OPTIMIZED_TYPE_CHANGED


def _data(e):
    """DATA entry 7-tuple -> (type, count, blocklen, extent, disp)."""
    assert e[0] & F_DATA
    return (e[1], e[2], e[4], e[5], e[6])


def _engine(rec):
    b = R.Built(rec)
    raw, fl = b.engine().to_opal_opt_desc()
    return b, S.unpack_entries(raw), fl


def _both(rec):
    """(oracle opt_desc, engine opt_desc, oracle restricted, engine restricted)."""
    b, eng, fl = _engine(rec)
    return b.o.opt_desc(), eng, b.o.restricted(), bool(fl & 0x10000)


# ------------------------------------------------------------------ Appendix A
def test_appendix_a_cfg1_and_halo_faces():
    """cfg1 vector(1024,1,2) double: FLOAT8 count 1024 blen 1 extent 16; the 256^3 x face
    vector(65536,1,256): FLOAT8 count 65536 extent 2048; the y face vector(256,256,65536):
    FLOAT8 count 256 blen 256 extent 524288 -- unchanged by the optimizer, no re-typing."""
    d = ("basic", FLOAT8)
    for rec, want in [
        (("vector", 1024, 1, 2, d), (FLOAT8, 1024, 1, 16, 0)),
        (("vector", 65536, 1, 256, d), (FLOAT8, 65536, 1, 2048, 0)),
        (("vector", 256, 256, 65536, d), (FLOAT8, 256, 256, 524288, 0)),
    ]:
        o, e, ro, re_ = _both(rec)
        assert [_data(x) for x in o] == [want] and o == e, rec
        assert not ro and not re_


def test_appendix_a_cfg3_thin_face():
    """512^3 float subarray, sub {512,512,1} at start 511 (C order): FLOAT4 count 262144
    disp 2044 blen 1 extent 2048."""
    rec = ("subarray", [512, 512, 512], [512, 512, 1], [0, 0, 511], 0, ("basic", FLOAT4))
    b, e, _ = _engine(rec)
    assert [_data(x) for x in e] == [(FLOAT4, 262144, 1, 2048, 2044)]
    assert b.o.opt_desc() == e


def test_appendix_a_cfg5_struct_and_hvector():
    """struct{double, int[3]}: opt_desc UINT4 count 1 blen 5 extent 20, RESTRICTED; hvector(N, 1,
    32 B) of it: UINT4 count N blen 5 extent 32 (the contiguous loop compressed and re-typed,
    :641-709).  N = 128 Mi through the engine (its description stays one LOOP entry), 64 Ki
    through the oracle (which also flattens the type map)."""
    st = ("struct", [1, 3], [0, 8], [("basic", FLOAT8), ("basic", INT4)])
    o, e, ro, re_ = _both(st)
    assert [_data(x) for x in e] == [(UINT4, 1, 5, 20, 0)] and o == e and ro and re_
    assert e[0][0] & CHANGED
    rec = ("hvector", 1 << 16, 1, 32, st)
    b, e, fl = _engine(rec)
    assert [_data(x) for x in e] == [(UINT4, 1 << 16, 5, 32, 0)] and fl & 0x10000
    assert b.o.opt_desc() == e and b.o.restricted()
    t = R.build_engine(("hvector", 128 << 20, 1, 32, st)).commit()   # engine only: no flat map
    raw, fl = t.to_opal_opt_desc()
    assert [_data(x) for x in S.unpack_entries(raw)] == [(UINT4, 128 << 20, 5, 32, 0)] and fl & 0x10000


def test_appendix_a_cfg4_two_block_pairs():
    """indexed(n, blocklens 1, LCG displacements) of float: the optimizer pairs consecutive
    one-element blocks into `FLOAT4 count 2 blen 1 extent (d2 - d1)` (:1179-1185), so opt_desc
    holds n/2 entries for n unique, non-adjacent displacements (App. A: 64 Mi -> 33,554,432)."""
    n = 4096
    x, disps = 0x5EED, []
    for _ in range(n):
        disps.append(x)
        x = (1664525 * x + 1013904223) % (1 << 28)
    rec = ("indexed", [1] * n, disps, ("basic", FLOAT4))
    b, e, _ = _engine(rec)
    o = b.o.opt_desc()
    assert o == e
    adjacent = sum(1 for a, c in zip(disps, disps[1:]) if c == a + 1)
    assert len(b.o.desc()) == n - adjacent
    pairs = [x for x in o if x[2] == 2]
    assert len(pairs) >= (n - adjacent) // 2 - 2
    for fl, ty, cnt, _, bl, ext, disp in pairs:
        assert ty == FLOAT4 and bl == 1 and ext != 4


# ------------------------------------------------------------------ reference answers
def test_position_c_segments_from_the_constructors():
    """position.c (:42-85, :211-272) on MPI_LONG_DOUBLE_INT x 2048 -- struct{long double @0,
    int @16} resized to 32 -- built with the constructors, not hand-written: both restatements
    fuse the 20 bytes into UINT4 x 5, so 113-byte fragments snap to 112 bytes: 365 segments of
    112 and one of 80, as the reference ran.  The engine's own send positions agree."""
    rec = ("resized", ("struct", [1, 1], [0, 16], [("basic", FLOAT12), ("basic", INT4)]), 0, 32)
    b, e, fl = _engine(rec)
    assert [_data(x) for x in e] == [(UINT4, 1, 5, 20, 0)] and fl & 0x10000
    segs = create_segments(2048 * 20, 113, lambda p: b.o.set_position(2048, p, send=True))
    assert [n for _, n in segs] == [112] * 365 + [80]
    eng = b.engine()
    assert segs == create_segments(2048 * 20, 113,
                                   lambda p: 2048 * 20 if p >= 2048 * 20 else eng.snap_position(p))


def test_merged_contig_with_gaps_is_one_byte_carrier():
    """datatype_corpus.c:59-97 struct{double @0, long @8, char @16}: 17 contiguous bytes of three
    types, no UINT8/4/2 tiles 17 -> UINT1 blen 17; a pack fragment may stop on any byte."""
    rec, _ = C.merged_contig_with_gaps()
    o, e, ro, re_ = _both(rec)
    assert [_data(x) for x in e] == [(UINT1, 1, 17, 17, 0)] and o == e and ro and re_
    b = R.Built(rec)
    assert [b.o.set_position(7, p) for p in (1, 12, 30, 119)] == [1, 12, 30, 119]


def test_mixed_same_size_blocks_take_the_aligned_carrier():
    """Equal-size blocks of different types merge into one count-2 entry (:1170-1199): int @0 and
    float @8 -> UINT4 count 2 extent 8; double @4 + long @12 abut, and at that 4-byte phase only
    UINT4 tiles them (UINT8 needs 8-byte alignment, :600-606): UINT4 count 2 blen 2 extent 8,
    which CREATE_ELEM collapses to one 16-byte block of UINT4 x 4; char[2] @0 + short @4 ->
    UINT2 count 2 (the chars' byte boundaries are gone)."""
    cases = [
        (("struct", [1, 1], [0, 8], [("basic", INT4), ("basic", FLOAT4)]), (UINT4, 2, 1, 8, 0)),
        (("struct", [1, 1], [4, 12], [("basic", FLOAT8), ("basic", LONG)]), (UINT4, 1, 4, 16, 4)),
        (("struct", [2, 1], [0, 4], [("basic", CHAR), ("basic", 5)]), (10, 2, 1, 4, 0)),
    ]
    for rec, want in cases:
        o, e, ro, re_ = _both(rec)
        assert [_data(x) for x in e] == [want] and o == e and ro and re_, (rec, e)


# ------------------------------------------------------------------ the two restatements agree
def _flatten(ents, at=0):
    """The byte runs a description moves, in order (adjacent runs joined)."""
    out = []

    def walk(lo, hi, base):
        pos = lo
        while pos < hi:
            fl, ty, cnt, loops, bl, ext, disp = ents[pos]
            if fl & F_DATA:
                n = bl * S.BASIC_SIZE[ty]
                for k in range(cnt):
                    a = base + disp + k * ext
                    if out and out[-1][0] + out[-1][1] == a:
                        out[-1][1] += n
                    else:
                        out.append([a, n])
                pos += 1
            elif ty == 0:
                for k in range(loops):
                    walk(pos + 1, pos + cnt, base + k * ext)
                pos += cnt + 1
            else:
                pos += 1
    walk(0, len(ents), at)
    return out


@pytest.mark.parametrize("kind,seed", [("any", 0), ("any", 1), ("mixed", 0), ("mixed", 1), ("mixed", 2)])
def test_engine_and_oracle_optimizers_agree(kind, seed):
    """desc, opt_desc and OPTIMIZED_RESTRICTED: engine == oracle on fuzzed recipes, and each
    opt_desc moves its desc's bytes in type-map order."""
    rng = random.Random(4400 + 17 * seed + (kind == "mixed"))
    gen = R.random_recipe if kind == "any" else R.random_mixed_recipe
    n = restricted = 0
    for _ in range(500):
        rec = gen(rng)
        b = R.Built(rec)
        if b.o.info()["size"] == 0:
            continue
        e = b.engine()
        od, oo = b.o.desc(), b.o.opt_desc()
        ed = S.unpack_entries(e.to_opal_desc())
        raw, fl = e.to_opal_opt_desc()
        eo = S.unpack_entries(raw)
        assert ed == od, rec
        assert eo == oo, rec
        assert bool(fl & 0x10000) == b.o.restricted(), rec
        if len(oo) < 4000:
            assert _flatten(oo) == _flatten(od), rec
        n += 1
        restricted += b.o.restricted()
    assert n > 300
    if kind == "mixed":
        assert restricted > 150


# the reference's optimizer MCA variables (opal_datatype_module.c:85-90, :347-383) away from
# their defaults: (max_desc_growth, loop_unroll_max_items, loop_unroll_max_data_bytes, preserve_type)
NONDEFAULT = {
    "no_preserve": (10, 8, 128, False),        # every fused mixed region a UINT1 carrier (:586-588)
    "unroll_2x32": (10, 2, 32, True),
    "unroll_32x1024": (10, 32, 1024, True),
    "growth_1": (1, 8, 128, True),
    "growth_0_no_unroll": (0, 0, 0, True),
}


def _configure(growth, items, nbytes, preserve):
    from ompi_amd._lib import lib
    O.optimize_config(growth, items, nbytes, preserve)
    for k, v in (("opt_growth", growth), ("opt_unroll_items", items), ("opt_unroll_bytes", nbytes),
                 ("opt_preserve", int(preserve))):
        assert lib().ddt_tune(k.encode(), v) == 0


@pytest.mark.parametrize("name", sorted(NONDEFAULT))
def test_optimizers_agree_under_nondefault_parameters(name):
    """The 2,500-recipe agreement (desc, opt_desc, RESTRICTED, engine == oracle) under the
    reference's optimizer parameters set away from their defaults, through the engine's ABI
    (ddt_tune opt_*) and the oracle's ort_optimize_config: 500 recipes each, half mixed-type."""
    growth, items, nbytes, preserve = NONDEFAULT[name]
    rng = random.Random(4700 + sorted(NONDEFAULT).index(name))
    _configure(growth, items, nbytes, preserve)
    n = wide = 0
    try:
        for i in range(500):
            rec = R.random_mixed_recipe(rng) if i % 2 else R.random_recipe(rng)
            b = R.Built(rec)
            if b.o.info()["size"] == 0:
                continue
            e = b.engine()
            oo = b.o.opt_desc()
            raw, fl = e.to_opal_opt_desc()
            eo = S.unpack_entries(raw)
            assert S.unpack_entries(e.to_opal_desc()) == b.o.desc(), rec
            assert eo == oo, (name, rec)
            assert bool(fl & 0x10000) == b.o.restricted(), rec
            if len(oo) < 4000:
                assert _flatten(oo) == _flatten(b.o.desc()), rec
            changed = [x for x in oo if x[0] & CHANGED]
            if not preserve:
                assert all(x[1] == UINT1 for x in changed), rec
            wide += any(x[1] in (10, 11, 12) for x in changed)
            n += 1
    finally:
        _configure(10, 8, 128, True)
    assert n > 300
    if not preserve:
        assert wide == 0
    # the defaults are back: struct{double,int[3]} is UINT4 x 5 again
    o, eng, _, _ = _both(("struct", [1, 3], [0, 8], [("basic", FLOAT8), ("basic", INT4)]))
    assert [_data(x) for x in eng] == [(UINT4, 1, 5, 20, 0)] and o == eng


def test_preserve_type_off_makes_byte_carriers_and_positions():
    """preserve_type = false (MCA opal_datatype_optimize_preserve_type): struct{double,int[3]}
    commits as UINT1 x 20 in both restatements, so a send position may stop on any byte of it
    (position.c's 113-byte fragments are no longer snapped to 112)."""
    st = ("struct", [1, 3], [0, 8], [("basic", FLOAT8), ("basic", INT4)])
    _configure(10, 8, 128, False)
    try:
        o, e, ro, re_ = _both(st)
        assert [_data(x) for x in e] == [(UINT1, 1, 20, 20, 0)] and o == e and ro and re_
        b = R.Built(st)
        eng = b.engine()
        for p in (1, 7, 13, 39):
            assert eng.snap_position(p) == p == b.o.set_position(3, p, send=True)
    finally:
        _configure(10, 8, 128, True)


@pytest.mark.parametrize("seed", range(3))
def test_engine_snap_follows_carriers_on_mixed_types(seed):
    """Send positions on mixed-type recipes: the engine's snap (its committed opt_desc) ==
    the oracle's walk of its own opt_desc, at random positions, counts 1-3."""
    rng = random.Random(4500 + seed)
    checked = 0
    for _ in range(150):
        b = R.Built(R.random_mixed_recipe(rng))
        info = b.o.info()
        if info["size"] == 0:
            continue
        e = b.engine()
        for count in (1, 2, 3):
            total = count * info["size"]
            if (info["flags"] & 0x20) or ((info["flags"] & 0x10) and count == 1):
                continue
            for p in {rng.randrange(total) for _ in range(10)}:
                assert e.snap_position(p) == b.o.set_position(count, p, send=True), (b.recipe, count, p)
                checked += 1
    assert checked > 500


def test_sealed_list_exports_the_reference_opt_desc():
    """An index list of more than 2^20 blocks passes the optimizer sealed (one opaque element),
    but its export applies the optimizer's DATA merges along the list (count-2 pairs at their
    distance, arithmetic runs extended, blocks the constructor already fused kept whole:
    opal_datatype_optimize.c:1146-1278), and the LOOPs around it count the expanded entries: the
    committed description equals the oracle's entry for entry, as config 4's 33.5 M pairs would
    (SURVEY.md §8a a3).  Boundaries with neighbouring elements: the next two tests."""
    import numpy as np
    rng = np.random.default_rng(5)
    n = (1 << 20) + 4099
    d = rng.permutation(8 * n)[:n] * 2
    d[1000:1100] = 5 * np.arange(100) + 20 * n     # an arithmetic run: one entry of count 100
    d[2000:2010] = np.arange(10) + 22 * n          # adjacent blocks: fused by the constructor
    lst = ("indexed_block", 1, d.tolist(), ("basic", FLOAT4))
    for rec in (lst, ("contig", 2, lst)):
        b, eng, fl = _engine(rec)
        assert eng == b.o.opt_desc(), rec[0]
        assert S.unpack_entries(b.e.to_opal_desc()) == b.o.desc(), rec[0]
        assert not fl & 0x10000


def test_sealed_list_boundaries_merge_like_separate_entries():
    """The elements around a sealed list meet its first and last blocks as the reference's
    separate DATA entries would: a FLOAT4 before the list pairs with block 0 (shifting the pairing
    of the whole list), an INT4 adjacent after the last block fuses into a UINT4 carrier
    (OPTIMIZED_RESTRICTED), a DOUBLE adjacent before block 0 fuses into a mixed region; also inside
    loops.  Engine == oracle entry for entry, and the committed tree (with the list sliced where
    its ends merged) still walks the type map's bytes in order (raw export == oracle's)."""
    import numpy as np
    from tests.test_cpu_raw import engine_raw_all, stitched
    rng = np.random.default_rng(9)
    n = (1 << 20) + 33
    d = (rng.permutation(8 * n)[:n] * 2 + 100).astype(np.int64)
    lst = ("hindexed_block", 1, (d * 4).tolist(), ("basic", FLOAT4))
    first, last = int(d[0]) * 4, int(d[-1]) * 4
    both = ("struct", [1, 1, 1], [first - 12, 0, last + 4], [("basic", FLOAT4), lst, ("basic", INT4)])
    cases = [both, ("struct", [1, 1], [first - 8, 0], [("basic", FLOAT8), lst]), ("contig", 2, both)]
    for rec in cases:
        b, eng, fl = _engine(rec)
        assert eng == b.o.opt_desc() and bool(fl & 0x10000) == b.o.restricted()
    b = R.Built(both)
    info = b.o.info()
    base = (1 << 40) + R.layout(info, 1)[1]
    full, got = b.o.raw(1, base, 0, 1 << 22)
    chunks, tot = engine_raw_all(b.engine(), 1, base, 1 << 22)
    assert tot == got == info["size"] and stitched(chunks) == full


def test_sealed_list_in_a_loop_boundary_fusion():
    """optimize_loop_boundary (:799-888) with a sealed list as the loop body's first and last
    item: when the list's last block is byte-adjacent to the next iteration's first block, the
    reference fuses them (a loop of count - 1 around the fused element); the engine splits the
    list's range the same way.  Engine == oracle entry for entry."""
    import numpy as np
    rng = np.random.default_rng(11)
    n = (1 << 20) + 17
    d = (rng.permutation(8 * n)[:n] * 2 + 100).astype(np.int64)
    if d[-1] < d[0]:
        d[0], d[-1] = d[-1], d[0]
    lst = ("hindexed_block", 1, (d * 4).tolist(), ("basic", FLOAT4))
    f, last = int(d[0]) * 4, int(d[-1]) * 4
    rec = ("contig", 3, ("resized", lst, 0, last + 4 - f))
    b, eng, fl = _engine(rec)
    o = b.o.opt_desc()
    assert eng == o
    assert any(e[1] == 0 and e[3] == 2 for e in o)   # the reference did fuse: a loop of 2


# OMPI_MCA_opal_datatype_optimize_preserve_type values and what mca_base_var_enum_bool_vfs
# (mca_base_var_enum.c:77-104) makes of them: None = refused, the default (true) kept
_MCA_BOOLS = [("0", False), ("1", True), ("2", True), (" 0", False), ("false", False), ("f", False),
              ("no", False), ("n", False), ("disabled", False), ("true", True), ("yes", True),
              ("enabled", True), ("t", True), ("y", True), ("off", None), ("FALSE", None), ("", False),
              ("bogus", None)]


def test_preserve_type_environment_is_parsed_as_an_mca_bool():
    """the environment form of preserve_type follows mca_base_var's bool rules, so
    'off' or 'FALSE' (refused by Open MPI) keep the default instead of turning preservation on
    or off; the effect is read off the committed carrier of struct{double,int[3]} (UINT4 x 5
    preserved, UINT1 x 20 not)."""
    import os
    import subprocess
    import sys
    code = (
        "import sys; sys.path.insert(0, %r)\n"
        "from tests import recipes as R\n"
        "from tests import opal_shapes as S\n"
        "b = R.Built(('struct', [1, 3], [0, 8], [('basic', 16), ('basic', 6)]))\n"
        "raw, fl = b.engine().to_opal_opt_desc()\n"
        "print(S.unpack_entries(raw)[0][1])\n" % os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    for val, expect in _MCA_BOOLS:
        env = dict(os.environ, OMPI_MCA_opal_datatype_optimize_preserve_type=val)
        r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr[-2000:]
        carrier = int(r.stdout.split()[-1])
        preserved = carrier == UINT4
        assert preserved == (True if expect is None else expect), (val, carrier)
