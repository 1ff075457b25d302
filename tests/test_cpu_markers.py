"""MPI_LB / MPI_UB bound markers (OPAL_DATATYPE_LB / _UB, ids 2 and 3) on CPU.

The reference handles them in opal_datatype_add unconditionally
(opal/datatype/opal_datatype_add.c:158-186): adding a marker moves the type's lower (upper) bound
to its displacement -- the min (max) with an earlier marker's -- sets USER_LB (USER_UB), drops
NO_GAPS when the extent no longer equals the size, and appends nothing.  Their predefined handles
have size 0 and no description (opal_datatype_constructors.h:77-85, 169-172), and a dup keeps the
id (opal_datatype_clone.c:74), so a duplicated marker still acts as one.  Engine and oracle are
held to each other on bounds, flags, desc and opt_desc, and to the MPI-1 known answer.
"""
from __future__ import annotations

import random

from tests import opal_shapes as S
from tests import recipes as R

LB, UB, INT4, FLOAT8, CHAR = 2, 3, 6, 16, 4
BOUND_FLAGS = 0x01F8   # OVERLAP | CONTIGUOUS | NO_GAPS | USER_LB | USER_UB | DATA


def _same(rec):
    b = R.Built(rec)
    o = b.o.info()
    e = b.engine().info()
    for k in ("size", "lb", "ub", "true_lb", "true_ub", "align"):
        assert o[k] == e[k], (k, o[k], e[k], rec)
    assert o["flags"] & BOUND_FLAGS == e["flags"] & BOUND_FLAGS, (hex(o["flags"]), hex(e["flags"]), rec)
    assert S.unpack_entries(b.e.to_opal_desc()) == b.o.desc(), rec
    assert S.unpack_entries(b.e.to_opal_opt_desc()[0]) == b.o.opt_desc(), rec
    return b, o


def test_mpi1_struct_known_answer():
    """MPI_Type_struct({1,1,1}, {-3,0,6}, {MPI_LB, MPI_INT, MPI_UB}): lb -3, ub 6 (extent 9),
    size 4, true bounds [0, 4), one INT4 entry; USER_LB and USER_UB set, NO_GAPS clear."""
    _, o = _same(("struct", [1, 1, 1], [-3, 0, 6], [("basic", LB), ("basic", INT4), ("basic", UB)]))
    assert (o["size"], o["lb"], o["ub"], o["true_lb"], o["true_ub"]) == (4, -3, 6, 0, 4)
    assert o["flags"] & 0xC0 == 0xC0 and not o["flags"] & 0x20


def test_markers_take_min_and_max():
    """Two LB markers keep the lower, two UB markers the higher (:164-166, :176-178); a marker
    inside the data pulls the bound inward (the user's bound wins over the data's)."""
    rec = ("struct", [1, 2, 1, 1, 1], [8, 0, -16, 40, 24],
           [("basic", LB), ("basic", FLOAT8), ("basic", LB), ("basic", UB), ("basic", UB)])
    _, o = _same(rec)
    assert (o["lb"], o["ub"]) == (-16, 40)
    _, o = _same(("struct", [1, 4, 1], [4, 0, 12], [("basic", LB), ("basic", INT4), ("basic", UB)]))
    assert (o["lb"], o["ub"], o["true_lb"], o["true_ub"]) == (4, 12, 0, 16)


def test_markers_through_constructors_and_dup():
    """Markers under contiguous / vector / resized / dup, and a dup of the marker itself (the id
    survives the clone, so it still only moves a bound)."""
    inner = ("struct", [1, 1, 1], [-8, 0, 16], [("basic", LB), ("basic", FLOAT8), ("basic", UB)])
    for rec in [("contig", 3, inner), ("vector", 3, 2, 3, inner), ("dup", inner),
                ("resized", inner, 0, 32), ("hvector", 2, 1, 100, inner),
                ("struct", [1, 2], [0, 4], [("dup", ("basic", LB)), ("basic", CHAR)]),
                ("struct", [2, 1], [0, 64], [("basic", INT4), ("dup", ("basic", UB))]),
                ("vector", 4, 1, 2, ("basic", UB)),
                ("struct", [1, 1], [5, 9], [("basic", LB), ("basic", UB)])]:
        _same(rec)


def marker_recipe(rng: random.Random, depth: int = 0):
    """A random recipe with LB / UB markers mixed into structs at every level."""
    if depth >= 2 or rng.random() < 0.3:
        return ("basic", rng.choice([INT4, FLOAT8, CHAR]))
    n = rng.randint(2, 4)
    subs = [marker_recipe(rng, depth + 1) for _ in range(n)]
    for _ in range(rng.randint(1, 2)):
        subs.insert(rng.randrange(len(subs) + 1), ("basic", rng.choice([LB, UB])))
    disps = sorted(rng.sample(range(-64, 256, 4), len(subs)))
    blens = [rng.randint(1, 3) for _ in subs]
    st = ("struct", blens, disps, subs)
    k = rng.random()
    if k < 0.3:
        return ("contig", rng.randint(1, 3), st)
    if k < 0.5:
        return ("vector", rng.randint(1, 3), rng.randint(1, 2), rng.randint(2, 3), st)
    return st


def test_random_marker_recipes():
    rng = random.Random(4242)
    for _ in range(300):
        _same(marker_recipe(rng))
