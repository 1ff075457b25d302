"""MPI_Pack / MPI_Unpack count consolidation (VERDICT r4 "missing" 3).

For count >= ompi_datatype_consolidate_threshold (250) MPI_Pack packs (1, contiguous(count, type))
instead of (count, type) (ompi/mpi/c/pack.c.in:118-125, unpack.c.in:122-129), built by
ompi_datatype_consolidate_create (ompi_datatype_create_contiguous.c:119-180): its opt_desc is one
LOOP of count over the type's committed opt_desc, re-optimized with loop-boundary expansion on that
loop only and the transforms ompi_datatype_consolidate_optimization_mask keeps
(opal_datatype_optimize_from_contiguous, opal_datatype_optimize.c:1480-1573).

Pinned by the reference's own dump (SURVEY.md Appendix A, cfg1 consolidated x2048) and by the
engine (ddt_type_consolidate) == the oracle (ort_consolidate) on fuzzed recipes, each
consolidated opt_desc moving exactly the bytes of `count` instances in type-map order.
"""
from __future__ import annotations

import random

import pytest

from tests import oracle as O
from tests import opal_shapes as S
from tests import recipes as R
from tests.test_cpu_optimizer import _flatten

FLOAT8, INT4 = 16, 6


def _both(rec, count):
    b = R.Built(rec)
    e = b.engine().consolidate(count)
    o = O.consolidate(b.o, count)
    return b, e, o


def test_appendix_a_cfg1_consolidated():
    """SURVEY App. A (the reference's opal_datatype_dump): vector(1024,1,2) double x 2048 through
    MPI_Pack = LOOP 2048 x (2 items) extent 16376 { FLOAT8 count 1024 blen 1 extent 16 } END_LOOP
    size 8192."""
    b, e, o = _both(("vector", 1024, 1, 2, ("basic", FLOAT8)), 2048)
    raw, fl = e.to_opal_opt_desc()
    ent = S.unpack_entries(raw)
    assert ent == o.opt_desc()
    loop, data, end = ent
    assert (loop[1], loop[2], loop[3], loop[5]) == (0, 2, 2048, 16376)           # LOOP 2048, 2 items
    assert (data[1], data[2], data[4], data[5], data[6]) == (FLOAT8, 1024, 1, 16, 0)
    assert (end[1], end[2], end[4]) == (1, 2, 8192)                               # END_LOOP size 8192
    assert e.info()["size"] == 2048 * 8192 and e.commit_info()["committed"] == 1
    assert e.commit_info()["stack_depth"] == 1


@pytest.mark.parametrize("rec,count", [
    (("vector", 1024, 1, 2, ("basic", FLOAT8)), 249),      # below the threshold
    (("contig", 7, ("basic", FLOAT8)), 4096),              # NO_GAPS: already contiguous
    (("basic", INT4), 1000),                               # predefined
    (("resized", ("contig", 3, ("basic", INT4)), 0, 0), 300),   # zero extent: not contiguous, consolidates
])
def test_when_the_reference_keeps_the_type(rec, count):
    b, e, o = _both(rec, count)
    assert (e is None) == (o is None)
    if e is not None:
        raw, _ = e.to_opal_opt_desc()
        assert S.unpack_entries(raw) == o.opt_desc()


def test_threshold_is_the_mca_variable():
    """ompi_datatype_consolidate_threshold (ompi_datatype_module.c:527-532): ddt_tune("consolidate")."""
    from ompi_amd._lib import lib
    rec = ("vector", 16, 1, 3, ("basic", FLOAT8))
    b = R.Built(rec)
    try:
        assert lib().ddt_tune(b"consolidate", 1000) == 0
        assert b.engine().consolidate(999) is None and O.consolidate(b.o, 999, 1000) is None
        assert b.engine().consolidate(1000) is not None
    finally:
        lib().ddt_tune(b"consolidate", 250)
    assert b.engine().consolidate(250) is not None


@pytest.mark.parametrize("kind,seed", [("any", 0), ("any", 1), ("mixed", 0), ("mixed", 1)])
def test_engine_and_oracle_consolidate_alike(kind, seed):
    """On fuzzed recipes and counts 250-700: the same decision, the same consolidated opt_desc and
    RESTRICTED flag, the contiguous constructor's desc, stack depth and bdt_used; the opt_desc
    moves count instances' bytes in type-map order."""
    rng = random.Random(5100 + 31 * seed + (kind == "mixed"))
    gen = R.random_recipe if kind == "any" else R.random_mixed_recipe
    made = 0
    for _ in range(150):
        rec = gen(rng)
        count = rng.choice([250, 256, 257, 300, 511, 700])
        b = R.Built(rec)
        if b.o.info()["size"] == 0:
            continue
        e = b.engine().consolidate(count)
        o = O.consolidate(b.o, count)
        assert (e is None) == (o is None), rec
        if e is None:
            continue
        made += 1
        raw, fl = e.to_opal_opt_desc()
        eo = S.unpack_entries(raw)
        assert eo == o.opt_desc(), (rec, count)
        assert bool(fl & 0x10000) == o.restricted(), rec
        assert S.unpack_entries(e.to_opal_desc()) == o.desc(), rec
        ec, oc = e.commit_info(), o.commit_info()
        assert (ec["stack_depth"], ec["bdt_used"]) == (oc["stack_depth"], oc["bdt_used"]), rec
        info = b.o.info()
        if len(eo) < 2000 and info["nruns"] * count < 200000:
            ext = info["ub"] - info["lb"]
            want = []
            for i in range(count):
                for d, n, *_ in b.o.runs():
                    a = d + i * ext
                    if want and want[-1][0] + want[-1][1] == a:
                        want[-1][1] += n
                    else:
                        want.append([a, n])
            assert _flatten(eo) == want, rec
    assert made > 40


def test_consolidated_send_positions_follow_its_description():
    """A send convertor on the consolidated type snaps to ITS opt_desc elements, as MPI_Pack's
    positions do: engine == oracle at random positions."""
    rng = random.Random(77)
    rec = ("struct", [1, 3], [0, 8], [("basic", FLOAT8), ("basic", INT4)])   # UINT4 x 5 carrier
    b, e, o = _both(("resized", rec, 0, 32), 300)
    assert e is not None and o is not None
    total = 300 * 20
    for p in sorted(rng.randrange(total) for _ in range(50)):
        assert e.snap_position(p) == o.set_position(1, p, send=True), p


def test_reset_restores_the_environment_threshold():
    """OMPI_MCA_datatype_consolidate_threshold sets the initial threshold; ddt_tune("reset")
    restores it (not the compiled default)."""
    import os
    import subprocess
    import sys
    code = (
        "import sys; sys.path.insert(0, %r)\n"
        "from tests import recipes as R\n"
        "from ompi_amd._lib import lib\n"
        "b = R.Built(('vector', 16, 1, 3, ('basic', 16)))\n"
        "assert b.engine().consolidate(999) is None\n"
        "assert lib().ddt_tune(b'consolidate', 5) == 0 and b.engine().consolidate(999) is not None\n"
        "assert lib().ddt_tune(b'reset', 0) == 0 and b.engine().consolidate(999) is None\n"
        "assert b.engine().consolidate(1000) is not None\n"
        "print('ok')\n" % os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    env = dict(os.environ, OMPI_MCA_datatype_consolidate_threshold="1000")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stderr[-2000:]


def test_committed_description_is_kept_across_tuning_changes():
    """the committed opt_desc is the one exported and consolidated later, whatever the
    optimizer parameters are by then (the reference keeps oldType->opt_desc; its MCA parameters
    are read at commit, opal_datatype_optimize.c:1739-1782).  struct{double,int[3]} committed
    with preserve_type on is UINT4 x 5; after preserve_type is turned off its export and its
    MPI_Pack consolidation still carry UINT4, while a type committed now carries UINT1."""
    from ompi_amd._lib import lib
    UINT1, UINT4 = 9, 11
    st = ("struct", [1, 3], [0, 8], [("basic", FLOAT8), ("basic", INT4)])
    b = R.Built(st)
    before = S.unpack_entries(b.engine().to_opal_opt_desc()[0])
    assert before[0][1] == UINT4
    assert lib().ddt_tune(b"opt_preserve", 0) == 0
    try:
        after = S.unpack_entries(b.engine().to_opal_opt_desc()[0])
        assert after == before
        cons = S.unpack_entries(b.engine().consolidate(300).to_opal_opt_desc()[0])
        assert [x[1] for x in cons if x[0] & 0x100] == [UINT4]
        fresh = S.unpack_entries(R.Built(st).engine().to_opal_opt_desc()[0])
        assert fresh[0][1] == UINT1
    finally:
        lib().ddt_tune(b"opt_preserve", 1)
