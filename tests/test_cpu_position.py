"""Send-side positioning on CPU: where set_position leaves a send
convertor, engine and bridge, against the oracle's restatement of
opal_convertor_position_generic (opal_convertor.c:445-471) + opal_datatype_position.c:167-367.

No data moves here: the engine's snap and the bridge's fPosition are host code.  The GPU suite
packs and unpacks through the positions these tests pin (test_gpu_position.py).
"""
from __future__ import annotations

import random

import pytest

from tests import corpus as C
from tests import opal_shapes as S
from tests import oracle as O
from tests import recipes as R
from tests.positioning import create_segments

UINT4, FLOAT8, INT4 = 11, 16, 6
FAKE_DEV = 0x7000_0000_0000   # the bridge's fPosition never touches the buffer


def _no_op(info, count):
    return bool(info["flags"] & 0x20) or (bool(info["flags"] & 0x10) and count == 1)


@pytest.mark.parametrize("seed", range(4))
def test_engine_snap_matches_oracle_send_position(seed):
    """ddt_type_snap_position == the oracle's send-convertor landing point on 400 random types
    (every constructor, nesting depth 3) at random and boundary positions."""
    rng = random.Random(7100 + seed)
    checked = 0
    for _ in range(100):
        b = R.Built(R.random_recipe(rng))
        info = b.o.info()
        if info["size"] == 0:
            continue
        e = b.engine()
        for count in (1, 2, 3):
            total = count * info["size"]
            ps = {0, total, total - 1, 1} | {rng.randrange(total + 1) for _ in range(12)}
            for p in sorted(x for x in ps if 0 <= x <= total):
                want = b.o.set_position(count, p, send=True)
                got = p if (p >= total or _no_op(info, count)) else e.snap_position(p)
                assert got == want, (b.recipe, count, p, got, want)
                assert b.o.set_position(count, p, send=False) == min(p, total)
                checked += 1
    assert checked > 1000


def _reference_ldi():
    """MPI_LONG_DOUBLE_INT as the reference commits it (ompi_datatype_module.c:449-474,584):
    struct {long double @0, int @16}, ub forced to 32, then the optimizer fuses the 20
    contiguous bytes of two types into one carrier of the widest UINTn that tiles them
    (opal_datatype_optimize.c:581-611): UINT4 count 1 blen 5.  Oracle twin: 5 UINT4, extent 32."""
    ot = S.OpalType([S.data(UINT4, 1, 5, 20, 0)], 20, 0, 32, 0, 20, flags=S.F_CONTIGUOUS)
    oo = O.resized(O.contiguous(5, O.basic(UINT4)), 0, 32)
    return ot, oo


def _bridge_send_positioner(ot, count):
    c = S.Convertor()
    assert c.prepare(ot, count, FAKE_DEV, send=True) == S.OPAL_SUCCESS
    return c


def test_bridge_position_c_segments_follow_the_reference():
    """position.c's create_segments (position.c:42-85) on MPI_LONG_DOUBLE_INT x 2048 with
    113-byte fragments, through opal_convertor_set_position -> opal_position_hip on Open MPI's
    own convertor.  Each set_position(start + 113) lands on the UINT4 carrier grid: 112-byte
    segments, so the reference's loop grows from 363 to 366 segments, the last of 80 bytes."""
    ot, oo = _reference_ldi()
    total = 2048 * 20
    c = _bridge_send_positioner(ot, 2048)
    segs = create_segments(total, 113, c.set_position)
    assert len(segs) == 366
    assert [n for _, n in segs] == [112] * 365 + [80]
    assert segs == create_segments(total, 113, lambda p: oo.set_position(2048, p, send=True))
    # a receive convertor keeps the byte (position.c's unpack side sets segment starts only)
    r = S.Convertor()
    r.prepare(ot, 2048, FAKE_DEV, send=False)
    assert r.set_position(113) == 113
    ot.destruct()


def test_bridge_send_position_snaps_on_the_imported_carriers():
    """cfg5's promoted record (UINT4 count 128M blen 5 extent 32, shrunk here)
    and the cfg2 x face (FLOAT8 count 256 blen 1 extent 2048): a send set_position lands on the
    carrier grid of use_desc; bConverted and the returned value agree; a position on the grid,
    0, and the end are unchanged."""
    cases = [
        (S.OpalType([S.data(UINT4, 4096, 5, 32, 0)], 4096 * 20, 0, 4096 * 32 - 12, 0, 4096 * 32 - 12),
         O.hvector(4096, 1, 32, O.contiguous(5, O.basic(UINT4))), 3),
        (S.OpalType([S.data(FLOAT8, 256, 1, 2048, 0)], 2048, 0, 255 * 2048 + 8, 0, 255 * 2048 + 8),
         O.vector(256, 1, 256, O.basic(FLOAT8)), 2),
    ]
    rng = random.Random(71)
    for ot, oo, count in cases:
        total = count * ot.dt.size
        assert oo.size * count == total
        for p in [0, 1, 3, 4, 5, 19, 20, 21, total - 1, total, total + 9] + \
                 [rng.randrange(total) for _ in range(200)]:
            c = _bridge_send_positioner(ot, count)
            got = c.set_position(p)
            assert got == oo.set_position(count, p, send=True), (p, got)
            assert c.c.bConverted == got and c.c.partial_length == 0
        ot.destruct()


def test_bridge_send_position_on_corpus_types():
    """Every corpus datatype (datatype_corpus.c:2143-2236) as a flat description (one DATA per
    run of the type map): random mid-element send positions land where the oracle's walk
    lands; ascending positions on one convertor (create_segments' pattern) as well."""
    rng = random.Random(72)
    n = 0
    for name in sorted(C.CORPUS):
        rec, _ = C.CORPUS[name]()
        oo = R.Built(rec).o
        info = oo.info()
        if info["size"] == 0:
            continue
        for count in (1, 7):
            if _no_op(info, count):
                continue
            ot = S.from_oracle(oo)
            total = count * info["size"]
            c = _bridge_send_positioner(ot, count)
            pos = 0
            while pos < total:   # one convertor, increasing targets, like create_segments
                tgt = pos + rng.randint(1, 97)
                pos = c.set_position(tgt)
                assert pos == oo.set_position(count, tgt, send=True), (name, count, tgt, pos)
                n += 1
            for _ in range(20):   # fresh convertors, arbitrary targets
                p = rng.randrange(total)
                c = _bridge_send_positioner(ot, count)
                assert c.set_position(p) == oo.set_position(count, p, send=True), (name, count, p)
            ot.destruct()
    assert n > 200
