"""Raw iovec export (opal_convertor_raw, opal_convertor_raw.c:65-283).

The engine's ddt_convertor_raw walks its committed type map; the oracle (ort_raw) walks
the flat type map.  Both must give the same iovec lists for every position and iovec
budget.  The reference's own raw test (ddt_raw2.c) is replayed on its hand-written
description: 300, 10 and 1 iovecs per call give the same list, covering `size` bytes.
No data moves, so these run on CPU (the base address is never dereferenced).
"""
from __future__ import annotations

import json
import os
import random
import struct

import pytest

import ompi_amd
from ompi_amd import datatype as D
from tests import recipes as R

HERE = os.path.dirname(os.path.abspath(__file__))
BASE = 1 << 40


def engine_raw_all(dt, count, base, cap, position=0):
    c = ompi_amd.Convertor()
    c.prepare_for_raw(dt, count, base)
    if position:
        c.set_position(position)
    out, calls, total = [], 0, 0
    while True:
        rc, iovs, n = c.raw(cap)
        assert len(iovs) <= cap
        assert sum(ln for _, ln in iovs) == n
        out.append(iovs)
        total += n
        calls += 1
        if rc == 1:
            return out, total
        assert iovs, "no progress"
        assert calls < 10 ** 6


def stitched(chunks):
    """Concatenate per-call lists, merging a region split across two calls."""
    flat = []
    for ch in chunks:
        for a, n in ch:
            if flat and flat[-1][0] + flat[-1][1] == a:
                flat[-1] = (flat[-1][0], flat[-1][1] + n)
            else:
                flat.append((a, n))
    return flat


@pytest.mark.parametrize("seed", range(4))
def test_raw_matches_oracle_fuzz(seed):
    rng = random.Random(4100 + seed)
    for n in range(80):
        b = R.Built(R.random_recipe(rng))
        oi = b.o.info()
        count = rng.choice([1, 2, 5])
        total = oi["size"] * count
        e = b.engine()
        base = BASE + R.layout(oi, count)[1]
        full, got = b.o.raw(count, base, 0, 1 << 20)
        assert got == total
        for cap in (1, 2, 7, 1 << 20):
            chunks, tot = engine_raw_all(e, count, base, cap)
            assert tot == total, (b.recipe, cap)
            assert stitched(chunks) == full, (b.recipe, cap)
        if total == 0:
            continue
        # every call from a random position equals the oracle's call there
        c = ompi_amd.Convertor()
        c.prepare_for_raw(e, count, base)
        for _ in range(4):
            want = rng.randrange(total)
            cap = rng.choice([1, 3, 16])
            # a raw convertor is a send convertor (ddt_raw2.c:42): set_position lands on the
            # element boundary at or below the target (opal_convertor.c:458-470)
            pos = c.set_position(want)
            assert pos == b.o.set_position(count, want, send=True), (b.recipe, want, pos)
            rc, iovs, nb = c.raw(cap)
            ref, rb = b.o.raw(count, base, pos, cap)
            assert iovs == ref and nb == rb, (b.recipe, pos, cap)
            assert rc == (1 if pos + nb == total else 0)
            assert c.position == pos + nb


def test_raw_contiguous_is_one_iovec():
    dt = D.create_contiguous(1000, D.predefined(D.FLOAT8)).commit()
    chunks, tot = engine_raw_all(dt, 3, BASE, 4)
    assert chunks == [[(BASE, 24000)]] and tot == 24000


def test_raw_vector_regions():
    # vector(3, 2, 4) double (partial.c): blocks of 16 B every 32 B
    dt = D.create_vector(3, 2, 4, D.predefined(D.FLOAT8)).commit()
    chunks, _ = engine_raw_all(dt, 2, BASE, 100)
    ext = 2 * 32 + 16
    want = [(BASE + i * ext + k * 32, 16) for i in range(2) for k in range(3)]
    # instance 0's last block ends at 80 == instance 1's first block: merged
    want = stitched([want])
    assert chunks == [want]


def test_raw_completed_and_empty():
    c = ompi_amd.Convertor()
    dt = D.create_contiguous(0, D.predefined(D.INT4)).commit()
    c.prepare_for_raw(dt, 4, BASE)
    assert c.raw(8) == (1, [], 0)


def _opal_desc_bytes(rows):
    out = b""
    for kind, flags, typ, a, b_, c, d in rows:
        if kind == "elem":
            out += struct.pack("<HHIQqq", flags, typ, a, b_, c, d)
        else:  # loop: items, loops, unused, extent; end: items, unused, size, first_elem_disp
            out += struct.pack("<HHII4xQq", flags, typ, a, b_ & 0xFFFFFFFF, c & (2 ** 64 - 1), d)
    return out


def _walk_desc(rows, i, end, base, out):
    """Literal walk of an opal description (opal_convertor_raw.c:148-262): DATA blocks of
    blocklen elements every extent bytes; LOOP bodies repeated every loop extent."""
    size1 = {9: 1}
    while i < end:
        kind, flags, typ, a, b_, c, d = rows[i]
        if kind == "elem":
            for k in range(a):
                out.append((base + d + k * c, b_ * size1[typ]))
            i += 1
        else:
            items, loops, extent = a, b_, d
            for it in range(loops):
                _walk_desc(rows, i + 1, i + items, base + it * extent, out)
            i += items + 1


def test_raw_reference_ddt_raw2_description():
    """ddt_raw2.c:104-211 replayed: the reference's committed description, imported as-is,
    exported with 300, 10 and 1 iovecs per call."""
    fx = json.load(open(os.path.join(HERE, "golden", "ddt_raw2_desc.json")))
    rows, used, bd = fx["desc"], fx["used"], fx["bounds"]
    dt = D.from_opal_desc(_opal_desc_bytes(rows[:used]), bd["size"], bd["lb"], bd["ub"],
                          bd["true_lb"], bd["true_ub"])
    lists = {}
    for cap in (300, 10, 1):
        chunks, tot = engine_raw_all(dt, 1, BASE, cap)
        assert tot == bd["size"]
        lists[cap] = [iov for ch in chunks for iov in ch]
    assert lists[300] == lists[10] == lists[1]
    pieces = []
    _walk_desc(rows, 0, used, BASE, pieces)
    assert stitched([pieces]) == lists[300]
    assert sum(n for _, n in pieces) == bd["size"]


def test_reference_large_data_c():
    """large_data.c: raw export of multi-GiB types, 10 iovecs per call, never dereferenced.
    The bytes described must add up to the type size: indexed({192,192}, {576,0}) and
    indexed({192,192}, {192,384}) of contiguous(20 M, float) (30.72 GB each),
    vector(INT_MAX/2, 4, 4, float) and contiguous(INT_MAX/2, contiguous(4, float))
    (16 GiB each; large_data.c:96-172)."""
    f = D.MPI.MPI_FLOAT
    ddt = D.create_contiguous(20_000_000, f)
    big = 2 ** 31 - 1
    types = [D.create_indexed([192, 192], [3 * 192, 0], ddt),
             D.create_indexed([192, 192], [192, 2 * 192], ddt),
             D.create_vector(big // 2, 4, 4, f),
             D.create_contiguous(big // 2, D.create_contiguous(4, f))]
    for t in types:
        t.commit()
        chunks, total = engine_raw_all(t, 1, BASE, 10)
        assert total == t.size == sum(n for ch in chunks for _, n in ch)
    # the sparse index type is its two 15.36 GB blocks; the others one contiguous region
    assert stitched(engine_raw_all(types[0], 1, BASE, 10)[0]) == [
        (BASE + 3 * 192 * 80_000_000, 192 * 80_000_000), (BASE, 192 * 80_000_000)]
    assert stitched(engine_raw_all(types[2], 1, BASE, 10)[0]) == [(BASE, (big // 2) * 16)]


def test_imported_indexed_description_folds_to_one_list():
    """An indexed type imported from its committed opal description (the bridge's path,
    INTEGRATION.md §1).  The reference's optimizer leaves an indexed type as two-block DATA
    entries (opal_datatype_optimize.c:1179-1185: 32 M of them for BASELINE config 4); the
    import folds a long run into ONE index list (one plan leaf, so the address-ordered
    engine applies) with the same type map; a short run stays one DATA node per entry."""
    import numpy as np
    from tests import plan_emu as E
    rng = np.random.default_rng(8)
    for n, leaves, lists in ((4096, 1, 1), (20, 10, 0)):
        d = rng.permutation(4 * n)[:n].astype(np.int64)
        b = R.Built(("indexed_block", 1, d.tolist(), ("basic", 15)))
        info = b.o.info()
        rows = [("elem", 0x0100, 15, 2, 1, int(d[k + 1] - d[k]) * 4, int(d[k]) * 4) for k in range(0, n, 2)]
        e = D.from_opal_desc(_opal_desc_bytes(rows), info["size"], info["lb"], info["ub"],
                             info["true_lb"], info["true_ub"])
        pi = e.plan_info()
        assert (pi["leaves"], pi["list_leaves"]) == (leaves, lists), pi
        np.testing.assert_array_equal(E.engine_blocks(e), E.oracle_blocks(b.o))
        span, origin = R.layout(info, 1)
        user = R.fill(span, 3)
        UA, PA = 1 << 40, 1 << 41
        its = E.items(e, 1, UA + origin, PA, 0, info["size"])
        packed = np.zeros(info["size"], dtype=np.uint8)
        E.emulate(its, user, UA, packed, PA, 0, E.list_tables(e))
        ref = np.frombuffer(b.o.pack(1, user, origin, 0, info["size"], element_granular=False), dtype=np.uint8)
        np.testing.assert_array_equal(packed, ref)


def test_convertor_clone_need_buffers_pointers_cleanup():
    """opal_convertor_clone(_with_position), need_buffers, get_current/offset_pointer,
    get_unpacked_size and cleanup (opal_convertor.h:208-312, opal_convertor.c:708-756),
    exercised on raw-prepared convertors (no data moves)."""
    f = D.MPI.MPI_FLOAT
    contig = D.create_contiguous(16, f).commit()
    vec = D.create_vector(8, 1, 2, f).commit()
    # need_buffers: no gaps or one contiguous instance -> 0; a gapped vector -> 1
    c = ompi_amd.Convertor().prepare_for_raw(contig, 3, BASE)
    assert not c.need_buffers()
    v = ompi_amd.Convertor().prepare_for_raw(vec, 2, BASE)
    assert v.need_buffers()
    assert v.unpacked_size == v.packed_size == 2 * 8 * 4
    # pointers: base + position (+ true_lb)
    c.set_position(40)
    assert c.current_pointer() == BASE + 40 and c.offset_pointer(100) == BASE + 100
    # clone keeps the message, resets or keeps the position; clone_with_position repositions
    d = c.clone()
    assert d.packed_size == c.packed_size and d.current_pointer() == BASE
    e = c.clone(copy_stack=True)
    assert e.current_pointer() == BASE + 40
    g = v.clone(position=12)
    rc, iovs, n = g.raw(64)
    assert rc == 1 and n == 2 * 8 * 4 - 12
    assert iovs[0] == (BASE + 3 * 8, 4)   # element 3 of the stream at byte 24 of the vector
    # cleanup: completed, unprepared, reusable
    v.cleanup()
    assert v.completed
    v.prepare_for_raw(contig, 1, BASE)
    assert v.packed_size == 64 and not v.completed
