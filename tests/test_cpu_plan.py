"""CPU tests: engine type bounds and compiled plans against the oracle (no GPU needed).

The engine's launch descriptors are replayed by tests/plan_emu.py with the kernel's
index arithmetic, so plan compilation, window clipping and fragment splitting are
checked bit-exactly here; the kernels themselves are checked in test_gpu_parity.py.
"""
from __future__ import annotations

import random

import numpy as np
import pytest

from . import plan_emu as E
from . import recipes as R

BOUND_KEYS = ("size", "lb", "ub", "true_lb", "true_ub", "align")


@pytest.mark.parametrize("seed", range(4))
def test_bounds_match_oracle(seed):
    rng = random.Random(seed)
    for _ in range(400):
        r = R.random_recipe(rng)
        b = R.Built(r)
        oi, ei = b.o.info(), b.engine().info()
        for k in BOUND_KEYS:
            assert oi[k] == ei[k], (k, oi, ei, r)
        assert (oi["flags"] & 0x1F0) == (ei["flags"] & 0x1F0), (hex(oi["flags"]), hex(ei["flags"]), r)


def _check_windows(b, rng, n_windows=3, seed=0):
    oi = b.o.info()
    if oi["size"] == 0:
        return
    e = b.engine()
    count = rng.choice([1, 2, 3, 7])
    span, origin = R.layout(oi, count)
    user = R.fill(span, seed)
    total = count * oi["size"]
    wins = [(0, total)]
    for _ in range(n_windows):
        a = rng.randint(0, total - 1)
        wins.append((a, rng.randint(a + 1, total)))
    lists = E.list_tables(e)
    for w0, w1 in wins:
        UA = (1 << 40) + 4096 * rng.randint(0, 3)
        PA = (1 << 41) + rng.choice([0, 4, 1, 64])
        its = E.items(e, count, UA + origin, PA, w0, w1)
        packed = np.zeros(w1 - w0, dtype=np.uint8)
        cov = E.emulate(its, user, UA, packed, PA, 0, lists)
        ref = np.frombuffer(b.o.pack(count, user, origin, w0, w1 - w0, element_granular=False),
                            dtype=np.uint8)
        assert np.all(cov == 1), (b.recipe, w0, w1)
        np.testing.assert_array_equal(packed, ref)
        dst = np.full(span, 0xA5, dtype=np.uint8)
        dref = dst.copy()
        E.emulate(its, dst, UA, packed, PA, 1, lists)
        b.o.unpack(count, dref, origin, w0, ref.tobytes())
        np.testing.assert_array_equal(dst, dref)


@pytest.mark.parametrize("seed", range(6))
def test_plan_blocks_and_items_match_oracle(seed):
    rng = random.Random(100 + seed)
    for n in range(120):
        b = R.Built(R.random_recipe(rng))
        if b.o.info()["size"] == 0:
            continue
        eb = E.engine_blocks(b.engine())
        ob = E.oracle_blocks(b.o)
        np.testing.assert_array_equal(eb, ob, err_msg=str(b.recipe))
        _check_windows(b, rng, seed=n)


def test_struct_in_hvector_merges_to_one_leaf():
    """cfg5: struct{double,int[3]} in hvector(.., 32 B) compiles to ONE 20-byte leaf
    (the reference's opt_desc is UINT4 count N blen 5 extent 32)."""
    st = ("struct", [1, 3], [0, 8], [("basic", 16), ("basic", 6)])
    b = R.Built(("hvector", 1000, 1, 32, st))
    lv = E.leaves(b.engine())
    assert len(lv) == 1 and lv[0]["blen"] == 20 and lv[0]["dims"] == [(1000, 32, 20)]
    oi = b.o.info()
    assert oi["size"] == 20000


def test_vector_faces_compile_to_single_affine_leaf():
    # 256^3 double x-face / y-face
    x = R.Built(("vector", 65536, 1, 256, ("basic", 16)))
    y = R.Built(("vector", 256, 256, 65536, ("basic", 16)))
    lx, ly = E.leaves(x.engine()), E.leaves(y.engine())
    assert lx == [dict(kind=0, blen=8, src=0, dst=0, dims=[(65536, 2048, 8)], index=0)]
    assert ly == [dict(kind=0, blen=2048, src=0, dst=0, dims=[(256, 524288, 2048)], index=0)]
    assert x.o.info()["size"] == 524288 and x.o.extent == 134215688
    assert y.o.extent == 133695488


def test_subarray_face_dim2_disp():
    """512^3 float subarray thin in dim 2 at start 511: true_lb 2044."""
    b = R.Built(("subarray", [512, 512, 512], [512, 512, 1], [0, 0, 511], 0, ("basic", 15)))
    oi, ei = b.o.info(), b.engine().info()
    assert oi["true_lb"] == ei["true_lb"] == 2044
    assert oi["ub"] - oi["lb"] == 536870912 == ei["ub"] - ei["lb"]
    lv = E.leaves(b.engine())
    assert len(lv) == 1 and lv[0]["src"] == 2044 and lv[0]["blen"] == 4


def test_extent_minus_one_quirk():
    """opal_datatype_add treats extent -1 as 'default extent' (opal_datatype_add.c:156-161):
    vector(4,3,-1,char) therefore packs like contiguous(12)."""
    b = R.Built(("vector", 4, 3, -1, ("basic", 4)))
    assert b.o.info()["lb"] == 0 and b.engine().info()["lb"] == 0
    assert b.engine().info()["ub"] == 12


@pytest.mark.parametrize("seed", range(3))
def test_typed_copy_items_match_oracle(seed):
    """Same-layout descriptors (opal_datatype_copy_content_same_ddt) move every byte of
    the type map once, from the source layout to the same offsets of the destination."""
    rng = random.Random(500 + seed)
    for n in range(80):
        b = R.Built(R.random_recipe(rng))
        oi = b.o.info()
        if oi["size"] == 0:
            continue
        count = rng.choice([1, 2, 5])
        span, origin = R.layout(oi, count)
        src = R.fill(span, n)
        dst = np.full(span, 0xA5, dtype=np.uint8)
        UA, PA = (1 << 40), (1 << 41)
        its = E.items(b.engine(), count, UA + origin, PA + origin, 0, oi["size"] * count,
                      same_layout=True)
        for it in its:
            if it.kind == E.ITEM_AFFINE:
                tot = it.upb
                for j in range(it.ndim):
                    tot *= it.cnt[j]
                assert it.u1 <= tot
        E.emulate(its, src, UA, dst, PA, 0, E.list_tables(b.engine()))
        exp = np.full(span, 0xA5, dtype=np.uint8)
        stream = b.o.pack(count, src, origin, 0, oi["size"] * count, element_granular=False)
        b.o.unpack(count, exp, origin, 0, stream)
        if not _overlap(b.o, count):
            np.testing.assert_array_equal(dst, exp, err_msg=str(b.recipe))


def _overlap(o, count):
    info = o.info()
    ext = info["ub"] - info["lb"]
    seen = set()
    for i in range(count):
        for d, n, _ in o.runs():
            for x in range(d + i * ext, d + i * ext + n):
                if x in seen:
                    return True
                seen.add(x)
    return False


@pytest.mark.parametrize("chunk", [1, 3])
def test_interleaved_task_order_matches_oracle(chunk):
    """ddt_tune("interleave") splits items into task runs and reorders them; every byte
    must still move exactly once to the oracle's packed position."""
    from ompi_amd import lib
    L = lib()
    L.ddt_tune(b"interleave", chunk)
    L.ddt_tune(b"task_kb", 1)
    try:
        rng = random.Random(900 + chunk)
        for n in range(60):
            b = R.Built(R.random_recipe(rng))
            if b.o.info()["size"] == 0:
                continue
            _check_windows(b, rng, seed=n)
    finally:
        L.ddt_tune(b"interleave", 0)
        L.ddt_tune(b"task_kb", 0)


def test_stream_policy_of_mixed_launches():
    """ddt_plan.cpp:stream_policy: the halo's streaming faces (y, z: U = 16, nt 3 = non-temporal
    loads) turn fully non-temporal (nt 2) beside isolated narrow blocks (the x faces, wt 3) only
    when those blocks' lines overflow the L2s (32 MiB: 2 fields of x lines fill it exactly);
    streams alone keep nt 3 at any size; snt -3 switches the rule off."""
    import bench
    from ompi_amd import lib
    from ompi_amd import recipe as ER
    halo, _ = bench.halo_recipe()
    faces = bench.face_recipes()

    def nts(recipe, count):
        t = ER.build_committed(recipe)
        its = E.items(t, count, 0, 0, 0, t.info()["size"] * count)
        return ({it.nt for it in its if it.kind == E.ITEM_AFFINE and it.U == 16},
                {it.wt for it in its if it.kind == E.ITEM_AFFINE and it.U == 8})

    assert nts(halo, 16) == ({2}, {3})
    assert nts(halo, 3) == ({2}, {3})
    assert nts(halo, 2) == ({3}, {3})
    assert nts(halo, 1) == ({3}, {3})
    assert nts(faces["y"], 64)[0] == {3} and nts(faces["z"], 64)[0] == {3}
    L = lib()
    L.ddt_tune(b"snt", -3)
    try:
        assert nts(halo, 16)[0] == {3}
    finally:
        L.ddt_tune(b"snt", -1)


def test_reference_resized_extent_bounds():
    """resized_extent.c:148-163 known answers, engine and oracle: resized(int, 0, 6) has
    lb 0 / extent 6 / true_lb 0 / true_extent 4; contiguous(3, it) keeps extent 18 (not the
    alignment-rounded 20) with true_extent 16; its packed stream picks the ints at 0, 6, 12."""
    for rec, want in ((("resized", ("basic", 6), 0, 6), (0, 6, 0, 4)),
                      (("contig", 3, ("resized", ("basic", 6), 0, 6)), (0, 18, 0, 16))):
        b = R.Built(rec)
        for i in (b.o.info(), b.engine().info()):
            assert (i["lb"], i["ub"] - i["lb"], i["true_lb"], i["true_ub"] - i["true_lb"]) == want
    b = R.Built(("contig", 3, ("resized", ("basic", 6), 0, 6)))
    user = np.arange(48, dtype=np.uint8)
    got = np.frombuffer(b.o.pack(2, user, 0, 0, 24, element_granular=True), dtype=np.uint8)
    want = np.concatenate([user[p:p + 4] for p in range(0, 36, 6)])
    np.testing.assert_array_equal(got, want)


def _oracle_get_elements(o, ucount):
    """ompi_datatype_get_elements restated on the oracle's type map (runs of whole basic
    elements of one size, in type-map order): whole instances count every element; the
    leftover walks the runs and is MPI_UNDEFINED (None) if it ends inside an element."""
    info = o.info()
    size = info["size"]
    if size == 0:
        return 0
    runs = o.runs()
    per = sum(n // e for _, n, e in runs)
    full, left = divmod(ucount, size)
    acc = full * per
    if left:
        for _, n, e in runs:
            if n >= left:
                return acc + left // e if left % e == 0 else None
            acc += n // e
            left -= n
    return acc


@pytest.mark.parametrize("seed", range(3))
def test_get_elements_matches_oracle(seed):
    """MPI_Get_elements (ompi_datatype_get_elements.c:30-76 with opal_datatype_get_count.c:32-92)
    on fuzzed types and byte counts, against the oracle's type map."""
    rng = random.Random(700 + seed)
    for _ in range(150):
        b = R.Built(R.random_recipe(rng))
        size = b.o.info()["size"]
        e = b.engine()
        for uc in {0, size, 3 * size, rng.randrange(0, 4 * size + 9), rng.randrange(0, size + 1) + size}:
            assert e.get_elements(uc) == _oracle_get_elements(b.o, uc), (b.recipe, uc)


def test_get_elements_known_answers():
    from ompi_amd import datatype as D
    st = D.create_struct([1, 3], [0, 8], [D.MPI.MPI_DOUBLE, D.MPI.MPI_INT]).commit()   # size 20
    assert st.get_elements(60) == 12 and st.get_elements(68) == 13 and st.get_elements(70) is None
    v = D.create_vector(3, 2, 4, D.MPI.MPI_DOUBLE).commit()                              # size 48
    assert v.get_elements(24) == 3 and v.get_elements(48 * 5) == 30 and v.get_elements(20) is None
    assert D.MPI.MPI_INT.get_elements(12) == 3 and D.MPI.MPI_INT.get_elements(6) is None


def test_opal_ddt_api_known_answers():
    """test/datatype/opal_ddt_api.c: get_element_count on a vector of 3 blocks of 4 ints at a
    stride of 6 (:233-260: the whole 48 bytes hold 12 elements, 4 bytes 1, 16 bytes 4), and the
    bounds of its two backward constructions (:162-218: a vector of 3 ints at a stride of -2
    spans true_lb -16 .. true_ub 4; ints added at 4 then 0 span 0 .. 8)."""
    from ompi_amd import datatype as D
    v = D.create_vector(3, 4, 6, D.MPI.MPI_INT).commit()
    assert v.size == 48
    assert v.get_elements(48) == 12 and v.get_elements(4) == 1 and v.get_elements(16) == 4
    neg = D.create_vector(3, 1, -2, D.MPI.MPI_INT).commit()
    i = neg.info()
    assert (i["true_lb"], i["true_ub"]) == (-16, 4)
    back = D.create_struct([1, 1], [4, 0], [D.MPI.MPI_INT, D.MPI.MPI_INT]).commit()
    i = back.info()
    assert (i["true_lb"], i["true_ub"]) == (0, 8)


def test_opal_bigcount_large_contiguous():
    """test/datatype/opal_datatype_bigcount.c:141-197: a contiguous run of INT_MAX + 1000 and of
    3 x INT_MAX bytes has that size and extent (64-bit arithmetic, no truncation at 2^31 or
    2^32); metadata only, no buffer.  The plan of the larger one is one leaf of 64-bit units."""
    from ompi_amd import datatype as D
    INT_MAX = 2**31 - 1
    for n in (INT_MAX + 1000, 3 * INT_MAX):
        t = D.create_contiguous(n, D.MPI.MPI_BYTE).commit()
        i = t.info()
        assert t.size == n and i["ub"] - i["lb"] == n and (i["true_lb"], i["true_ub"]) == (0, n)
        assert t.get_elements(n) == n
    assert t.plan_info()["leaves"] == 1


def test_sparse_only_launch_task_floor():
    """ddt_plan.cpp:assign_tasks: a launch of sparse gathers alone with fewer tasks than CUs (a single-field x face,
    one 8-B element per line) takes four units per lane per task (1024 units); beside streams
    (the single-field halo) its x leaves keep two (512); ddt_tune("sfloor", -1) switches it off
    (profiles/r5_b2b_x_tasks.jsonl)."""
    import bench
    from ompi_amd import lib
    from ompi_amd import recipe as ER
    L = lib()
    x = ER.build_committed(bench.face_recipes()["x"])
    halo = ER.build_committed(bench.halo_recipe()[0])

    def upt(t, count):
        its = E.items(t, count, 0, 0, 0, t.info()["size"] * count)
        return {int(it.units_per_task) for it in its if it.kind == E.ITEM_AFFINE and it.U == 8}

    try:
        assert upt(x, 1) == {1024}
        assert upt(halo, 1) == {512}
        L.ddt_tune(b"sfloor", -1)
        assert upt(x, 1) == {512}
    finally:
        L.ddt_tune(b"reset", 0)
