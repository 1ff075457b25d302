"""The opal fAdvance bridge on CPU: layout of Open MPI's objects, attach semantics of the
post-prepare hook, and the per-datatype import cache (no data moves without a GPU)."""
from __future__ import annotations

import ctypes

import pytest

from tests import opal_shapes as S
from tests import recipes as R

FLOAT8, FLOAT4, INT4, UINT4 = 16, 15, 6, 11


def _xface(n=16):
    """Appendix A shape of a 3D-vector x face: FLOAT8 count n*n blen 1 extent 8n."""
    ents = [S.data(FLOAT8, n * n, 1, 8 * n, 0)]
    size = 8 * n * n
    ub = (n * n - 1) * 8 * n + 8
    return S.OpalType(ents, size, 0, ub, 0, ub)


def test_layout_matches_compiled_bridge():
    compiled, mine = S.check_layout()
    assert compiled == mine
    # the layout notes of the reference headers (opal_datatype.h:204-211, opal_convertor.h:136,149)
    assert compiled[0] == 200 and compiled[3] == 64 and S.OpalConvertor.sizes.offset == 128


def test_attach_installs_movers_on_accelerator_convertors():
    L = S.bridge_lib()
    t = _xface()
    c = S.Convertor()
    assert c.prepare(t, 3, 0x7000_0000_0000, send=True) == S.OPAL_SUCCESS
    assert c.c.fAdvance == ctypes.cast(L.opal_pack_hip, ctypes.c_void_p).value
    assert c.c.fPosition == ctypes.cast(L.opal_position_hip, ctypes.c_void_p).value
    assert c.c.local_size == 3 * t.dt.size and not (c.c.flags & S.CONVERTOR_NO_OP)
    r = S.Convertor()
    assert r.prepare(t, 1, 0x7000_0000_0000, send=False) == S.OPAL_SUCCESS
    assert r.c.fAdvance == ctypes.cast(L.opal_unpack_hip, ctypes.c_void_p).value
    # a host buffer (check_addr == 0) keeps the reference movers: the bridge declines
    h = S.Convertor()
    assert h.prepare(t, 1, 0x1000, send=True, device=False) == S.OPAL_ERR_NOT_SUPPORTED
    assert not h.c.fAdvance
    t.destruct()


def test_position_function_resumes_at_byte_offset():
    t = _xface()
    c = S.Convertor()
    c.prepare(t, 2, 0x7000_0000_0000, send=False)
    assert c.set_position(777) == 777
    assert c.c.bConverted == 777 and not (c.c.flags & S.CONVERTOR_COMPLETED)
    assert c.set_position(10 ** 9) == 2 * t.dt.size   # clamped, completed (opal_convertor.h:372-377)
    assert c.c.flags & S.CONVERTOR_COMPLETED
    t.destruct()


def test_import_cache_hits_invalidation_and_stale_addresses():
    S.bridge_lib().opal_hip_bridge_finalize()
    base = S.stats()
    t = _xface()
    for _ in range(4):
        S.Convertor().prepare(t, 1, 0x7000_0000_0000, send=True)
    st = S.stats()
    assert st["imports"] - base["imports"] == 1 and st["hits"] - base["hits"] >= 3
    assert st["entries"] == 1
    # opal_datatype_destruct drops the entry; the next prepare imports again
    t.destruct()
    assert S.stats()["entries"] == 0
    S.Convertor().prepare(t, 1, 0x7000_0000_0000, send=True)
    assert S.stats()["imports"] - base["imports"] == 2
    # a different description at the same opal_datatype_t address (destruct never called):
    # the fingerprint notices and re-imports instead of serving the old plan
    raw2 = t.raw.copy()
    t.raw = raw2
    t.dt.opt_desc.desc = raw2.ctypes.data
    S.Convertor().prepare(t, 1, 0x7000_0000_0000, send=True)
    st = S.stats()
    assert st["stale"] - base["stale"] == 1 and st["entries"] == 1
    S.bridge_lib().opal_hip_bridge_finalize()
    assert S.stats()["entries"] == 0


def test_commit_hook_imports_large_descriptions_at_commit():
    """opal_hip_bridge_datatype_commit (called at the end of opal_datatype_commit): a
    description of >= 64 Ki opt_desc entries is imported there, so the first prepare of a
    message only hits the cache; a small one is left to its first prepare."""
    L = S.bridge_lib()
    L.opal_hip_bridge_finalize()
    base = S.stats()
    n = 70000
    big = S.OpalType([S.data(FLOAT8, 1, 1, 8, 24 * i) for i in range(n)], 8 * n, 0, 24 * n, 0,
                     24 * (n - 1) + 8)
    assert big.commit_hook() == S.OPAL_SUCCESS
    st = S.stats()
    assert st["imports"] - base["imports"] == 1 and st["entries"] == 1
    assert S.Convertor().prepare(big, 2, 0x7000_0000_0000, send=True) == S.OPAL_SUCCESS
    st2 = S.stats()
    assert st2["imports"] == st["imports"] and st2["hits"] - st["hits"] == 1
    assert big.commit_hook() == S.OPAL_SUCCESS and S.stats()["imports"] == st["imports"]   # idempotent
    small = _xface()
    assert small.commit_hook() == S.OPAL_SUCCESS
    assert S.stats()["imports"] == st["imports"] and S.stats()["entries"] == 1
    big.destruct()
    small.destruct()
    assert S.stats()["entries"] == 0


def test_no_op_and_empty_convertors_skip_the_bridge():
    """OPAL_CONVERTOR_PREPARE returns before dispatch for NO_GAPS types (opal_convertor.c:
    562-567) and empty messages (:539-544): opal_convertor_pack copies those itself."""
    contig = S.OpalType([S.data(FLOAT8, 1, 64, 512, 0)], 512, 0, 512, 0, 512,
                        flags=S.F_CONTIGUOUS | S.F_NO_GAPS)
    c = S.Convertor()
    c.prepare(contig, 4, 0x7000_0000_0000, send=True)
    assert c.c.flags & S.CONVERTOR_NO_OP and not c.c.fAdvance
    e = S.Convertor()
    e.prepare(_xface(), 0, 0x7000_0000_0000, send=True)
    assert e.c.flags & S.CONVERTOR_COMPLETED and e.c.local_size == 0


@pytest.mark.parametrize("case", ["end_missing", "end_items", "end_size", "past_used"])
def test_malformed_descriptions_are_refused(case):
    """The import validates LOOP/END_LOOP pairing (CREATE_LOOP_START/END,
    opal_datatype_internal.h:171-189) before anything reads past the description."""
    body = S.data(FLOAT4, 4, 1, 8, 0)
    if case == "end_missing":
        ents = [S.loop(3, 2, 64), body, S.data(FLOAT4, 1, 1, 4, 40)]
    elif case == "end_items":
        ents = [S.loop(3, 2, 64), body, S.end_loop(3, 16, 0)]
    elif case == "end_size":
        ents = [S.loop(3, 2, 64), body, S.end_loop(2, 20, 0)]
    else:
        ents = [S.loop(3, 4, 64), body, S.end_loop(2, 16, 0)]
    t = S.OpalType(ents, 48, 0, 64 * 2 + 28, 0, 64 * 2 + 28)
    c = S.Convertor()
    assert c.prepare(t, 1, 0x7000_0000_0000, send=True) == -5   # OPAL_ERR_BAD_PARAM
    ok = S.OpalType([S.loop(3, 2, 64), body, S.end_loop(2, 16, 0)], 48, 0, 64 * 2 + 28, 0, 64 * 2 + 28)
    assert S.Convertor().prepare(ok, 1, 0x7000_0000_0000, send=True) == S.OPAL_SUCCESS
    ok.destruct()


def test_flat_descriptions_of_corpus_types_import():
    from tests import corpus
    for name in sorted(corpus.CORPUS):
        rec, _ = corpus.CORPUS[name]()
        b = R.Built(rec)
        t = S.flat_from_oracle(b.o)
        c = S.Convertor()
        rc = c.prepare(t, 2, 0x7000_0000_0000, send=True)
        assert rc == S.OPAL_SUCCESS, name
        t.destruct()


def test_exported_descriptions_round_trip():
    """ddt_type_to_opal_desc writes the uncommitted type map as dt_elem_desc_t entries
    (LOOP/END_LOOP pairs as CREATE_LOOP_START/END make them); importing that description
    gives the same type map as the oracle on 600 random recipes (every constructor, nesting
    depth 3, negative strides, resized bounds)."""
    import random
    import numpy as np
    from ompi_amd import datatype as D
    from tests import plan_emu as E
    rng = random.Random(2024)
    loops = 0
    for _ in range(600):
        rec = R.random_recipe(rng)
        b = R.Built(rec)
        info = b.o.info()
        if info["size"] == 0:
            continue
        desc = b.engine().to_opal_desc()
        loops += any(desc[32 * i + 2] == 0 and desc[32 * i + 3] == 0 for i in range(len(desc) // 32))
        t = D.from_opal_desc(desc, info["size"], info["lb"], info["ub"], info["true_lb"], info["true_ub"])
        np.testing.assert_array_equal(E.engine_blocks(t), E.oracle_blocks(b.o))
    assert loops > 50


@pytest.mark.parametrize("seed", range(6))
def test_streamed_import_of_folded_runs(seed):
    """ddt_type_from_opal_desc streams runs of small DATA entries into one index list: runs
    around the 64-entry fold threshold, block lengths that start to differ after the list has
    begun (the lengths array is materialised mid-run), a type change that starts a new list,
    short runs kept as DATA entries and non-foldable entries between them.  The imported type
    map must be the description's blocks in order."""
    import random
    import numpy as np
    from ompi_amd import datatype as D
    from tests import plan_emu as E
    rng = random.Random(900 + seed)
    sizes = {FLOAT4: 4, FLOAT8: 8, INT4: 4}
    ents, blocks, pos = [], [], 0
    for _ in range(rng.randint(3, 6)):
        tid = rng.choice([FLOAT4, FLOAT8, INT4])
        esz = sizes[tid]
        n = rng.choice([1, 20, 63, 64, 65, 130, 300])
        change_at = rng.choice([None, 0, 1, n // 2, n - 1])
        for i in range(n):
            count = rng.randint(1, 16) if rng.random() < 0.97 else rng.randint(17, 40)   # > 16: not foldable
            blen = 1 if change_at is None or i < change_at else rng.randint(1, 3)
            extent = esz * rng.randint(blen + 1, blen + 5)
            disp = pos
            ents.append(S.data(tid, count, blen, extent, disp))
            for k in range(count):
                blocks.append((disp + k * extent, blen * esz))
            pos = disp + count * extent + esz * rng.randint(0, 3)
    size = sum(b[1] for b in blocks)
    desc = b"".join(ents)
    t = D.from_opal_desc(desc, size, 0, pos, 0, pos)
    want, p = [], 0
    for d, ln in blocks:
        want.append((d, p, ln))
        p += ln
    np.testing.assert_array_equal(E.engine_blocks(t), E.merge_runs(np.array(want, dtype=np.int64)))


def test_streamed_import_materialises_lengths_mid_run():
    """130 one-type entries whose block length changes at entry 100 (after the list began at
    entry 64): one list leaf with per-block lengths, blocks in description order."""
    import numpy as np
    from ompi_amd import datatype as D
    from tests import plan_emu as E
    ents, blocks, pos = [], [], 0
    for i in range(130):
        blen = 1 if i < 100 else 2
        ents.append(S.data(FLOAT4, 2, blen, 16, pos))
        blocks += [(pos, 4 * blen), (pos + 16, 4 * blen)]
        pos += 40
    size = sum(b[1] for b in blocks)
    t = D.from_opal_desc(b"".join(ents), size, 0, pos, 0, pos)
    lv = E.leaves(t)
    assert len(lv) == 1 and lv[0]["kind"] != 0
    _, ln = E.plan_list(t, lv[0]["index"])
    assert list(ln) == [4] * 200 + [8] * 60
    want, p = [], 0
    for d, n in blocks:
        want.append((d, p, n))
        p += n
    np.testing.assert_array_equal(E.engine_blocks(t), E.merge_runs(np.array(want, dtype=np.int64)))


def test_import_cache_under_concurrent_threads():
    """One thread per convertor is the reference's contract, but many threads share the
    datatypes: eight threads attach convertors to the same six descriptions at once (ctypes
    releases the GIL inside the calls).  Each description is imported exactly once and
    every later attach hits the cache."""
    import threading
    L = S.bridge_lib()
    L.opal_hip_bridge_finalize()
    base = S.stats()
    types = [_xface(n) for n in (8, 12, 16, 20, 24, 28)]
    errors = []

    def worker(k):
        try:
            for i in range(60):
                t = types[(k + i) % len(types)]
                rc = S.Convertor().prepare(t, 1 + i % 3, 0x7000_0000_0000, send=bool(i % 2))
                assert rc == S.OPAL_SUCCESS
        except Exception as ex:   # noqa: BLE001 - reported below
            errors.append(repr(ex))

    ths = [threading.Thread(target=worker, args=(k,)) for k in range(8)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    assert not errors, errors
    st = S.stats()
    assert st["imports"] - base["imports"] == len(types)
    assert st["hits"] - base["hits"] == 8 * 60 - len(types)
    assert st["entries"] == len(types)
    for t in types:
        t.destruct()
    assert S.stats()["entries"] == 0


def test_import_cache_under_threads_with_destructs():
    """MPI_THREAD_MULTIPLE on the import cache (r6: per-bucket spin locks, per-thread pinned
    entries): eight threads attach convertors of their own datatype and of one shared datatype
    while a ninth destructs and re-creates types; every attach succeeds, and once the threads
    are done and the cache finalized no entry is left and every lookup was counted as an import
    or a hit."""
    import threading
    L = S.bridge_lib()
    L.opal_hip_bridge_finalize()
    base = S.stats()
    shared = _xface()
    own = [_xface(8 + i) for i in range(8)]
    errors, calls = [], [0] * 8
    stop = threading.Event()

    def worker(i):
        try:
            for k in range(400):
                t = shared if k % 2 else own[i]
                rc = S.Convertor().prepare(t, 1 + k % 3, 0x7000_0000_0000, send=bool(k % 4 < 2))
                if rc != S.OPAL_SUCCESS:
                    errors.append((i, k, rc))
                    return
                calls[i] += 1
        except Exception as ex:   # surface to the main thread
            errors.append(repr(ex))

    def churn():
        while not stop.is_set():
            t = _xface(5)
            S.Convertor().prepare(t, 1, 0x7000_0000_0000, send=True)
            t.destruct()

    th = [threading.Thread(target=worker, args=(i,)) for i in range(8)]
    ch = threading.Thread(target=churn)
    ch.start()
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    stop.set()
    ch.join(timeout=60)
    assert not errors, errors
    assert sum(calls) == 8 * 400
    st = S.stats()
    # each attach is one lookup: served by an import or a hit (shared or pinned)
    assert (st["imports"] - base["imports"]) + (st["hits"] - base["hits"]) >= 8 * 400
    for t in own + [shared]:
        t.destruct()
    L.opal_hip_bridge_finalize()
    assert S.stats()["entries"] == 0
