"""The drop-in boundary on the GPU: opal-shaped convertors (tests/opal_shapes.py builds
opal_datatype_t / opal_convertor_t as Open MPI lays them out and prepares them the way
opal_convertor_prepare_for_{send,recv} does) whose fAdvance / fPosition were swapped for
the bridge after prepare, as pack_description_sweep.c:877-965 swaps the reference's
movers.  Every byte is checked against the reference's known answers (golden digests of
the corpus by-hand packers, unpack_ooo.c's expected struct contents, ddt_raw2.c's
description walked literally) or the CPU oracle.
"""
from __future__ import annotations

import hashlib
import json
import os
import random
import struct

import numpy as np
import pytest

from . import corpus
from . import opal_shapes as S
from . import oracle as O
from . import recipes as R

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = json.load(open(os.path.join(HERE, "golden", "corpus_sha256.json")))
FLOAT8, FLOAT4, INT4, UINT4 = 16, 15, 6, 11


def _dev(arr, device):
    import torch
    return torch.from_numpy(np.ascontiguousarray(arr)).to(device)


def _host(t):
    import torch
    torch.cuda.synchronize()
    return t.cpu().numpy()


def _pack_fragments(conv, base, size, frag, expect=None, limit=None):
    """opal_convertor_pack in fragments of `frag` bytes (ob1's prepare_src loop,
    btl_sm_module.c:450-473); past `limit` bytes the rest goes in one call.  Returns the
    (position, bytes) windows."""
    pos, rc, wins = 0, 0, []
    while rc == 0:
        cap = min(frag if limit is None or pos < limit else size, size - pos)
        rc, iovs, md = conv.pack([(base + pos, cap)])
        assert rc >= 0
        if expect is not None:
            assert md == expect(pos, cap), (pos, cap, md)
        if md == 0:   # a predefined element larger than the fragment
            rc, iovs, md = conv.pack([(base + pos, size - pos)])
        wins.append((pos, md))
        pos += md
    assert pos == size and rc == 1
    return wins


def _unpack_windows(conv, base, wins, rng):
    """Out-of-order fragments: set_position then unpack (MCA_PML_OB1_RECV_REQUEST_UNPACK,
    pml_ob1_recvreq.h:275-310)."""
    order = list(wins)
    rng.shuffle(order)
    for pos, n in order:
        assert conv.set_position(pos) == pos
        rc, iovs, md = conv.unpack([(base + pos, n)])
        assert rc >= 0 and md == n


def _overlaps(runs, count, ext):
    seen = set()
    for i in range(count):
        for d, n, *_ in runs:
            for b in range(d + i * ext, d + i * ext + n):
                if b in seen:
                    return True
                seen.add(b)
    return False


# ------------------------------------------------------------------ the reference corpus
@pytest.mark.parametrize("name", sorted(corpus.CORPUS))
def test_bridge_corpus_fragments_vs_golden(device, name):
    """Every corpus type (datatype_corpus.c:2143-2236) through the bridge, whole and in the
    opt_desc_equiv.c:63 fragment matrix: the packed stream's SHA-256 is the by-hand packer's,
    per-fragment max_data is the oracle's element-granular answer, and shuffled unpack
    windows rebuild the oracle's user buffer."""
    import torch
    rec, _ = corpus.CORPUS[name]()
    b = R.Built(rec)
    g = GOLD[name]
    info = b.o.info()
    count = g["count"]
    size = info["size"] * count
    span, origin = R.layout(info, count)
    host = R.fill(span, 0x5A)
    user = _dev(host, device)
    ot = S.from_oracle(b.o)
    packed = torch.zeros(max(size, 1), dtype=torch.uint8, device=device)
    ref = np.frombuffer(b.o.pack(count, host, origin, 0, size, element_granular=False), dtype=np.uint8)
    rng = random.Random(name)
    for frag in (12, 16, 40, 4096, size):
        packed.zero_()
        conv = S.Convertor()
        assert conv.prepare(ot, count, user.data_ptr() + origin, send=True) == S.OPAL_SUCCESS
        exp = (lambda p, c: len(b.o.pack(count, host, origin, p, c, element_granular=True)))
        wins = _pack_fragments(conv, packed.data_ptr(), size, frag,
                               None if conv.c.flags & S.CONVERTOR_NO_OP else exp, limit=8 << 10)
        got = _host(packed)[:size]
        assert hashlib.sha256(got.tobytes()).hexdigest() == g["sha256"], (name, frag)
        np.testing.assert_array_equal(got, ref)
        if _overlaps(b.o.runs(), count, info["ub"] - info["lb"]):
            continue
        out = torch.full((span,), 0xA5, dtype=torch.uint8, device=device)
        cu = S.Convertor()
        cu.prepare(ot, count, out.data_ptr() + origin, send=False)
        _unpack_windows(cu, packed.data_ptr(), wins, rng)
        want = np.full(span, 0xA5, dtype=np.uint8)
        b.o.unpack(count, want, origin, 0, ref.tobytes())
        np.testing.assert_array_equal(_host(out), want)
    ot.destruct()


# ------------------------------------------------------------------ BASELINE shapes
def _halo_desc(n=256):
    """The 6-face halo of an n^3 double field as its committed description: one DATA entry
    per face, in the forms SURVEY.md Appendix A records from the reference's optimizer
    (x: FLOAT8 count n*n blen 1 extent 8n; y: FLOAT8 count n blen n extent 8n*n; z: a
    contiguous plane, CREATE_ELEM-collapsed to count 1), resized to the field."""
    row, plane, field = 8 * n, 8 * n * n, 8 * n * n * n
    ents = [S.data(FLOAT8, n * n, 1, row, 0), S.data(FLOAT8, n * n, 1, row, row - 8),
            S.data(FLOAT8, n, n, plane, 0), S.data(FLOAT8, n, n, plane, (n - 1) * row),
            S.data(FLOAT8, 1, n * n, plane, 0), S.data(FLOAT8, 1, n * n, plane, (n - 1) * plane)]
    return S.OpalType(ents, 6 * 8 * n * n, 0, field, 0, field)


def test_bridge_halo_cfg2_fragments_and_ooo(device):
    """BASELINE config 2's message (2 fields here) through the bridge: 1 MiB fragments
    packed in order, unpacked out of order at windows cut mid-element, against the oracle
    of the bench's own recipe (bench.halo_recipe)."""
    import torch
    import bench
    rec, field = bench.halo_recipe()
    b = R.Built(rec)
    count = 2
    info = b.o.info()
    size = info["size"] * count
    span, origin = R.layout(info, count)
    assert origin == 0
    host = R.fill_fast(span, 7)
    user = _dev(host, device)
    ot = _halo_desc()
    assert (ot.dt.size, ot.extent) == (info["size"], info["ub"] - info["lb"])
    packed = torch.zeros(size, dtype=torch.uint8, device=device)
    conv = S.Convertor()
    assert conv.prepare(ot, count, user.data_ptr(), send=True) == S.OPAL_SUCCESS
    wins = _pack_fragments(conv, packed.data_ptr(), size, 1 << 20)
    ref = np.frombuffer(b.o.pack(count, host, 0, 0, size, element_granular=False), dtype=np.uint8)
    np.testing.assert_array_equal(_host(packed), ref)
    # unpack windows of 1 MiB + 3 bytes: every cut lands inside a double
    cuts = list(range(0, size, (1 << 20) + 3)) + [size]
    wins = [(a, c - a) for a, c in zip(cuts, cuts[1:])]
    out = torch.full((span,), 0xA5, dtype=torch.uint8, device=device)
    cu = S.Convertor()
    cu.prepare(ot, count, out.data_ptr(), send=False)
    _unpack_windows(cu, packed.data_ptr(), wins, random.Random(2))
    want = np.full(span, 0xA5, dtype=np.uint8)
    b.o.unpack(count, want, 0, 0, ref.tobytes())
    np.testing.assert_array_equal(_host(out), want)
    ot.destruct()


def _roundtrip_desc(device, ot, rec, count, frag=None, granule=None, seed=3):
    """Pack `count` instances of description `ot` through the bridge (optionally in
    fragments whose max_data must be a multiple of `granule`) and unpack them back; bytes
    against the oracle of `rec`."""
    import torch
    b = R.Built(rec)
    info = b.o.info()
    assert (ot.dt.size, ot.extent, ot.dt.true_lb) == (info["size"], info["ub"] - info["lb"], info["true_lb"])
    size = info["size"] * count
    span, origin = R.layout(info, count)
    host = R.fill_fast(span, seed)
    user = _dev(host, device)
    packed = torch.zeros(size, dtype=torch.uint8, device=device)
    conv = S.Convertor()
    assert conv.prepare(ot, count, user.data_ptr() + origin, send=True) == S.OPAL_SUCCESS
    if frag is None:
        rc, iovs, md = conv.pack([(packed.data_ptr(), size)])
        assert rc == 1 and md == size
        wins = [(0, size)]
    else:
        exp = None
        if granule:
            exp = (lambda p, c: c if p + c == size else (c // granule) * granule)
        wins = _pack_fragments(conv, packed.data_ptr(), size, frag, exp)
    ref = np.frombuffer(b.o.pack(count, host, origin, 0, size, element_granular=False), dtype=np.uint8)
    np.testing.assert_array_equal(_host(packed), ref)
    out = torch.full((span,), 0xA5, dtype=torch.uint8, device=device)
    cu = S.Convertor()
    cu.prepare(ot, count, out.data_ptr() + origin, send=False)
    _unpack_windows(cu, packed.data_ptr(), wins, random.Random(seed))
    want = np.full(span, 0xA5, dtype=np.uint8)
    b.o.unpack(count, want, origin, 0, ref.tobytes())
    np.testing.assert_array_equal(_host(out), want)
    ot.destruct()


def test_bridge_appendix_a_cfg1_plain_and_consolidated(device):
    """cfg1's opt_desc (FLOAT8 count 1024 blen 1 extent 16) x 2048, and MPI_Pack's
    consolidated form LOOP 2048 x {...} END_LOOP size 8192 (Appendix A, pack.c.in:118-125)."""
    vec = ("vector", 1024, 1, 2, ("basic", FLOAT8))
    ot = S.OpalType([S.data(FLOAT8, 1024, 1, 16, 0)], 8192, 0, 16376, 0, 16376)
    _roundtrip_desc(device, ot, vec, 2048, frag=4100, granule=8)
    cons = S.OpalType([S.loop(2048, 2, 16376), S.data(FLOAT8, 1024, 1, 16, 0), S.end_loop(2, 8192, 0)],
                      2048 * 8192, 0, 2048 * 16376, 0, 2047 * 16376 + 16376)
    _roundtrip_desc(device, cons, ("contig", 2048, vec), 1, frag=1 << 20, granule=8)


def test_bridge_appendix_a_cfg3_dim2_face(device):
    """512^3 float subarray face on dim 2 (start 511): FLOAT4 count 262144 disp 2044 blen 1
    extent 2048, resized to the 512 MiB array (Appendix A)."""
    n = 512
    rec = ("subarray", [n, n, n], [n, n, 1], [0, 0, n - 1], 0, ("basic", FLOAT4))
    ot = S.OpalType([S.data(FLOAT4, n * n, 1, 2048, 2044)], 4 * n * n, 0, 4 * n * n * n, 2044,
                    2044 + (n * n - 1) * 2048 + 4)
    _roundtrip_desc(device, ot, rec, 1, frag=65539, granule=4)


def test_bridge_appendix_a_cfg5_promoted_struct(device):
    """hvector(N,1,32) of struct{double,int[3]}: the reference's optimizer re-types the
    20-byte record as UINT4 blen 5 (opal_datatype_optimize.c:581-611, Appendix A).  Through
    the bridge the pack's fragment boundaries follow that description: max_data is a
    multiple of 4 bytes, exactly as opal_pack_accelerator_simple would cut it
    (_pack_accelerator.c:52-58), not of the struct's double."""
    N = 1 << 18
    st = ("struct", [1, 3], [0, 8], [("basic", FLOAT8), ("basic", INT4)])
    rec = ("hvector", N, 1, 32, st)
    ot = S.OpalType([S.data(UINT4, N, 5, 32, 0)], 20 * N, 0, (N - 1) * 32 + 24, 0, (N - 1) * 32 + 20)
    _roundtrip_desc(device, ot, rec, 1, frag=(1 << 16) + 6, granule=4)


def _lcg(n, mod_bits):
    out = np.empty(n, dtype=np.int64)
    x, m = 0x5EED, (1 << mod_bits) - 1
    for i in range(n):
        out[i] = x
        x = (1664525 * x + 1013904223) & m
    return out


def test_bridge_appendix_a_cfg4_indexed_pairs(device):
    """An indexed type as the reference's optimizer leaves it: pairs fused into
    FLOAT4 count 2 blen 1 extent (d2-d1) entries (opal_datatype_optimize.c:1179-1185,
    Appendix A), here 1 Mi unique LCG displacements (the §8d recipe on a 2^24-float span).
    The import folds the run into one index list, so the whole message takes the
    address-ordered engine."""
    n = 1 << 20
    d = _lcg(n, 24)
    assert len(np.unique(d)) == n
    ents = [S.data(FLOAT4, 2, 1, int(d[k + 1] - d[k]) * 4, int(d[k]) * 4) for k in range(0, n, 2)]
    rec = ("indexed_block", 1, d.tolist(), ("basic", FLOAT4))
    b = R.Built(rec)
    info = b.o.info()
    ot = S.OpalType(ents, info["size"], info["lb"], info["ub"], info["true_lb"], info["true_ub"])
    _roundtrip_desc(device, ot, rec, 1)


def test_bridge_ddt_raw2_description(device):
    """ddt_raw2.c's hand-written committed description (185 entries of LOOP/DATA/END_LOOP,
    tests/golden/ddt_raw2_desc.json) imported through the bridge: the packed stream is the
    description walked literally (opal_convertor_raw.c:148-262 order), whole and in
    fragments, and unpacking it restores exactly those bytes."""
    import torch
    from .test_cpu_raw import _opal_desc_bytes, _walk_desc
    fx = json.load(open(os.path.join(HERE, "golden", "ddt_raw2_desc.json")))
    rows, used, bd = fx["desc"], fx["used"], fx["bounds"]
    raw = _opal_desc_bytes(rows[:used])
    ents = [raw[32 * i:32 * i + 32] for i in range(used)]
    ot = S.OpalType(ents, bd["size"], bd["lb"], bd["ub"], bd["true_lb"], bd["true_ub"], flags=bd["flags"] & 0xFFF0)
    pieces = []
    _walk_desc(rows, 0, used, 0, pieces)
    span = bd["true_ub"] + 64
    host = R.fill(span, 11)
    user = _dev(host, device)
    ref = np.concatenate([host[a:a + n] for a, n in pieces])
    size = bd["size"]
    assert len(ref) == size
    packed = torch.zeros(size, dtype=torch.uint8, device=device)
    for frag in (size, 1000, 37):
        packed.zero_()
        conv = S.Convertor()
        assert conv.prepare(ot, 1, user.data_ptr(), send=True) == S.OPAL_SUCCESS
        wins = _pack_fragments(conv, packed.data_ptr(), size, frag)
        np.testing.assert_array_equal(_host(packed), ref)
    out = torch.full((span,), 0xA5, dtype=torch.uint8, device=device)
    cu = S.Convertor()
    cu.prepare(ot, 1, out.data_ptr(), send=False)
    _unpack_windows(cu, packed.data_ptr(), wins, random.Random(5))
    want = np.full(span, 0xA5, dtype=np.uint8)
    for (a, n), off in zip(pieces, np.cumsum([0] + [n for _, n in pieces])[:-1]):
        want[a:a + n] = ref[off:off + n]
    np.testing.assert_array_equal(_host(out), want)
    ot.destruct()


# ------------------------------------------------------------------ fuzz through the bridge
@pytest.mark.parametrize("seed", range(int(os.environ.get("DDT_BRIDGE_FUZZ_SEEDS", "3"))))
def test_bridge_fuzz_descriptions(device, seed):
    """Random recipes (half of them mixed-type structs in loops) handed to the bridge as the
    opal_datatype_t Open MPI commits, in two forms -- desc and opt_desc from the oracle's
    restatement of opal_datatype_add + opal_datatype_commit, and the engine's own export of
    the same (ddt_type_to_opal_desc / ddt_type_to_opal_opt_desc) -- packed in random fragments
    (element-granular max_data == the oracle's walk of opt_desc) and unpacked in shuffled
    windows, counts 1-3; bytes == oracle."""
    import torch
    rng = random.Random(1000 + seed)
    done = 0
    while done < 20:
        rec = R.random_recipe(rng) if done % 2 else R.random_mixed_recipe(rng)
        b = R.Built(rec)
        info = b.o.info()
        count = rng.choice([1, 2, 3])
        size = info["size"] * count
        if size == 0 or size > (1 << 20):
            continue
        if (info["flags"] & S.F_NO_GAPS) and info["ub"] - info["lb"] != info["size"] and count > 1:
            # a reference quirk, not a parity case: adding an empty sub-type moves lb/ub but
            # returns before the flags are recomputed (opal_datatype_add.c:255, :285), so NO_GAPS
            # survives with extent != size, and the NO_OP path (opal_convertor.c:262-302) would
            # copy count*size contiguous bytes instead of the type map; the engine follows the map
            continue
        span, origin = R.layout(info, count)
        host = R.fill(span, seed * 31 + done)
        user = _dev(host, device)
        ref = np.frombuffer(b.o.pack(count, host, origin, 0, size, element_granular=False), dtype=np.uint8)
        overlap = _overlaps(b.o.runs(), count, info["ub"] - info["lb"])
        committed = S.from_oracle(b.o)
        ents = b.engine().to_opal_desc()
        opt, oflags = b.engine().to_opal_opt_desc()
        split = lambda raw: [raw[32 * i:32 * i + 32] for i in range(len(raw) // 32)]  # noqa: E731
        engine = S.OpalType(split(ents), info["size"], info["lb"], info["ub"], info["true_lb"],
                            info["true_ub"], flags=committed.dt.flags, opt_entries=split(opt))
        for form, ot in (("committed", committed), ("engine", engine)):
            packed = torch.zeros(size, dtype=torch.uint8, device=device)
            conv = S.Convertor()
            assert conv.prepare(ot, count, user.data_ptr() + origin, send=True) == S.OPAL_SUCCESS
            exp = None if conv.c.flags & S.CONVERTOR_NO_OP else \
                (lambda p, c: len(b.o.pack(count, host, origin, p, c, element_granular=True)))
            frag = rng.choice([5, 12, 40, 333, size])
            wins = _pack_fragments(conv, packed.data_ptr(), size, frag, exp, limit=4096)
            got = _host(packed)
            bad = np.nonzero(got != ref)[0]
            assert len(bad) == 0, (form, rec, count, frag, size, info, bad[:16].tolist(), len(bad),
                                   wins[:8], (user.data_ptr() + origin) % 64, packed.data_ptr() % 64)
            if not overlap:
                out = torch.full((span,), 0xA5, dtype=torch.uint8, device=device)
                cu = S.Convertor()
                cu.prepare(ot, count, out.data_ptr() + origin, send=False)
                _unpack_windows(cu, packed.data_ptr(), wins, rng)
                want = np.full(span, 0xA5, dtype=np.uint8)
                b.o.unpack(count, want, origin, 0, ref.tobytes())
                np.testing.assert_array_equal(_host(out), want)
            ot.destruct()
        done += 1


# ------------------------------------------------------------------ async + staging
def test_bridge_async_stream_host_fragments(device):
    """CONVERTOR_ACCELERATOR_ASYNC with convertor->stream (pml_ob1_recvfrag.c:761-769): the
    bridge queues on that stream and returns.  Back-to-back asynchronous unpacks from
    pinned host fragments (>16 MiB and small ones, no synchronisation between them) reuse
    the staging slots only after the previous kernel has read them."""
    import torch
    rec = ("vector", 1 << 20, 5, 9, ("basic", FLOAT8))   # 40 MiB packed
    b = R.Built(rec)
    info = b.o.info()
    size = info["size"]
    span, origin = R.layout(info, 1)
    host = R.fill(span, 13)
    ref = np.frombuffer(b.o.pack(1, host, origin, 0, size, element_granular=False), dtype=np.uint8)
    pinned = torch.from_numpy(ref.copy()).pin_memory()
    ot = S.OpalType([S.data(FLOAT8, 1 << 20, 5, 72, 0)], size, info["lb"], info["ub"], info["true_lb"],
                    info["true_ub"])
    s = torch.cuda.Stream(device)
    out = torch.full((span,), 0xA5, dtype=torch.uint8, device=device)
    cu = S.Convertor()
    cu.prepare(ot, 1, out.data_ptr() + origin, send=False, stream=s.cuda_stream)
    cuts = [0, 20 << 20, (20 << 20) + 4096, (21 << 20) + 3, (38 << 20) + 1, size]
    for a, c in zip(cuts, cuts[1:]):
        cu.set_position(a)
        rc, iovs, md = cu.unpack([(pinned.data_ptr() + a, c - a)])
        assert md == c - a
    s.synchronize()
    want = np.full(span, 0xA5, dtype=np.uint8)
    b.o.unpack(1, want, origin, 0, ref.tobytes())
    np.testing.assert_array_equal(_host(out), want)
    # async pack into pinned host memory: the stream carries the D2H copies too
    user = _dev(host, device)
    dst = torch.zeros(size, dtype=torch.uint8).pin_memory()
    cp = S.Convertor()
    cp.prepare(ot, 1, user.data_ptr() + origin, send=True, stream=s.cuda_stream)
    pos, k, rc = 0, 1, 0
    while rc == 0:   # in order; each capacity ends at the next cut (pack stops on elements)
        cap = max(cuts[k] - pos, 0) or size - pos
        rc, iovs, md = cp.pack([(dst.data_ptr() + pos, cap)])
        assert md == (cap if pos + cap == size else cap // 8 * 8)
        pos += md
        k = min(k + 1, len(cuts) - 1)
    assert pos == size
    s.synchronize()
    np.testing.assert_array_equal(dst.numpy(), ref)
    ot.destruct()


@pytest.mark.parametrize("mode", ["pinned-direct", "pinned-staged", "pageable-staged"])
def test_engine_async_unpack_slot_reuse_across_calls(device, mode):
    """back-to-back asynchronous unpacks from host buffers through ONE
    engine convertor, each call reusing both staging slots while the previous call's
    kernels may still run; bytes must match the oracle.  Pinned host memory is read by the
    kernel itself by default (hostdirect); staging is forced for the pinned-staged case and
    is the only path for pageable memory."""
    import torch
    import ompi_amd
    ompi_amd.lib().ddt_tune(b"hostdirect", 0 if mode == "pinned-staged" else 3)
    rec = ("vector", 1 << 19, 16, 24, ("basic", FLOAT4))   # 32 MiB packed
    b = R.Built(rec)
    e = b.engine()
    info = b.o.info()
    size = info["size"]
    span, origin = R.layout(info, 1)
    host = R.fill(span, 17)
    ref = np.frombuffer(b.o.pack(1, host, origin, 0, size, element_granular=False), dtype=np.uint8)
    if mode.startswith("pinned"):
        src = [torch.from_numpy(ref.copy()).pin_memory() for _ in range(2)]
    else:
        src = [torch.from_numpy(ref.copy()) for _ in range(2)]
    s = torch.cuda.Stream(device)
    outs = [torch.full((span,), 0xA5, dtype=torch.uint8, device=device) for _ in range(3)]
    c = ompi_amd.Convertor()
    c.set_stream(s, True)
    for k, out in enumerate(outs):
        c.prepare_for_recv(e, 1, out.data_ptr() + origin)
        # a 25 MiB window (staged in two overlapped chunks), 3 bytes, the rest (one chunk)
        for a, n in ((0, 25 << 20), (25 << 20, 3), ((25 << 20) + 3, size - (25 << 20) - 3)):
            c.set_position(a)
            rc, _, md = c.unpack([(src[k % 2].data_ptr() + a, n)])
            assert md == n
    s.synchronize()
    want = np.full(span, 0xA5, dtype=np.uint8)
    b.o.unpack(1, want, origin, 0, ref.tobytes())
    ompi_amd.lib().ddt_tune(b"hostdirect", 3)
    for out in outs:
        np.testing.assert_array_equal(_host(out), want)


@pytest.mark.parametrize("mode", ["pinned-staged", "pageable-staged"])
def test_engine_async_pack_staging_across_calls(device, mode):
    """Back-to-back asynchronous packs into host buffers through ONE engine convertor: each
    call's kernels rewrite the staging buffer only after the previous call's D2H copies have
    read it; windows of 30 MiB (two overlapped chunks, kernels queued before the copies) and
    10 MiB (one chunk)."""
    import torch
    import ompi_amd
    ompi_amd.lib().ddt_tune(b"hostdirect", 0 if mode == "pinned-staged" else 3)
    rec = ("vector", 5 << 20, 2, 3, ("basic", FLOAT4))   # 40 MiB packed
    b = R.Built(rec)
    e = b.engine()
    info = b.o.info()
    size = info["size"]
    span, origin = R.layout(info, 1)
    srcs = [R.fill(span, 40 + k) for k in range(3)]
    users = [_dev(h, device) for h in srcs]
    refs = [np.frombuffer(b.o.pack(1, h, origin, 0, size, element_granular=False), dtype=np.uint8)
            for h in srcs]
    pin = mode.startswith("pinned")
    dsts = [torch.zeros(size, dtype=torch.uint8, pin_memory=pin) for _ in range(3)]
    s = torch.cuda.Stream(device)
    c = ompi_amd.Convertor()
    c.set_stream(s, True)
    for k in range(3):
        c.prepare_for_send(e, 1, users[k].data_ptr() + origin)
        for a, n in ((0, 30 << 20), (30 << 20, size - (30 << 20))):
            rc, _, md = c.pack([(dsts[k].data_ptr() + a, n)])
            assert md == n
    s.synchronize()
    ompi_amd.lib().ddt_tune(b"hostdirect", 3)
    for k in range(3):
        np.testing.assert_array_equal(dsts[k].numpy(), refs[k])


# ------------------------------------------------------------------ unpack_ooo.c
N_OOO = 331
OOO_TRACES = {   # unpack_ooo.c:223-258: (bytes_received, data_offset) of real BTL fragment streams
    "test1": [(992, 0), (1325, 992), (992, 2317), (992, 3309), (992, 4301), (992, 5293), (992, 6285),
              (667, 7277)],
    "test2": [(992, 0), (992, 2317), (992, 3309), (992, 4301), (992, 5293), (992, 6285), (1325, 992),
              (667, 7277)],
    "test3": [(992, 0), (4960, 2317), (1325, 992), (667, 7277)],
    "test4": [(992, 0), (992, 2976), (992, 1984), (992, 992), (3976, 3968)],
}


def _ooo_buffers():
    """pbar (the packed stream: struct pfoo_t {int i[2]; double d[2];}) and the initial bar
    (struct foo_t {int i[3]; double d[3];}, 40 bytes) of unpack_ooo.c:90-101."""
    pbar = bytearray()
    bar = bytearray()
    ff4, ff8 = b"\xff" * 4, b"\xff" * 8
    for j in range(N_OOO):
        pbar += struct.pack("<iidd", 123 + j, 789 + j, 123.456 + j, 789.123 + j)
        bar += ff4 + struct.pack("<i", 0) + ff4 + b"\x77" * 4 + ff8 + struct.pack("<d", 0.0) + ff8
    return np.frombuffer(bytes(pbar), dtype=np.uint8), np.frombuffer(bytes(bar), dtype=np.uint8).copy()


def _check_ooo(bar_bytes):
    """unpack_ooo.c:132-134: i[0], i[2], d[0], d[2] from pbar; i[1] and d[1] untouched (and,
    stricter than the reference, the 4 padding bytes too)."""
    for j in range(N_OOO):
        r = bar_bytes[40 * j:40 * j + 40].tobytes()
        i0, i1, i2 = struct.unpack_from("<iii", r, 0)
        d0, d1, d2 = struct.unpack_from("<ddd", r, 16)
        assert (i0, i1, i2) == (123 + j, 0, 789 + j), j
        assert (d0, d1, d2) == (123.456 + j, 0.0, 789.123 + j), j
        assert r[12:16] == b"\x77" * 4


OOO_REC = ("struct", [1, 1], [0, 16], [("vector", 2, 1, 2, ("basic", INT4)),
                                       ("vector", 2, 1, 2, ("basic", FLOAT8))])


@pytest.mark.parametrize("trace", sorted(OOO_TRACES))
@pytest.mark.parametrize("path", ["bridge", "engine"])
@pytest.mark.parametrize("iov", ["host", "device"])
def test_reference_unpack_ooo_traces(device, trace, path, iov):
    """unpack_ooo.c restated: 331 instances of struct{vector(2,1,2,int) @0,
    vector(2,1,2,double) @16} received through the real BTL fragment traces test1-test4,
    out of order via set_position; the struct contents must be the reference's."""
    import torch
    import ompi_amd
    pbar, bar0 = _ooo_buffers()
    b = R.Built(OOO_REC)
    info = b.o.info()
    assert (info["size"], info["ub"] - info["lb"]) == (24, 40)
    assert sum(n for n, _ in OOO_TRACES[trace]) == 24 * N_OOO
    bar = _dev(bar0, device)
    src = torch.from_numpy(pbar.copy())
    src = src.pin_memory() if iov == "host" else src.to(device)
    if path == "bridge":
        ot = S.from_oracle(b.o)
        conv = S.Convertor()
        assert conv.prepare(ot, N_OOO, bar.data_ptr(), send=False) == S.OPAL_SUCCESS
    else:
        conv = ompi_amd.Convertor().prepare_for_recv(b.engine(), N_OOO, bar.data_ptr())
    for n, off in OOO_TRACES[trace]:
        assert conv.set_position(off) == off
        rc, iovs, md = conv.unpack([(src.data_ptr() + off, n)])
        assert md == n
    _check_ooo(_host(bar))
    if path == "bridge":
        ot.destruct()


# ------------------------------------------------------------------ cache under capture
def test_descriptor_sets_follow_shape_not_buffers_and_survive_capture(device):
    """Descriptor sets are keyed by the request's shape and pointer alignment: alternating
    buffer pairs reuse ONE set.  Inside a HIP-graph capture, 100 distinct windows (each used
    twice, so the second use launches by pointer) force evictions far past the 32-entry
    cache; captured sets are held for the graph, and replaying the graph stays bit-exact.
    No call in this sequence synchronises the device (retirement is event-based)."""
    import torch
    import ompi_amd
    rec = ("vector", 4096, 3, 7, ("basic", FLOAT4))
    b = R.Built(rec)
    e = b.engine()
    info = b.o.info()
    size = info["size"]
    span, origin = R.layout(info, 1)
    hosts = [R.fill(span, 21 + k) for k in range(2)]
    users = [_dev(h, device) for h in hosts]
    pks = [torch.zeros(size, dtype=torch.uint8, device=device) for _ in range(2)]
    c = ompi_amd.Convertor()
    for rep in range(3):
        for k in range(2):
            c.prepare_for_send(e, 1, users[k].data_ptr() + origin)
            c.pack([(pks[k], size)])
    assert e.cache_info()["cached"] == 1
    refs = [np.frombuffer(b.o.pack(1, h, origin, 0, size, element_granular=False), dtype=np.uint8)
            for h in hosts]
    for k in range(2):
        np.testing.assert_array_equal(_host(pks[k]), refs[k])
    # capture: 100 windows x 2 uses, alternating buffers
    s = torch.cuda.Stream(device)
    g = torch.cuda.CUDAGraph()
    W = size // 100 // 4 * 4
    for p in pks:
        p.zero_()
    torch.cuda.synchronize()
    with torch.cuda.graph(g, stream=s, capture_error_mode="relaxed"):
        cs = torch.cuda.current_stream(device)
        for w in range(100):
            for k in range(2):
                ompi_amd.lib().ddt_pack_window(e.handle, 1, users[k].data_ptr() + origin, w * W,
                                               pks[k].data_ptr() + w * W, W, None, cs.cuda_stream)
    ci = e.cache_info()
    assert ci["cached"] <= 32 and ci["pinned"] >= 50, ci
    g.replay()
    torch.cuda.synchronize()
    for k in range(2):
        np.testing.assert_array_equal(_host(pks[k])[:100 * W], refs[k][:100 * W])
    for p in pks:
        p.zero_()
    g.replay()
    torch.cuda.synchronize()
    for k in range(2):
        np.testing.assert_array_equal(_host(pks[k])[:100 * W], refs[k][:100 * W])


@pytest.mark.parametrize("rec", [
    ("vector", 4096, 3, 7, ("basic", FLOAT4)),
    # nine interleaved leaves: every window's descriptor set is beyond the kernel-argument
    # block and lives in HBM from its first launch
    ("struct", [1] * 9, [4 * i for i in range(9)], [("vector", 2048, 1, 9, ("basic", FLOAT4))] * 9),
])
def test_descriptor_sets_shared_by_threads(device, rec):
    """One committed datatype driven by four host threads at once, each on its own stream:
    48 distinct windows (shared shapes across threads, so the threads hit each other's
    descriptor sets), swept three times so sets are launched by pointer, and more shapes than
    the 32-entry cache, so sets are evicted and recycled while other threads are enqueuing
    launches of them.  Every window of every sweep is bit-exact with the oracle."""
    import threading
    import torch
    import ompi_amd
    b = R.Built(rec)
    e = b.engine()
    info = b.o.info()
    size = info["size"]
    span, origin = R.layout(info, 1)
    host = R.fill(span, 77)
    user = _dev(host, device)
    ref = np.frombuffer(b.o.pack(1, host, origin, 0, size, element_granular=False), dtype=np.uint8)
    NW, SWEEPS, NT = 48, 3, 4
    W = size // NW // 4 * 4
    streams = [torch.cuda.Stream(device) for _ in range(NT)]
    outs = [torch.zeros(SWEEPS * size, dtype=torch.uint8, device=device) for _ in range(NT)]
    errors = []
    lib = ompi_amd.lib()

    def worker(t):
        try:
            rng = random.Random(500 + t)
            for sweep in range(SWEEPS):
                order = list(range(NW))
                rng.shuffle(order)
                base = outs[t].data_ptr() + sweep * size
                for w in order:
                    rc = lib.ddt_pack_window(e.handle, 1, user.data_ptr() + origin, w * W, base + w * W, W, None,
                                             streams[t].cuda_stream)
                    if rc < 0:
                        errors.append((t, sweep, w, rc))
                        return
            streams[t].synchronize()
        except Exception as ex:   # pragma: no cover - reported below
            errors.append((t, repr(ex)))

    torch.cuda.synchronize()
    ths = [threading.Thread(target=worker, args=(t,)) for t in range(NT)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    assert not errors, errors
    torch.cuda.synchronize()
    for t in range(NT):
        got = _host(outs[t])
        for sweep in range(SWEEPS):
            np.testing.assert_array_equal(got[sweep * size: sweep * size + NW * W], ref[:NW * W],
                                          err_msg=f"thread {t} sweep {sweep}")
    ci = e.cache_info()
    assert ci["cached"] <= 32, ci


def test_bridge_from_c(device):
    """bridge/bridge_demo.c: the same drop-in driven from C on opal_datatype_t /
    opal_convertor_t structs compiled against include/opal_layout.h -- prepare as
    OPAL_CONVERTOR_PREPARE does, opal_hip_bridge_attach, fAdvance in 7000-byte fragments,
    fPosition + fAdvance in 4099-byte windows last to first -- checked against the closed form
    of the x face on the host."""
    import subprocess
    exe = os.path.join(os.path.dirname(HERE), "bridge", "bridge_demo")
    assert os.path.exists(exe), "build() compiles bridge/bridge_demo"
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "bridge_demo ok" in r.stdout
