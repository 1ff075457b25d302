"""Line-dense records through the LDS path (run_dense / ddt_dense_kernel, round 3).

A leaf whose records of several 4-byte units sit at a stride of at most four record lengths
(cfg5's 20-byte struct{double,int[3]} at 32 bytes) is moved a chunk of records at a time:
whole 16-byte loads of the span into LDS, then 16-byte packed stores (pack), or the packed
chunk into LDS and record-wide stores (unpack).  The reference has no such path: it walks
the same records with one memcpy per block (opal_datatype_pack.c, pack_predefined_data /
opal_pack_homogeneous_contig_with_gaps_function), and the bytes must be identical.

Every shape here qualifies (ddt_plan.cpp dense_records), at record sizes 12..240 bytes,
records 4- but not 16-byte aligned, counts whose instances break the record runs inside a
task (the unit-loop fallback), fragment pipelines (the inline-descriptor kernel), both task
mappings of the unpack (ddt_tune dsplit) and a capped grid over pinned host memory, and the
by-value launch of a large single dense item (ddt_dense1_kernel, >= 1024 chunks: a workgroup per
chunk, ddt_tune dfast) on one- and two-dim nests, 16- and 4-byte phases, both directions.
"""
from __future__ import annotations

import numpy as np
import pytest

from . import recipes as R
from .test_gpu_parity import _roundtrip

pytestmark = pytest.mark.gpu

FLOAT4, FLOAT8, INT4 = 15, 16, 6
REC20 = ("struct", [1, 3], [0, 8], [("basic", FLOAT8), ("basic", INT4)])   # cfg5's record

SHAPES = {
    "cfg5_rec": ("hvector", 50_000, 1, 32, REC20),              # 20 B at 32 B
    "f3_of_4": ("vector", 40_000, 3, 4, ("basic", FLOAT4)),      # 12 B at 16 B
    "f7_of_9": ("vector", 30_001, 7, 9, ("basic", FLOAT4)),      # 28 B at 36 B: 4-byte aligned only
    "f60_of_100": ("vector", 5_000, 60, 100, ("basic", FLOAT4)),  # 240 B at 400 B: 10 per chunk
    "d2_of_3": ("vector", 20_000, 2, 3, ("basic", FLOAT8)),      # 16 B at 24 B, 8-byte units
}


@pytest.fixture
def knobs():
    import ompi_amd
    L = ompi_amd.lib()

    def set_(**kv):
        for k, v in kv.items():
            L.ddt_tune(k.encode(), v)
    yield set_
    set_(dense=-1, dsplit=1, dfast=1, hd_grid=256, hd_grid_pack=0)   # ddt_plan.h Tuning defaults


@pytest.mark.parametrize("dsplit", [1, 0])
@pytest.mark.parametrize("name", sorted(SHAPES))
def test_dense_records_whole_message(device, knobs, name, dsplit):
    """Whole-message pack and unpack, one instance and three (a resized extent that is not a
    multiple of the stride: every instance starts at another 16-byte phase), and with the
    buffer 4 bytes off its allocation."""
    knobs(dsplit=dsplit)
    rec = SHAPES[name]
    b = R.Built(rec)
    _roundtrip(b, 1, device, 11)
    _roundtrip(b, 1, device, 12, shift=4)
    info = b.o.info()
    ext = info["ub"] - info["lb"] + 52
    _roundtrip(R.Built(("resized", rec, 0, ext)), 3, device, 13)


@pytest.mark.parametrize("dsplit", [1, 0])
def test_dense_records_runs_break_inside_tasks(device, knobs, dsplit):
    """Instances of 100 records (fewer than one task): the tasks of a count > 1 message
    cross instance boundaries, so run_dense refuses them and the unit loop of the same
    kernel moves them; bit-exact both ways."""
    knobs(dsplit=dsplit)
    inner = ("hvector", 100, 1, 32, REC20)
    b = R.Built(("resized", inner, 0, 100 * 32 + 64))
    _roundtrip(b, 37, device, 21)


def test_dense_records_fragments(device, knobs):
    """A fragment pipeline (descriptors in the kernel arguments): record-aligned and
    ragged fragments, pack and unpack."""
    b = R.Built(SHAPES["cfg5_rec"])
    _roundtrip(b, 1, device, 31, frags=[20 * 1000, 20 * 777 + 8, 65536, 4096])


def test_dense_records_same_as_unit_loop(device, knobs):
    """The LDS path and the unit loop (ddt_tune dense 0) give the same bytes on cfg5's
    record at a count of 2."""
    import torch
    import ompi_amd
    b = R.Built(SHAPES["cfg5_rec"])
    info = b.o.info()
    size = info["size"] * 2
    span, origin = R.layout(info, 2)
    user = torch.from_numpy(R.fill(span, 41)).to(device)
    outs = []
    for d in (-1, 0):
        knobs(dense=d)
        e = R.Built(SHAPES["cfg5_rec"]).engine()   # a fresh plan under each setting
        pk = torch.zeros(size, dtype=torch.uint8, device=device)
        assert ompi_amd.pack(user.data_ptr() + origin, 2, e, pk, size, 0) == size
        outs.append(pk.cpu().numpy())
    np.testing.assert_array_equal(outs[0], outs[1])


@pytest.mark.parametrize("dsplit", [1, 0])
def test_dense_records_pinned_capped_grid(device, knobs, dsplit):
    """Packed stream in pinned host memory with the workgroup cap of such launches at 8:
    the dense kernel loops over its (half) tasks."""
    import torch
    import ompi_amd
    knobs(hd_grid=8, hd_grid_pack=8, dsplit=dsplit)
    b = R.Built(SHAPES["f7_of_9"])
    info = b.o.info()
    size = info["size"]
    span, origin = R.layout(info, 1)
    host = R.fill(span, 51)
    user = torch.from_numpy(host).to(device)
    e = b.engine()
    ref = np.frombuffer(b.o.pack(1, host, origin, 0, size, element_granular=False), dtype=np.uint8)
    pk = torch.zeros(size, dtype=torch.uint8).pin_memory()
    assert ompi_amd.pack(user.data_ptr() + origin, 1, e, pk.data_ptr(), size, 0) == size
    torch.cuda.synchronize()
    np.testing.assert_array_equal(pk.numpy(), ref)
    out = torch.full((span,), 0xA5, dtype=torch.uint8, device=device)
    exp = np.full(span, 0xA5, dtype=np.uint8)
    b.o.unpack(1, exp, origin, 0, ref.tobytes())
    assert ompi_amd.unpack(pk.data_ptr(), size, 0, out.data_ptr() + origin, 1, e) == size
    np.testing.assert_array_equal(out.cpu().numpy(), exp)


BIG = {
    # one dim: 1563 chunks of 128 records
    "cfg5_rec_1d": (("hvector", 200_000, 1, 32, REC20), 1),
    # two dims (instances of 131072 records, a multiple of the 128-record chunk): 2048 chunks
    "cfg5_rec_2d": (("resized", ("hvector", 131_072, 1, 32, REC20), 0, 131_072 * 32 + 64), 2),
    # 28-byte records every 36 bytes (113 per chunk, 4-byte phases): 2655 chunks
    "f7_of_9_1d": (("vector", 300_000, 7, 9, ("basic", FLOAT4)), 1),
    # two dims whose inner count is NOT a multiple of the chunk: the descriptor path instead
    "cfg5_rec_2d_ragged": (("resized", ("hvector", 150_000, 1, 32, REC20), 0, 150_000 * 32 + 64), 2),
}


@pytest.mark.parametrize("dfast", [1, 3, 0])
@pytest.mark.parametrize("name", sorted(BIG))
def test_dense_by_value_launch(device, knobs, name, dfast):
    """Large single-item dense launches: the by-value kernel for the pack (dfast 1, default),
    both directions (3) or neither (0), aligned and 4 bytes off, bit-exact vs the oracle."""
    knobs(dfast=dfast)
    rec, count = BIG[name]
    b = R.Built(rec)
    _roundtrip(b, count, device, 61)
    _roundtrip(b, count, device, 62, shift=4)
