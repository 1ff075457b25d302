"""Single-item launches with the item's fields passed by value (ddt_affine1_kernel,
ddt_dense1_kernel; ddt_kernels.hip launch_single_item, late round 3).

A launch of ONE affine item of >= 1024 tasks skips the descriptor set: its fields travel in the
kernel arguments and each workgroup takes one task (streaming items of 16-byte units,
ddt_tune "afast") or one LDS chunk (line-dense items, "dfast").  The bytes must be those of the
reference's convertor walking the same type (opal_datatype_pack.c / opal_datatype_unpack.c,
restated by the oracle) whatever the launch form; each shape runs with the by-value launch in
the pack, in both directions and in neither, and the two forms must also agree byte for byte
with each other.
"""
from __future__ import annotations

import numpy as np
import pytest

from . import recipes as R
from .test_gpu_parity import _roundtrip

pytestmark = pytest.mark.gpu

FLOAT8 = 16

SHAPES = {
    # 512-byte rows every 1 KiB: a streaming leaf (non-temporal loads), 1024 tasks
    "rows512": (("vector", 32768, 64, 128, ("basic", FLOAT8)), 1),
    # 2 KiB rows every 4 KiB, three instances (a two-dim nest), 1536 tasks
    "rows2k_x3": (("resized", ("vector", 4096, 256, 512, ("basic", FLOAT8)), 0, 4096 * 4096 + 256), 3),
    # 64-byte blocks every 128 bytes (plain loads), 1024 tasks
    "blk64": (("vector", 262144, 8, 16, ("basic", FLOAT8)), 1),
    # one contiguous 16 MiB run
    "contig": (("contig", 1 << 21, ("basic", FLOAT8)), 1),
}


@pytest.fixture
def knobs():
    import ompi_amd
    L = ompi_amd.lib()

    def set_(**kv):
        for k, v in kv.items():
            L.ddt_tune(k.encode(), v)
    yield set_
    set_(afast=0, dfast=1)   # ddt_plan.h Tuning defaults


@pytest.mark.parametrize("afast", [1, 3, 0])
@pytest.mark.parametrize("name", sorted(SHAPES))
def test_streaming_item_by_value(device, knobs, name, afast):
    """Pack and unpack against the oracle, the buffer aligned and 4 bytes off (4-byte units:
    the descriptor path)."""
    knobs(afast=afast)
    rec, count = SHAPES[name]
    b = R.Built(rec)
    _roundtrip(b, count, device, 71)
    _roundtrip(b, count, device, 72, shift=4)


def test_by_value_matches_descriptor_launch(device, knobs):
    """The same message packed through the by-value kernels and through the descriptor kernel:
    identical packed bytes, and identical user bytes after unpacking them into a pre-filled
    buffer (gaps untouched by both)."""
    import torch
    import ompi_amd
    rec, count = SHAPES["rows2k_x3"]
    b = R.Built(rec)
    info = b.o.info()
    size = info["size"] * count
    span, origin = R.layout(info, count)
    user = torch.from_numpy(R.fill(span, 81)).to(device)
    packs, unpacks = [], []
    for fast in (3, 0):
        knobs(afast=fast)
        e = R.Built(rec).engine()
        pk = torch.zeros(size, dtype=torch.uint8, device=device)
        assert ompi_amd.pack(user.data_ptr() + origin, count, e, pk, size, 0) == size
        out = torch.full((span,), 0x3C, dtype=torch.uint8, device=device)
        assert ompi_amd.unpack(pk, size, 0, out.data_ptr() + origin, count, e) == size
        torch.cuda.synchronize()
        packs.append(pk.cpu().numpy())
        unpacks.append(out.cpu().numpy())
    np.testing.assert_array_equal(packs[0], packs[1])
    np.testing.assert_array_equal(unpacks[0], unpacks[1])
