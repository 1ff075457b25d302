"""pack_description_sweep.c on the GPU through the drop-in boundary.

Each configuration of the sweep's matrix (tests/sweep.py) is an opal_datatype_t whose opt_desc is
the sweep's exact synthetic shape -- LOOP over `loop_items` uncollapsed `count x blocklen` DATA
entries, tail entries after it -- or, with --commit-description, the optimizer's result for the
struct of vectors.  The bridge is swapped in after prepare like the sweep's accelerator backend
(:877-960) and driven by its fragment loop (run_prepared_convertor, :962-996): pack and unpack,
whole and in `fragment_bytes` pieces.  Every packed stream is pack_reference's (:454-476); a pack
fragment never splits an element (max_data = whole elements of the fragment, :52-58 of
opal_datatype_pack_accelerator.c, as the sweep requires fragment_bytes >= element size);
unpack takes any byte fragment; gaps of the target keep their bytes.
"""
from __future__ import annotations

import random

import numpy as np
import pytest

from . import opal_shapes as S
from . import recipes as R
from . import sweep as W

pytestmark = pytest.mark.gpu


def _dev(arr, device):
    import torch
    return torch.from_numpy(np.ascontiguousarray(arr)).to(device)


def _host(t):
    import torch
    torch.cuda.synchronize()
    return t.cpu().numpy()


def _run(conv, base, packed_size, frag, unpack, es):
    """run_prepared_convertor (:962-996): set_position(0), then fragments until done."""
    assert conv.set_position(0) == 0
    converted, complete = 0, 0
    while converted < packed_size:
        fragment = packed_size - converted
        if frag and frag < fragment:
            fragment = frag
        iov = [(base + converted, fragment)]
        complete, _, md = conv.unpack(iov) if unpack else conv.pack(iov)
        assert complete >= 0 and 0 < md <= fragment, (converted, fragment, md)
        if not unpack:
            assert md == fragment - fragment % es, (converted, fragment, md)
        converted += md
    assert complete == 1 and converted == packed_size


def _check(sw, ot, device, rng):
    import torch
    span = sw.span()
    host = R.fill(span, 77 + sw.dc)
    user = _dev(host, device)
    total = sw.count * sw.size
    ref = sw.pack_reference(host)
    frags = [0, sw.es, 12 if sw.es == 4 else 24, 40, 4096, rng.choice([sw.es * 3 + sw.es // 2, 1000, 65536])]
    for frag in frags:
        if frag and frag < sw.es:
            continue
        packed = torch.zeros(total, dtype=torch.uint8, device=device)
        conv = S.Convertor()
        assert conv.prepare(ot, sw.count, user.data_ptr(), send=True) == S.OPAL_SUCCESS
        _run(conv, packed.data_ptr(), total, frag, False, sw.es)
        np.testing.assert_array_equal(_host(packed), ref, err_msg=f"{sw} pack frag {frag}")
        out = torch.full((span,), 0xA5, dtype=torch.uint8, device=device)
        cu = S.Convertor()
        assert cu.prepare(ot, sw.count, out.data_ptr(), send=False) == S.OPAL_SUCCESS
        ufrag = frag if frag == 0 else frag + rng.randint(0, 3)   # unpack: any byte boundary
        _run(cu, packed.data_ptr(), total, ufrag, True, sw.es)
        want = sw.unpack_reference(ref, np.full(span, 0xA5, dtype=np.uint8))
        np.testing.assert_array_equal(_host(out), want, err_msg=f"{sw} unpack frag {ufrag}")


@pytest.mark.parametrize("seed", range(3))
def test_sweep_synthetic_descriptions_through_the_bridge(device, seed):
    rng = random.Random(6100 + seed)
    for sw in W.random_sweeps(rng, 12):
        ot = sw.opal_type()
        _check(sw, ot, device, rng)
        ot.destruct()


def test_sweep_default_and_edge_shapes(device):
    """The sweep's own defaults-like shapes and the edges of the matrix: one item per loop,
    a single loop iteration with every item a tail, gapless blocks (uncollapsed counts), the
    longest blocks, 4- and 8-byte elements, three datatypes per convertor."""
    rng = random.Random(6200)
    for kw in [dict(), dict(loop_items=1, total_items=7), dict(loop_items=5, total_items=9),
               dict(block_gap=0, data_count=5, item_gap=2), dict(blocklen=64, data_count=2),
               dict(element_size=4, blocklen=1, data_count=5, block_gap=3, total_items=11, loop_items=3),
               dict(datatype_count=3, total_items=13, loop_items=6)]:
        sw = W.Sweep(**kw)
        if sw.contiguous:
            continue
        ot = sw.opal_type()
        _check(sw, ot, device, rng)
        ot.destruct()


@pytest.mark.parametrize("seed", range(2))
def test_sweep_committed_descriptions_bridge_and_engine(device, seed):
    """--commit-description: the optimizer's opt_desc (oracle restatement) through the bridge,
    and the same datatype built with the engine's constructors through its own convertor."""
    import torch
    import ompi_amd
    rng = random.Random(6300 + seed)
    for sw in W.random_sweeps(rng, 8, commit=True):
        ot = sw.opal_type()
        _check(sw, ot, device, rng)
        ot.destruct()
        e = R.build_engine(sw.recipe()).commit()
        span = sw.span()
        host = R.fill(span, 5)
        user = _dev(host, device)
        total = sw.count * sw.size
        packed = torch.zeros(total, dtype=torch.uint8, device=device)
        c = ompi_amd.Convertor().prepare_for_send(e, sw.count, user.data_ptr())
        pos = 0
        while pos < total:
            rc, _, md = c.pack([(packed.data_ptr() + pos, min(40, total - pos))])
            assert md > 0
            pos += md
        np.testing.assert_array_equal(_host(packed), sw.pack_reference(host), err_msg=repr(sw))
