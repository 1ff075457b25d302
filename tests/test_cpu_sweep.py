"""pack_description_sweep.c's descriptions through the import, on CPU.

The sweep (ompi/test/datatype/pack_description_sweep.c, restated in tests/sweep.py) hands the
convertor exact opt_desc shapes: a LOOP over `loop_items` DATA entries of `count x blocklen` at a
block stride -- not CREATE_ELEM-collapsed -- with the tail items after it as straight-line DATA
entries (install_synthetic_description, :254-316), or the optimizer's own result for a struct of
vectors (--commit-description).  Here each description is imported as the bridge imports it
(ddt_type_from_opal_desc) and the engine's compiled plan must move exactly pack_reference's blocks
(:454-476); the bridge must accept every one on an accelerator convertor.  The GPU half
(test_gpu_sweep.py) moves the bytes.
"""
from __future__ import annotations

import random

import numpy as np
import pytest

from tests import opal_shapes as S
from tests import plan_emu as E
from tests import recipes as R
from tests import sweep as W

FAKE_DEV = 0x7000_0000_0000


def _import(sw):
    from ompi_amd import datatype as D
    i = sw.info
    ents = b"".join(sw.synthetic_entries())
    return D.from_opal_desc(ents, i["size"], i["lb"], i["ub"], i["true_lb"], i["true_ub"])


def _reference_blocks(sw):
    one = W.Sweep(sw.es, sw.dc, sw.bl, sw.bg, sw.ig, sw.total, sw.loop, 1, sw.commit)
    return E.merge_runs(np.array(one.blocks(), dtype=np.int64).reshape(-1, 3))


@pytest.mark.parametrize("seed", range(4))
def test_synthetic_descriptions_import_to_the_reference_blocks(seed):
    rng = random.Random(5100 + seed)
    n = 0
    for sw in W.random_sweeps(rng, 60):
        t = _import(sw)
        np.testing.assert_array_equal(E.engine_blocks(t), _reference_blocks(sw), err_msg=repr(sw))
        # the constructors' type map moves the same bytes (the sweep replaces only opt_desc)
        np.testing.assert_array_equal(E.oracle_blocks(sw.otype), _reference_blocks(sw), err_msg=repr(sw))
        ot = sw.opal_type()
        c = S.Convertor()
        assert c.prepare(ot, sw.count, FAKE_DEV, send=True) == S.OPAL_SUCCESS, sw
        assert c.c.fAdvance, sw
        ot.destruct()
        n += 1
    assert n == 60


def test_tail_entries_and_uncollapsed_counts_are_exercised():
    """The matrix reaches the shapes the review asked for: tail entries after the LOOP, DATA
    entries whose stride equals their block (count > 1 that CREATE_ELEM would have collapsed),
    and block lengths up to 64."""
    rng = random.Random(5200)
    sws = W.random_sweeps(rng, 200)
    assert sum(sw.total % sw.loop != 0 for sw in sws) > 50
    assert sum(sw.bg == 0 and sw.dc > 1 for sw in sws) > 20
    assert max(sw.bl for sw in sws) == 64
    assert {sw.es for sw in sws} == {4, 8} and {sw.count for sw in sws} == {1, 2, 3}


@pytest.mark.parametrize("seed", range(2))
def test_committed_descriptions_engine_equals_oracle(seed):
    """--commit-description: the optimizer's opt_desc for the sweep's struct of vectors, from the
    oracle's restatement and from the engine's commit, entry for entry, and the blocks of
    pack_reference."""
    rng = random.Random(5300 + seed)
    for sw in W.random_sweeps(rng, 40, commit=True):
        e = R.build_engine(sw.recipe()).commit()
        raw, fl = e.to_opal_opt_desc()
        assert S.unpack_entries(raw) == sw.otype.opt_desc(), sw
        np.testing.assert_array_equal(E.engine_blocks(e), _reference_blocks(sw), err_msg=repr(sw))
