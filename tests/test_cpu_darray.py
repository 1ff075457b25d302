"""MPI_Type_create_darray (ompi_datatype_create_darray.c:187-312).

* The engine's and the oracle's darray issue the reference's constructor calls in its
  order (block / cyclic / none helpers, the trailing struct of a partial cyclic block,
  the final displaced add plus resize).  Bounds, flags and type maps must agree on fuzzed
  distributions.
* Semantics pin independent of both: the darrays of all ranks of a process grid
  partition the global array.  Every element is owned by exactly one rank.
* The reference's big-count known answers (mpi_datatype_bigcount.c:563-680): size and
  extent of darrays whose counts exceed INT_MAX (engine only; the oracle is flat).
"""
from __future__ import annotations

import random

import numpy as np
import pytest

from ompi_amd import datatype as D
from tests import oracle as O
from tests import plan_emu as E
from tests import recipes as R

BIG = 2 ** 31 - 1


def random_darray(rng):
    ndims = rng.randint(1, 3)
    gs = [rng.randint(1, 7) for _ in range(ndims)]
    ps = [rng.randint(1, 3) for _ in range(ndims)]
    size = int(np.prod(ps))
    dist, darg = [], []
    for g, p in zip(gs, ps):
        k = rng.choice([0, 1, 2])
        if k == 2:
            dist.append(2)
            darg.append(-1)
        elif k == 0:
            dist.append(0)
            lo = -(-g // p)   # a block darg must cover the dimension
            darg.append(rng.choice([-1, lo, lo + 1]))
        else:
            dist.append(1)
            darg.append(rng.choice([-1, 1, 2, 3]))
    # MPI_DISTRIBUTE_NONE requires a process-grid dimension of 1
    ps = [1 if d == 2 else p for d, p in zip(dist, ps)]
    size = int(np.prod(ps))
    old = ("basic", rng.choice([4, 6, 16, 21]))
    if rng.random() < 0.3:
        old = ("vector", 2, 1, 3, old)
    return size, gs, dist, darg, ps, rng.randint(0, 1), old


def test_darray_bounds_and_type_map_match_oracle():
    rng = random.Random(5200)
    n = 0
    while n < 150:
        size, gs, dist, darg, ps, order, old = random_darray(rng)
        rank = rng.randrange(size)
        rec = ("darray", size, rank, gs, dist, darg, ps, order, old)
        b = R.Built(rec)
        oi, ei = b.o.info(), b.engine().info()
        for k in ("size", "lb", "ub", "true_lb", "true_ub"):
            if oi["size"] or k in ("size", "lb", "ub"):
                assert oi[k] == ei[k], (rec, k, oi, ei)
        np.testing.assert_array_equal(E.engine_blocks(b.engine()), E.oracle_blocks(b.o),
                                      err_msg=str(rec))
        n += 1


def test_darrays_of_all_ranks_partition_the_global_array():
    rng = random.Random(5300)
    for _ in range(60):
        size, gs, dist, darg, ps, order, _ = random_darray(rng)
        old = O.basic(4)   # 1-byte elements: offsets are element indices
        owner = np.zeros(int(np.prod(gs)), dtype=np.int64)
        for rank in range(size):
            t = O.darray(size, rank, gs, dist, darg, ps, order, old)
            assert t.info()["lb"] == 0 and t.info()["ub"] == len(owner)
            for d, ln, _ in t.runs():
                owner[d:d + ln] += 1
        assert np.all(owner == 1), (gs, dist, darg, ps, order)


def _size_extent(t):
    i = t.info()
    return i["size"], i["lb"], i["ub"] - i["lb"]


def test_reference_bigcount_darray_known_answers():
    byte = D.predefined(D.UINT1)
    # test_darray_c_bigcount: 2-D block on one process owns everything
    t = D.create_darray(1, 0, [BIG + 5, BIG + 6], [0, 0], [-1, -1], [1, 1], 0, byte).commit()
    g = (BIG + 5) * (BIG + 6)
    assert _size_extent(t) == (g, 0, g)
    # test_darray_cyclic_c_bigcount
    t = D.create_darray(1, 0, [BIG + 5], [1], [-1], [1], 0, byte).commit()
    assert _size_extent(t) == (BIG + 5, 0, BIG + 5)
    # test_darray_multiproc_c_bigcount: rank 1 of 2 owns the upper half
    t = D.create_darray(2, 1, [4 * BIG], [0], [-1], [2], 0, byte).commit()
    assert _size_extent(t) == (2 * BIG, 0, 4 * BIG)
    # test_darray_blockcyclic_c_bigcount: cyclic(3) with a partial last block (struct path)
    t = D.create_darray(1, 0, [BIG + 7], [1], [3], [1], 0, byte).commit()
    assert _size_extent(t) == (BIG + 7, 0, BIG + 7)


def test_darray_zero_dims_is_empty():
    t = D.create_darray(1, 0, [], [], [], [], 0, D.predefined(D.INT4)).commit()
    assert t.info()["size"] == 0


@pytest.mark.parametrize("order", [0, 1])
def test_darray_block_2d_layout(order):
    # 4x6 global int array on a 2x2 grid, rank 3 owns the bottom-right 2x3 block
    t = O.darray(4, 3, [4, 6], [0, 0], [-1, -1], [2, 2], order, O.basic(6))
    offs = []
    for d, ln, _ in t.runs():
        offs += list(range(d // 4, (d + ln) // 4))
    if order == 0:   # C order: row-major
        want = [r * 6 + c for r in (2, 3) for c in (3, 4, 5)]
    else:            # Fortran order: column-major
        want = [c * 4 + r for c in (3, 4, 5) for r in (2, 3)]
    assert offs == want
