"""Multi-rank sharding on CPU: world_size 2 and 3 with the gloo backend.

Each rank packs its instance range of one message (here with the CPU oracle, the
checker -- the GPU engine is exercised by the same shard arithmetic in bench.py), the
shards are all-gathered, and the concatenation must equal the whole-message stream.
"""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest

from ompi_amd import shard


def test_count_shards_cover_and_balance():
    for count in (0, 1, 7, 16, 64, 1001):
        for world in (1, 2, 3, 8):
            s = shard.count_shards(count, world)
            assert sum(n for _, n in s) == count
            assert all(s[i][0] + s[i][1] == s[i + 1][0] for i in range(world - 1))
            assert max(n for _, n in s) - min(n for _, n in s) <= 1


def test_position_shards():
    for total in (0, 5, 4096, 100003):
        for world in (1, 2, 8):
            for g in (1, 4, 8):
                s = shard.position_shards(total, world, g)
                assert sum(n for _, n in s) == total
                assert all(a % g == 0 for a, n in s if n)


def _oinfo(recipe):
    from tests import recipes as R
    i = R.Built(recipe).o.info()
    return i["size"], i["ub"] - i["lb"]


SPLIT_CASES = [
    # count > 1: top-level count split (cfg2/cfg3 shape)
    (("resized", ("vector", 16, 1, 8, ("basic", 16)), 0, 1024), 7),
    # count 1: outer-loop split of an hvector of structs (cfg5 shape) and of a vector
    (("hvector", 1001, 1, 32, ("struct", [1, 3], [0, 8], [("basic", 16), ("basic", 6)])), 1),
    (("vector", 999, 3, 5, ("basic", 15)), 1),
    # count 1: index-prefix split (cfg4 shape: unique LCG displacements) and variable lengths
    (("indexed_block", 1, [(1664525 * i + 1013904223) % 4099 for i in range(1500)], ("basic", 15)), 1),
    (("indexed", [1 + (i * 7) % 5 for i in range(800)], [i * 11 for i in range(800)], ("basic", 16)), 1),
]


@pytest.mark.parametrize("case", range(len(SPLIT_CASES)))
@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_split_recipe_shards_concatenate_to_the_message(case, world):
    """SURVEY.md §8e partitioning: each rank's (recipe, count, user offset) packs exactly
    its byte range of the whole stream; the ranges tile the stream in rank order, and the
    shards' unpacks together rebuild the whole unpack (oracle on both sides)."""
    from tests import recipes as R
    rec, count = SPLIT_CASES[case]
    b = R.Built(rec)
    info = b.o.info()
    total = info["size"] * count
    span, origin = R.layout(info, count)
    host = R.fill(span, 9)
    whole = b.o.pack(count, host, origin, 0, total, element_granular=False)
    parts, pos = [], 0
    out = np.full(span, 0xA5, dtype=np.uint8)
    for r in range(world):
        sr, n, uoff, poff = shard.split_recipe(rec, count, r, world, info=_oinfo)
        assert poff == pos
        sb = R.Built(sr)
        ln = sb.o.info()["size"] * n
        part = sb.o.pack(n, host, origin + uoff, 0, ln, element_granular=False) if ln else b""
        parts.append(part)
        if ln:
            sb.o.unpack(n, out, origin + uoff, 0, part)
        pos += ln
    assert pos == total and b"".join(parts) == whole
    want = np.full(span, 0xA5, dtype=np.uint8)
    b.o.unpack(count, want, origin, 0, whole)
    np.testing.assert_array_equal(out, want)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    try:
        import torch
        import torch.distributed as dist
        from tests import recipes as R
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        # 32^3 float subarray face stack (BASELINE config 3 shape, scaled), 7 fields
        rec = ("resized", ("subarray", [32, 32, 32], [32, 32, 1], [0, 0, 31], 0, ("basic", 15)),
               0, 32 ** 3 * 4)
        b = R.Built(rec)
        info = b.o.info()
        count = 7   # uneven split over 2 and 3 ranks
        span, origin = R.layout(info, count)
        host = R.fill(span, 42)
        first, n, uoff, poff = shard.shard_of(count, info["size"], info["ub"] - info["lb"], rank, world)
        part = b.o.pack(n, host, origin + uoff, 0, n * info["size"], element_granular=False)
        full = shard.gather_packed(torch.from_numpy(np.frombuffer(part, dtype=np.uint8).copy()))
        if rank == 0:
            ref = b.o.pack(count, host, origin, 0, count * info["size"], element_granular=False)
            q.put(bytes(full.numpy().tobytes()) == ref)
        dist.barrier()
        dist.destroy_process_group()
    except Exception as ex:  # surface failures to the parent
        q.put(repr(ex))


@pytest.mark.parametrize("world", [2, 3])   # 3 ranks: uneven count split
def test_gather_of_shards_equals_whole_message_gloo(world):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    res = q.get(timeout=10)
    assert res is True, res
