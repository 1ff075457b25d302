"""bench.py's multi-rank harness on CPU (gloo, world size 2): the self-launch command of
`--gpus N`, the timed region (barrier + synchronize on both sides, wall time max over ranks)
and the post-run all-gather check of the packed shards.  The GPU run of the same harness is
test_gpu_bench.py (two ranks self-launched on one GPU)."""
from __future__ import annotations

import os
import time

import pytest

import bench


def test_self_launch_argv_is_one_rank_per_gpu_on_localhost():
    argv = bench.self_launch_argv(8, ["--gpus", "8", "--steps", "5"], 29555)
    assert argv[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in argv and "--nnodes=1" in argv
    assert "--master-addr=127.0.0.1" in argv and "--master-port=29555" in argv
    i = argv.index(os.path.abspath(bench.__file__))
    assert argv[i + 1:] == ["--gpus", "8", "--steps", "5"]


def _worker(rank, world, port, q):
    try:
        import torch
        import torch.distributed as dist
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        calls = []

        def step(i):   # rank 1 is the slow rank: 20 ms per step
            calls.append(i)
            time.sleep(0.02 if rank == 1 else 0.001)

        def reduce_max(x):
            t = torch.tensor([x], dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            return float(t.item())

        wall = bench.timed_region(step, 5, world, lambda: None, reduce_max, dist.barrier)
        # shards of different sizes and contents, like a count split over the ranks
        S = 4000 if rank == 0 else 3000
        packed = torch.arange(S, dtype=torch.int64).to(torch.uint8) + rank
        chk = bench.gather_check(packed, S, world, rank, torch.device("cpu"), "gloo")
        pr = bench.per_rank_times(0.001 * (rank + 1), 0.002 * (rank + 1), world, torch.device("cpu"), "gloo")
        q.put((rank, calls, wall, (chk, pr)))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as ex:  # surface failures to the parent
        q.put((rank, repr(ex), None, None))


@pytest.mark.parametrize("world", [2, 4])
def test_timed_region_and_gather_check_gloo(world):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = bench.free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    total = 4000 + 3000 * (world - 1)
    for rank, calls, wall, extra in res:
        assert calls == list(range(5)), calls
        chk, pr = extra
        # every rank reports the slow rank's time (max over ranks), >= 5 x 20 ms
        assert wall >= 0.1
        assert chk["ok"] and chk["gathered_bytes"] == total and chk["backend"] == "gloo"
        # per-rank event times in rank order, min / max over ranks
        assert pr["ranks"] == [[round(1.0 * (r + 1), 4), round(2.0 * (r + 1), 4)] for r in range(world)]
        assert pr["pack"] == {"min": 1.0, "max": 1.0 * world}
        assert pr["unpack"] == {"min": 2.0, "max": 2.0 * world}
    assert len({r[2] for r in res}) == 1


@pytest.mark.parametrize("cfg", ["cfg1", "cfg2", "cfg3"])
def test_floor_parts_move_exactly_the_workloads_bytes(cfg):
    """bench.py's floor (bare kernels, ompi_amd/csrc/ddt_floor.hip) is priced on the workload's
    own accesses: the user-side runs of its parts are exactly the type map's runs of `count`
    instances (as sets of (offset, bytes)), and together they produce S packed bytes."""
    import numpy as np
    from ompi_amd import recipe as ER
    from tests import plan_emu as E
    rec, count, _ = bench.make_workload(cfg)
    t = ER.build_committed(rec)
    info = t.info()
    ext = info["ub"] - info["lb"]
    blk = E.engine_blocks(t)                    # (src, dst, len) of one instance
    want = np.concatenate([blk[:, 0] + i * ext for i in range(count)])
    wlen = np.tile(blk[:, 2], count)
    got, glen = [], []
    for _, kind, es, ls, ss, base, lw in bench.floor_parts(cfg):
        i0 = np.arange(1 << ls[0], dtype=np.int64)
        i1 = np.arange(1 << ls[1], dtype=np.int64)
        i2 = np.arange(1 << ls[2], dtype=np.int64)
        off = (base + i2[:, None, None] * ss[2] + i1[None, :, None] * ss[1] + i0[None, None, :] * ss[0]).reshape(-1)
        got.append(off)
        glen.append(np.full(off.size, es if kind == 0 else 16 << lw, dtype=np.int64))
    got, glen = np.concatenate(got), np.concatenate(glen)
    assert int(glen.sum()) == info["size"] * count

    es = 8 if cfg != "cfg3" else 4   # the workload's element size: compare element multisets

    def elements(o, n):   # faces share edge elements, so compare with multiplicity
        reps = n // es
        starts = np.repeat(o, reps)
        k = np.arange(reps.sum(), dtype=np.int64) - np.repeat(np.cumsum(reps) - reps, reps)
        return np.sort(starts + k * es)
    np.testing.assert_array_equal(elements(want, wlen), elements(got, glen))


def test_floor_parts_of_cfg4_and_cfg5():
    """The floors of BASELINE configs 4 and 5: config 5's record part is the
    hvector's type map (128 Mi records of 20 bytes at a 32-byte pitch, S packed bytes); config 4's
    listed part moves every element of the indexed type once (its 64 Mi displacements, S bytes)
    and its permutation pass runs between scratch buffers of S bytes, outside the packed count."""
    rec5, count5, _ = bench.make_workload("cfg5")
    (label, kind, es, ls, ss, base, lw), = bench.floor_parts("cfg5")
    n = 1 << sum(ls)
    assert kind == 2 and (n, es, ss[0], base) == (rec5[1], 20, rec5[3], 0)
    from ompi_amd import recipe as ER
    i5 = ER.build_committed(("hvector", 64, 1, 32, rec5[4])).info()
    assert i5["size"] == 64 * 20 and n * es * count5 == (128 << 20) * 20
    rec4, count4, _ = bench.make_workload("cfg4")
    parts = bench.floor_parts("cfg4")
    lst = [p for p in parts if len(p) > 7 and p[7].get("list")]
    scr = [p for p in parts if len(p) > 7 and p[7].get("scratch")]
    assert len(lst) == 1 and len(scr) == 1
    assert lst[0][7]["count"] == len(rec4[2]) and lst[0][2] == 4 and rec4[1] == 1
    S = len(rec4[2]) * 4
    assert scr[0][7]["scratch"] == S == (1 << sum(scr[0][3])) * (16 << scr[0][6])


def test_strong_cfg3_over_eight_ranks_covers_all_64_fields():
    """The driver's 8-GPU strong run of BASELINE config 3 (`--gpus 8 --strong --config cfg3`): the
    self-launch command is one rank per GPU with the same arguments, and the eight ranks' splits
    (ompi_amd.shard.split_recipe by top-level count) take 8 fields each, in order, their packed
    ranges tiling the whole 64-field stream."""
    from ompi_amd import shard
    argv = bench.self_launch_argv(8, ["--gpus", "8", "--strong", "--config", "cfg3"], 29600)
    assert "--nproc-per-node=8" in argv
    i = argv.index(os.path.abspath(bench.__file__))
    assert argv[i + 1:] == ["--gpus", "8", "--strong", "--config", "cfg3"]
    recipe, count, _ = bench.make_workload("cfg3")
    field_size = shard._engine_info(recipe)[0]
    total, first_pk = 0, 0
    for rank in range(8):
        rrec, rcount, uoff, poff = shard.split_recipe(recipe, 64, rank, 8)
        assert rrec == recipe and rcount == 8
        assert poff == first_pk and uoff == rank * 8 * shard._engine_info(recipe)[1]
        first_pk += rcount * field_size
        total += rcount
    assert total == 64 and first_pk == 64 * field_size


def test_gather_packed_equal_shards_skip_padding():
    """shard.gather_packed with equal shards gathers in place (gloo, world 1 here: the same code
    path as the equal-size branch) and returns the concatenation."""
    import torch
    import torch.distributed as dist
    from ompi_amd import shard
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29611")
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        x = torch.arange(100, dtype=torch.uint8)
        assert torch.equal(shard.gather_packed(x), x)
    finally:
        dist.destroy_process_group()


def test_touched_lines_counts_128_byte_lines():
    """bench.line_floor's line count (the engine's raw iovec export on a NULL base): known answers
    -- a 300-byte contiguous run from 0 touches 3 lines; vector(4,1,32) of double (one element per
    256 bytes) 4; vector(4,2,8) of double (16 B every 64 B, 256 B span) 2; two instances of a
    type whose extent is half a line share lines; cfg2's halo: 2 x-face lines per row plus the y
    rows and z planes, shared edge lines counted once."""
    from ompi_amd import recipe as ER
    D = ("basic", 16)
    cases = [(("contig", 300, ("basic", 4)), 1, 3),
             (("vector", 4, 1, 32, D), 1, 4),
             (("vector", 4, 2, 8, D), 1, 2),
             (("resized", ("contig", 8, D), 0, 64), 4, 2)]
    for rec, count, want in cases:
        assert bench.touched_lines(ER.build_committed(rec), count) == want, rec
    rec, count, _ = bench.make_workload("cfg2")
    n, lpr = 256, 256 * 8 // 128                    # 16 lines per 2 KiB row
    x, y, z = 2 * n * n, 2 * n * lpr, 2 * n * lpr     # x: a line per row; y: 2 x 256 rows; z: 2 planes
    xy, xz, yz, xyz = 2 * n * 2, 2 * n * 2, 2 * 2 * lpr, 2 * 2 * 2   # lines the faces share
    per_field = x + y + z - xy - xz - yz + xyz        # inclusion-exclusion: 145,352
    assert bench.touched_lines(ER.build_committed(rec), count) == count * per_field
