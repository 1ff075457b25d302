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
        # shards of different sizes and contents, like a count split 7 over 2 ranks
        S = 4000 if rank == 0 else 3000
        packed = torch.arange(S, dtype=torch.int64).to(torch.uint8) + rank
        chk = bench.gather_check(packed, S, world, rank, torch.device("cpu"), "gloo")
        q.put((rank, calls, wall, chk))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as ex:  # surface failures to the parent
        q.put((rank, repr(ex), None, None))


def test_timed_region_and_gather_check_world2_gloo():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = bench.free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    for rank, calls, wall, chk in res:
        assert calls == list(range(5)), calls
        # both ranks report the slow rank's time (max over ranks), >= 5 x 20 ms
        assert wall >= 0.1
        assert chk["ok"] and chk["gathered_bytes"] == 7000 and chk["backend"] == "gloo"
    assert res[0][2] == res[1][2]
