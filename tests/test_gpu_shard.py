"""Multi-rank sharding with the GPU engine on every rank.

Two and three ranks share cuda:0 (the one-GPU box) and exchange over gloo on host tensors,
so no RCCL is needed: each rank packs its instance range of one message with the HIP
engine (shard.pack_shard -> ddt_pack_window), the shards are all-gathered, and the
concatenation must equal the oracle's whole-message stream.  Each rank then unpacks its
own slice of that stream into a 0xA5-filled device buffer and checks it against the
oracle's unpack of the same instances.
"""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


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
        import ompi_amd
        from ompi_amd import shard
        from ompi_amd.convertor import unpack_window
        from tests import recipes as R
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        import datetime
        dist.init_process_group("gloo", rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=60))
        dev = torch.device("cuda:0")
        # 64^3 float subarray x-face stack (BASELINE config 3 shape, scaled), 7 fields
        n3 = 64
        rec = ("resized", ("subarray", [n3, n3, n3], [n3, n3, 1], [0, 0, n3 - 1], 0, ("basic", 15)),
               0, n3 ** 3 * 4)
        b = R.Built(rec)
        e = b.engine()
        info = b.o.info()
        size, ext = info["size"], info["ub"] - info["lb"]
        count = 7
        span, origin = R.layout(info, count)
        host = R.fill(span, 42)
        user = torch.from_numpy(host).to(dev)
        first, n, uoff, poff = shard.shard_of(count, size, ext, rank, world)
        local = torch.zeros(max(n * size, 1), dtype=torch.uint8, device=dev)
        got = shard.pack_shard(e, count, user.data_ptr() + origin, rank, world, local)
        assert got == n * size, (got, n * size)
        torch.cuda.synchronize()
        full = shard.gather_packed(local[:n * size].cpu())
        ref = np.frombuffer(b.o.pack(count, host, origin, 0, count * size, element_granular=False),
                            dtype=np.uint8)
        assert np.array_equal(full.numpy(), ref), "gathered shards != oracle stream"
        # unpack this rank's slice of the whole stream
        out = torch.full((span,), 0xA5, dtype=torch.uint8, device=dev)
        if n:
            src = torch.from_numpy(ref[poff:poff + n * size].copy()).to(dev)
            unpack_window(e, n, out.data_ptr() + origin + uoff, 0, src, n * size)
        torch.cuda.synchronize()
        exp = np.full(span, 0xA5, dtype=np.uint8)
        if n:
            b.o.unpack(n, exp, origin + uoff, 0, ref[poff:poff + n * size].tobytes())
        assert np.array_equal(out.cpu().numpy(), exp), "unpacked shard != oracle"
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, True))
    except Exception as ex:  # surface failures to the parent
        q.put((rank, repr(ex)))


def _split_worker(rank, world, port, q, case):
    """count = 1 messages split with shard.split_recipe: each rank commits ITS part (the
    outer loop's blocks first..first+n, or its prefix of the index list) and packs it with
    the HIP engine; gathered shards == the oracle's whole stream; each rank's unpack of its
    part == the oracle's unpack of the same part."""
    try:
        import datetime
        import torch
        import torch.distributed as dist
        from ompi_amd import recipe as ER
        from ompi_amd import shard
        from ompi_amd.convertor import pack, unpack
        from tests import recipes as R
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=60))
        dev = torch.device("cuda:0")
        if case == "hvector":   # cfg5 shape, 256 Ki records
            rec = ("hvector", 1 << 18, 1, 32, ("struct", [1, 3], [0, 8], [("basic", 16), ("basic", 6)]))
        else:                   # cfg4 shape: 1 Mi unique LCG displacements into 64 MiB
            d, x = [], 0x5EED
            for _ in range(1 << 20):
                d.append(x)
                x = (1664525 * x + 1013904223) & ((1 << 24) - 1)
            rec = ("indexed_block", 1, d, ("basic", 15))
        b = R.Built(rec)
        info = b.o.info()
        span, origin = R.layout(info, 1)
        host = R.fill_fast(span, 5)
        user = torch.from_numpy(host).to(dev)
        sr, n, uoff, poff = shard.split_recipe(rec, 1, rank, world)
        st = ER.build_committed(sr)
        ln = st.info()["size"] * n
        local = torch.zeros(max(ln, 1), dtype=torch.uint8, device=dev)
        if ln:
            assert pack(user.data_ptr() + origin + uoff, n, st, local, ln, 0) == ln
        torch.cuda.synchronize()
        full = shard.gather_packed(local[:ln].cpu())
        ref = np.frombuffer(b.o.pack(1, host, origin, 0, info["size"], element_granular=False), dtype=np.uint8)
        assert np.array_equal(full.numpy(), ref), "gathered shards != oracle stream"
        out = torch.full((span,), 0xA5, dtype=torch.uint8, device=dev)
        if ln:
            unpack(local, ln, 0, out.data_ptr() + origin + uoff, n, st)
        torch.cuda.synchronize()
        exp = np.full(span, 0xA5, dtype=np.uint8)
        if ln:
            R.Built(sr).o.unpack(n, exp, origin + uoff, 0, ref[poff:poff + ln].tobytes())
        assert np.array_equal(out.cpu().numpy(), exp), "unpacked shard != oracle"
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, True))
    except Exception as ex:  # surface failures to the parent
        q.put((rank, repr(ex)))


def _run(target, world, *args):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, q) + args) for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = [q.get(timeout=100) for _ in range(world)]
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    assert all(ok is True for _, ok in res), res


@pytest.mark.parametrize("case", ["hvector", "indexed"])
@pytest.mark.parametrize("world", [2, 3])
def test_gpu_ranks_split_count1_types_gloo(world, case):
    _run(_split_worker, world, case)


@pytest.mark.parametrize("world", [2, 3])
def test_gpu_ranks_shard_pack_unpack_gloo(world):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = [q.get(timeout=100) for _ in range(world)]
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    assert all(ok is True for _, ok in res), res
