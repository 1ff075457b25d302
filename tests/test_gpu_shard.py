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
