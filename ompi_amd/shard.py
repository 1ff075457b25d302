"""Multi-GPU sharding of one datatype message.

For a homogeneous type the packed offset of top-level instance i is exactly i*size, so
shard k of G owns instances [first_k, first_k + n_k) and writes packed bytes
[first_k*size, (first_k+n_k)*size) -- no exchange is needed to pack.  This is the
same partition the reference applies with opal_convertor_set_position for multi-BTL
scheduling (pml_ob1_sendreq.c:1184-1194).  A consumer that needs the whole packed
stream on one device gets it with one all-gather of equal-size shards (RCCL over
xGMI on GPUs; gloo in the CPU tests).
"""
from __future__ import annotations

from typing import List, Tuple


def count_shards(count: int, world: int) -> List[Tuple[int, int]]:
    """Balanced split of `count` top-level instances: [(first, n)] per rank."""
    if world <= 0:
        raise ValueError("world must be positive")
    base, rem = divmod(count, world)
    out, first = [], 0
    for r in range(world):
        n = base + (1 if r < rem else 0)
        out.append((first, n))
        first += n
    return out


def position_shards(total: int, world: int, granule: int = 1) -> List[Tuple[int, int]]:
    """Split the packed stream [0, total) into `world` byte ranges on `granule` boundaries
    (opal_convertor_set_position-style sharding of a count-1 type)."""
    per = -(-total // world)
    per = -(-per // granule) * granule
    out = []
    for r in range(world):
        a = min(r * per, total)
        b = min(a + per, total)
        out.append((a, b - a))
    return out


def shard_of(count: int, size: int, extent: int, rank: int, world: int):
    """(first instance, n instances, user byte offset, packed byte offset) of `rank`."""
    first, n = count_shards(count, world)[rank]
    return first, n, first * extent, first * size


def pack_shard(dt, count: int, buf, rank: int, world: int, out, stream=None) -> int:
    """Pack this rank's instances of a `count`-instance message at `buf` into `out`
    (a buffer of n*size bytes).  Returns the bytes packed."""
    from .convertor import addr, pack_window
    info = dt.info()
    size, extent = info["size"], info["ub"] - info["lb"]
    first, n, uoff, poff = shard_of(count, size, extent, rank, world)
    if n == 0:
        return 0
    return pack_window(dt, n, addr(buf) + uoff, 0, out, n * size, stream=stream)


def _engine_info(recipe):
    from .recipe import build_committed
    i = build_committed(recipe).info()
    return i["size"], i["ub"] - i["lb"]


def split_recipe(recipe, count: int, rank: int, world: int, info=_engine_info):
    """This rank's share of a `count`-instance message of `recipe`, as a message of its own:
    (recipe_r, count_r, user_offset, packed_offset).  Packing recipe_r x count_r at
    buf + user_offset produces bytes [packed_offset, packed_offset + len) of the whole
    message's stream, so the shards concatenate to it with no exchange.

      count > 1             -> split the top-level count (instances first .. first+n)
      vector / hvector x 1  -> split the outer loop (blocks first .. first+n)
      indexed* x 1          -> split the index list by the prefix sum of block lengths
    The reference's own precedent is ob1's multi-BTL scheduling, which hands each BTL a
    byte range through opal_convertor_set_position (pml_ob1_sendreq.c:1184-1194).  Other
    count-1 shapes return None: the caller shards the byte stream with position_shards and
    windows (ddt_pack_window).  `info(recipe) -> (size, extent)`."""
    if count > 1 or count == 0:
        size, ext = info(recipe)
        first, n = count_shards(count, world)[rank]
        return recipe, n, first * ext, first * size
    k = recipe[0]
    if k in ("vector", "hvector"):
        _, cnt, blen, stride, sub = recipe
        ssize, sext = info(sub)
        first, n = count_shards(cnt, world)[rank]
        step = stride * sext if k == "vector" else stride
        return (k, n, blen, stride, sub), 1, first * step, first * blen * ssize
    if k in ("indexed_block", "hindexed_block"):
        _, blen, disps, sub = recipe
        ssize, _ = info(sub)
        first, n = count_shards(len(disps), world)[rank]
        return (k, blen, disps[first:first + n], sub), 1, 0, first * blen * ssize
    if k in ("indexed", "hindexed"):
        _, blens, disps, sub = recipe
        ssize, _ = info(sub)
        total = sum(blens)
        # block boundaries nearest to r * total / world (prefix sum of lengths)
        bounds, acc, r = [0], 0, 1
        for i, b in enumerate(blens):
            acc += b
            while r < world and acc * world >= r * total:
                bounds.append(i + 1)
                r += 1
        while len(bounds) < world + 1:
            bounds.append(len(blens))
        a, c = bounds[rank], bounds[rank + 1]
        return (k, blens[a:c], disps[a:c], sub), 1, 0, sum(blens[:a]) * ssize
    return None


def gather_packed(local, group=None):
    """All-gather equal-size packed shards into the full stream (torch.distributed;
    backend 'nccl' is RCCL on ROCm).  `local` is a 1-D uint8 tensor; shards are padded to
    the largest one and trimmed by the caller with `count_shards`."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    n = torch.tensor([local.numel()], device=local.device, dtype=torch.int64)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n, group=group)
    lens = [int(s.item()) for s in sizes]
    mx = max(lens)
    if all(x == mx for x in lens):
        # equal shards (the weak-scaling bench, an even split): gather in place, no padding copies
        out = torch.empty(world * mx, dtype=local.dtype, device=local.device)
        dist.all_gather_into_tensor(out, local.contiguous(), group=group)
        return out
    buf = torch.zeros(mx, dtype=local.dtype, device=local.device)
    buf[:local.numel()] = local
    out = torch.empty(world * mx, dtype=local.dtype, device=local.device)
    dist.all_gather_into_tensor(out, buf, group=group)
    parts = [out[r * mx: r * mx + lens[r]] for r in range(world)]
    return torch.cat(parts)
