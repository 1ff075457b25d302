"""Datatype recipes: one description, built both by the CPU oracle and by the HIP engine.

A recipe is a nested tuple:
    ("basic", opal_id)
    ("contig", count, sub)
    ("vector", count, blocklen, stride, sub)          ompi_datatype_create_vector
    ("hvector", count, blocklen, stride_bytes, sub)
    ("indexed", blocklens, disps, sub) / ("hindexed", ...)
    ("indexed_block", blocklen, disps, sub) / ("hindexed_block", ...)
    ("struct", blocklens, disps, [subs])
    ("subarray", sizes, subsizes, starts, order, sub)
    ("resized", sub, lb, extent)
    ("dup", sub)
The same Python object used twice inside a recipe builds ONE datatype (struct's
same-type merge compares handles, ompi_datatype_create_struct.c:55).
"""
from __future__ import annotations

import random
from typing import Any

import numpy as np

from . import oracle as O

# (opal id, size) of the basic types the fuzzer draws from
BASICS = [(4, 1), (5, 2), (6, 4), (15, 4), (16, 8), (7, 8), (21, 16), (11, 4), (9, 1)]
# every type with an external32 form: adds INT16, FLOAT2, the complex types, BOOL, WCHAR,
# LONG and UNSIGNED_LONG (size-changing), the long doubles (FLOAT12 = MPI_LONG_DOUBLE, FLOAT16 =
# _Float128, LONG_DOUBLE_COMPLEX converted x87 <-> IEEE quad)
EXT_BASICS = BASICS + [(8, 16), (14, 2), (19, 4), (20, 8), (23, 1), (24, 4), (25, 8), (26, 8),
                       (12, 8), (10, 2), (17, 16), (18, 16), (22, 32)]


def build_oracle(recipe, memo=None):
    memo = {} if memo is None else memo
    key = id(recipe)
    if key in memo:
        return memo[key][0]
    k = recipe[0]
    if k == "basic":
        # predefined handles are unique per id
        bk = ("basic", recipe[1])
        if bk in memo:
            return memo[bk][0]
        t = O.basic(recipe[1])
        memo[bk] = (t, recipe)
        return t
    sub = lambda r: build_oracle(r, memo)  # noqa: E731
    if k == "contig":
        t = O.contiguous(recipe[1], sub(recipe[2]))
    elif k == "vector":
        t = O.vector(recipe[1], recipe[2], recipe[3], sub(recipe[4]))
    elif k == "hvector":
        t = O.hvector(recipe[1], recipe[2], recipe[3], sub(recipe[4]))
    elif k == "indexed":
        t = O.indexed(recipe[1], recipe[2], sub(recipe[3]))
    elif k == "hindexed":
        t = O.hindexed(recipe[1], recipe[2], sub(recipe[3]))
    elif k == "indexed_block":
        t = O.indexed_block(recipe[1], recipe[2], sub(recipe[3]))
    elif k == "hindexed_block":
        t = O.hindexed_block(recipe[1], recipe[2], sub(recipe[3]))
    elif k == "struct":
        t = O.struct(recipe[1], recipe[2], [sub(r) for r in recipe[3]])
    elif k == "subarray":
        t = O.subarray(recipe[1], recipe[2], recipe[3], recipe[4], sub(recipe[5]))
    elif k == "darray":
        t = O.darray(*recipe[1:8], sub(recipe[8]))
    elif k == "resized":
        t = O.resized(sub(recipe[1]), recipe[2], recipe[3])
    elif k == "dup":
        t = O.dup(sub(recipe[1]))
    else:
        raise ValueError(k)
    memo[key] = (t, recipe)   # keep recipe alive so id() stays unique
    return t


def build_engine(recipe, memo=None):
    from ompi_amd import recipe as ER
    return ER.build(recipe, memo)


class Built:
    """Oracle type + engine type of one recipe (keeps every sub-type alive)."""

    def __init__(self, recipe):
        self.recipe = recipe
        self.omemo: dict = {}
        self.ememo: dict = {}
        self.o = build_oracle(recipe, self.omemo)
        self.e = None

    def engine(self):
        if self.e is None:
            self.e = build_engine(self.recipe, self.ememo)
            self.e.commit()
        return self.e


def layout(info: dict, count: int):
    """Byte range touched by `count` instances (opt_desc_equiv.c:330-356).

    Returns (span, origin): a buffer of `span` bytes whose byte `origin` is the type
    origin (the pointer handed to pack/unpack)."""
    size = info["size"]
    ext = info["ub"] - info["lb"]
    tlb, tub = info["true_lb"], info["true_ub"]
    if size == 0:
        return 16, 0
    lo = hi = None
    for i in (0, count - 1):
        s = tlb + i * ext
        e = tub + i * ext
        lo = s if lo is None else min(lo, s)
        hi = e if hi is None else max(hi, e)
    span = max(hi - lo, 1)
    return span, -lo


def fill(n: int, seed: int) -> np.ndarray:
    """Position hash with no zero bytes."""
    idx = np.arange(n, dtype=np.uint64)
    h = (idx + np.uint64(seed)) * np.uint64(0x9E3779B97F4A7C15)
    b = ((h >> np.uint64(29)) & np.uint64(0xFF)).astype(np.uint8)
    return np.where(b == 0, np.uint8(0x5A), b)


def fill_fast(n: int, seed: int) -> np.ndarray:
    """Random non-zero bytes for buffers of hundreds of MiB (fill() needs 8 bytes of
    temporaries per byte)."""
    return np.random.default_rng(seed).integers(1, 256, size=n, dtype=np.uint8)


# ------------------------------------------------------------------ fuzzing
def random_recipe(rng: random.Random, depth: int = 0, basics=None) -> Any:
    basics = basics or BASICS
    if depth >= 3 or rng.random() < 0.25:
        return ("basic", rng.choice(basics)[0])
    k = rng.choice(["contig", "vector", "vector", "hvector", "indexed", "hindexed",
                    "indexed_block", "hindexed_block", "struct", "struct", "subarray",
                    "resized", "dup"])
    sub = random_recipe(rng, depth + 1, basics)
    if k == "contig":
        return ("contig", rng.randint(1, 5), sub)
    if k == "vector":
        return ("vector", rng.randint(1, 6), rng.randint(0, 4), rng.choice([-3, -1, 1, 2, 3, 5, 7]), sub)
    if k == "hvector":
        return ("hvector", rng.randint(1, 6), rng.randint(0, 3), rng.choice([-40, -8, 4, 8, 12, 24, 40, 100]), sub)
    if k in ("indexed", "hindexed"):
        n = rng.choice([1, 2, 3, 5, 12, 20])
        bl = [rng.randint(0, 3) for _ in range(n)]
        if k == "indexed":
            ds = [rng.randint(-4, 12) for _ in range(n)]
        else:
            ds = [rng.randint(-40, 120) for _ in range(n)]
        if rng.random() < 0.5:   # sorted, abutting runs exercise the merge rule
            ds = sorted(ds)
        return (k, bl, ds, sub)
    if k in ("indexed_block", "hindexed_block"):
        n = rng.choice([1, 3, 9, 16])
        ds = [rng.randint(-4, 12) if k == "indexed_block" else rng.randint(-40, 120) for _ in range(n)]
        return (k, rng.randint(0, 3), ds, sub)
    if k == "struct":
        n = rng.randint(1, 4)
        subs = [sub] + [random_recipe(rng, depth + 1, basics) for _ in range(n - 1)]
        if n > 1 and rng.random() < 0.3:
            subs[1] = subs[0]   # same handle: exercises the struct merge
        return ("struct", [rng.randint(0, 3) for _ in range(n)],
                [rng.randint(-16, 64) for _ in range(n)], subs)
    if k == "subarray":
        nd = rng.randint(1, 3)
        sizes = [rng.randint(1, 5) for _ in range(nd)]
        subs_ = [rng.randint(1, s) for s in sizes]
        starts = [rng.randint(0, s - ss) for s, ss in zip(sizes, subs_)]
        return ("subarray", sizes, subs_, starts, rng.randint(0, 1), sub)
    if k == "resized":
        return ("resized", sub, rng.randint(-8, 8), rng.choice([-16, 0, 4, 8, 24, 64, 96]))
    return ("dup", sub)


def random_mixed_recipe(rng: random.Random, depth: int = 0) -> Any:
    """Recipes whose type maps put elements of different types side by side -- the regions
    opal_datatype_commit fuses and re-types to UINT8/4/2/1 carriers
    (opal_datatype_optimize.c:581-630, :1195-1199, :1250-1252) -- nested in the loops its
    boundary fusion, compression, short-loop expansion and unrolling act on (:641-888, :1054-1122).
    Structs are mostly packed (member i+1 starts where member i ends, or 1-3 bytes later), so
    the merges and the carriers' alignment rules are exercised at every byte phase."""
    if depth >= 3 or (depth > 0 and rng.random() < 0.2):
        return ("basic", rng.choice(EXT_BASICS[:16])[0])
    k = rng.choice(["struct", "struct", "struct", "vector", "hvector", "contig", "resized",
                    "hindexed", "indexed_block"])
    if k == "struct":
        n = rng.randint(2, 5)
        subs = [random_mixed_recipe(rng, depth + 1) for _ in range(n)]
        built = [build_oracle(s) for s in subs]
        blens = [rng.randint(1, 3) for _ in range(n)]
        disps, at = [], rng.choice([0, 0, 1, 2, 4])
        for b, t in zip(blens, built):
            disps.append(at)
            ext = t.extent if t.size else 1
            at += b * ext + (rng.choice([0, 0, 0, 1, 2, 3, 4, 8]) if rng.random() < 0.4 else 0)
        return ("struct", blens, disps, subs)
    sub = random_mixed_recipe(rng, depth + 1)
    t = build_oracle(sub)
    ext = t.extent if t.size else 1
    if k == "vector":
        return ("vector", rng.randint(2, 9), rng.randint(1, 3), rng.choice([1, 2, 3, 4]), sub)
    if k == "hvector":
        return ("hvector", rng.randint(2, 9), rng.randint(1, 2),
                rng.choice([ext, ext, ext + 4, ext + 8, 2 * ext, ext * 3 + 1]), sub)
    if k == "contig":
        return ("contig", rng.randint(2, 6), sub)
    if k == "resized":
        return ("resized", sub, 0, rng.choice([t.size, t.size, ext + 4, max(t.size, 1) * 2]))
    if k == "hindexed":
        n = rng.randint(2, 10)
        ds, at = [], 0
        bl = [rng.randint(1, 2) for _ in range(n)]
        for b in bl:
            ds.append(at)
            at += b * ext + rng.choice([0, ext, 4, 8])
        return ("hindexed", bl, ds, sub)
    n = rng.randint(2, 10)
    return ("indexed_block", rng.randint(1, 2), sorted(rng.sample(range(0, 3 * n), n)), sub)
