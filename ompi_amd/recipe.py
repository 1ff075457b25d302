"""Build engine datatypes from nested-tuple type descriptions.

    ("basic", opal_id) | ("contig", n, sub) | ("vector", n, blen, stride, sub)
    ("hvector", n, blen, stride_bytes, sub) | ("indexed", blens, disps, sub)
    ("hindexed", blens, disps, sub) | ("indexed_block", blen, disps, sub)
    ("hindexed_block", blen, disps, sub) | ("struct", blens, disps, [subs])
    ("subarray", sizes, subsizes, starts, order, sub) | ("resized", sub, lb, extent)
  | ("darray", size, rank, gsizes, distribs, dargs, psizes, order, sub)
    ("dup", sub)

Each constructor maps 1:1 to ompi_datatype_create_* (ompi/datatype/ompi_datatype.h:217-284).
The same tuple object used twice builds one datatype (struct's same-type merge compares
handles, ompi_datatype_create_struct.c:55-58).
"""
from __future__ import annotations

from . import datatype as D


def build(recipe, memo=None):
    memo = {} if memo is None else memo
    key = id(recipe)
    if key in memo:
        return memo[key][0]
    k = recipe[0]
    if k == "basic":
        t = D.predefined(recipe[1])
        memo[key] = (t, recipe)
        return t
    sub = lambda r: build(r, memo)  # noqa: E731
    if k == "contig":
        t = D.create_contiguous(recipe[1], sub(recipe[2]))
    elif k == "vector":
        t = D.create_vector(recipe[1], recipe[2], recipe[3], sub(recipe[4]))
    elif k == "hvector":
        t = D.create_hvector(recipe[1], recipe[2], recipe[3], sub(recipe[4]))
    elif k == "indexed":
        t = D.create_indexed(recipe[1], recipe[2], sub(recipe[3]))
    elif k == "hindexed":
        t = D.create_hindexed(recipe[1], recipe[2], sub(recipe[3]))
    elif k == "indexed_block":
        t = D.create_indexed_block(recipe[1], recipe[2], sub(recipe[3]))
    elif k == "hindexed_block":
        t = D.create_hindexed_block(recipe[1], recipe[2], sub(recipe[3]))
    elif k == "struct":
        t = D.create_struct(recipe[1], recipe[2], [sub(r) for r in recipe[3]])
    elif k == "subarray":
        t = D.create_subarray(recipe[1], recipe[2], recipe[3], recipe[4], sub(recipe[5]))
    elif k == "darray":
        t = D.create_darray(*recipe[1:8], sub(recipe[8]))
    elif k == "resized":
        t = D.create_resized(sub(recipe[1]), recipe[2], recipe[3])
    elif k == "dup":
        t = D.duplicate(sub(recipe[1]))
    else:
        raise ValueError(f"unknown constructor {k!r}")
    memo[key] = (t, recipe)
    return t


def build_committed(recipe):
    """Build and commit; the returned type keeps its sub-types alive (and frees them with it)."""
    memo: dict = {}
    t = build(recipe, memo)
    t.commit()
    t.subtypes = tuple(v[0] for v in memo.values() if v[0] is not t)
    return t
