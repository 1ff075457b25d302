"""CPU checks of the engine's plan compiler (test infrastructure).

The engine exposes its compiled plan (leaf streams) and the exact launch descriptors
(``Item``, ompi_amd/csrc/ddt_device.h) a pack/unpack would run.  This module
re-executes those descriptors with numpy, following the kernel's index arithmetic
(ompi_amd/csrc/ddt_move.hip.h), so the plan compiler is verified bit-exactly against
the oracle on CPU.  It is a checker only: the product never runs it.
"""
from __future__ import annotations

import ctypes

import numpy as np

from ompi_amd._lib import lib, check

MAXD = 8


class FastDiv(ctypes.Structure):
    _fields_ = [("d", ctypes.c_uint32), ("m", ctypes.c_uint32), ("l", ctypes.c_uint32),
                ("pad", ctypes.c_uint32)]


class Item(ctypes.Structure):
    _fields_ = [
        ("kind", ctypes.c_uint32), ("U", ctypes.c_uint32), ("ndim", ctypes.c_uint32),
        ("idx64", ctypes.c_uint32),
        ("u0", ctypes.c_uint64), ("u1", ctypes.c_uint64), ("units_per_task", ctypes.c_uint64),
        ("task_begin", ctypes.c_uint32), ("ntasks", ctypes.c_uint32),
        ("upb", ctypes.c_uint64), ("fd_upb", FastDiv),
        ("user", ctypes.c_uint64), ("packed", ctypes.c_uint64),
        ("cnt", ctypes.c_uint64 * MAXD), ("fd", FastDiv * MAXD),
        ("ustr", ctypes.c_int64 * MAXD), ("pstr", ctypes.c_int64 * MAXD),
        ("ldisp", ctypes.c_uint64), ("llen", ctypes.c_uint64), ("lgoff", ctypes.c_uint64),
        ("nblk", ctypes.c_uint64), ("fd_nblk", FastDiv), ("ulen", ctypes.c_uint64),
        ("ldisp32", ctypes.c_uint32), ("leaf", ctypes.c_uint32),
        ("same", ctypes.c_uint32), ("nt", ctypes.c_uint32),
        ("w0", ctypes.c_int64), ("w1", ctypes.c_int64), ("nbytes", ctypes.c_uint64),
        ("wt", ctypes.c_uint32), ("slab", ctypes.c_uint32),
    ]


ITEM_AFFINE, ITEM_LIST_UNI, ITEM_LIST_VAR, ITEM_FRAG = 0, 1, 2, 3


def leaves(dt):
    L = lib()
    n = L.ddt_type_plan_leaves(dt.handle, None, 0)
    need = -n if n < 0 else n
    buf = (ctypes.c_int64 * max(need, 1))()
    got = check(L.ddt_type_plan_leaves(dt.handle, buf, need), "plan_leaves")
    vals = list(buf)[:got]
    out, i = [], 0
    while i < len(vals):
        kind, blen, src, dst, nd, idx = vals[i:i + 6]
        i += 6
        dims = [tuple(vals[i + 3 * j:i + 3 * j + 3]) for j in range(nd)]
        i += 3 * nd
        out.append(dict(kind=kind, blen=blen, src=src, dst=dst, dims=dims, index=idx))
    return out


def plan_list(dt, leaf_index):
    L = lib()
    n = L.ddt_type_plan_list(dt.handle, leaf_index, None, None, 0)
    n = -n
    d = np.zeros(n, dtype=np.int64)
    ln = np.zeros(n, dtype=np.uint64)
    check(L.ddt_type_plan_list(dt.handle, leaf_index, d.ctypes.data_as(ctypes.c_void_p),
                               ln.ctypes.data_as(ctypes.c_void_p), n), "plan_list")
    return d, ln


def _multi_index(dims):
    """All (src_off, dst_off) of an affine nest, lexicographic order."""
    src = np.zeros(1, dtype=np.int64)
    dst = np.zeros(1, dtype=np.int64)
    for cnt, ss, ds in dims:
        k = np.arange(cnt, dtype=np.int64)
        src = (src[:, None] + k[None, :] * ss).reshape(-1)
        dst = (dst[:, None] + k[None, :] * ds).reshape(-1)
    return src, dst


def engine_blocks(dt):
    """(src, dst, len) of every block of one instance, from the engine's plan."""
    S, Dd, N = [], [], []
    for lf in leaves(dt):
        so, do = _multi_index(lf["dims"])
        if lf["kind"] == 0:
            S.append(so + lf["src"])
            Dd.append(do + lf["dst"])
            N.append(np.full(so.shape, lf["blen"], dtype=np.int64))
        else:
            d, ln = plan_list(dt, lf["index"])
            poff = np.concatenate([[0], np.cumsum(ln.astype(np.int64))[:-1]])
            S.append((so[:, None] + d[None, :] + lf["src"]).reshape(-1))
            Dd.append((do[:, None] + poff[None, :] + lf["dst"]).reshape(-1))
            N.append(np.tile(ln.astype(np.int64), len(so)))
    if not S:
        return np.zeros((0, 3), dtype=np.int64)
    src, dst, n = np.concatenate(S), np.concatenate(Dd), np.concatenate(N)
    o = np.argsort(dst, kind="stable")
    return merge_runs(np.stack([src[o], dst[o], n[o]], axis=1))


def merge_runs(blocks):
    """Merge consecutive (src, dst, len) blocks contiguous on both sides."""
    out = []
    for s, d, n in blocks:
        if n == 0:
            continue
        if out and out[-1][0] + out[-1][2] == s and out[-1][1] + out[-1][2] == d:
            out[-1][2] += n
        else:
            out.append([int(s), int(d), int(n)])
    return np.array(out, dtype=np.int64).reshape(-1, 3)


def oracle_blocks(otype):
    runs = otype.runs()
    blocks, p = [], 0
    for disp, ln, _ in runs:
        blocks.append((disp, p, ln))
        p += ln
    return merge_runs(np.array(blocks, dtype=np.int64).reshape(-1, 3))


def items(dt, count, user, pk, w0, w1, same_layout=False):
    L = lib()
    nitems = ctypes.c_size_t()
    isz = ctypes.c_size_t()
    L.ddt_debug_items(dt.handle, count, user, pk, w0, w1, int(same_layout), None, 0,
                      ctypes.byref(nitems), ctypes.byref(isz))
    assert isz.value == ctypes.sizeof(Item), (isz.value, ctypes.sizeof(Item))
    arr = (Item * max(nitems.value, 1))()
    check(L.ddt_debug_items(dt.handle, count, user, pk, w0, w1, int(same_layout), arr,
                            ctypes.sizeof(arr), ctypes.byref(nitems), ctypes.byref(isz)),
          "ddt_debug_items")
    return list(arr)[:nitems.value]


def _nest(it, blk):
    """blk (array) -> user/packed offsets over the item's dims (kernel nest_offsets)."""
    uo = np.zeros(blk.shape, dtype=np.int64)
    po = np.zeros(blk.shape, dtype=np.int64)
    b = blk.astype(np.int64).copy()
    for j in range(it.ndim - 1, 0, -1):
        c = int(it.cnt[j])
        idx = b % c
        b //= c
        uo += idx * it.ustr[j]
        po += idx * it.pstr[j]
    if it.ndim > 0:
        uo += b * it.ustr[0]
        po += b * it.pstr[0]
    return uo, po


def list_tables(dt):
    """{leaf index: (disp, disp_base, len)} for every LIST leaf (disp_base as the plan's
    32-bit compression uses: the minimum displacement when the span fits 31 bits)."""
    out = {}
    for lf in leaves(dt):
        if lf["kind"] == 1:
            d, ln = plan_list(dt, lf["index"])
            span = int(np.max(d + ln.astype(np.int64)) - np.min(d))
            base = int(np.min(d)) if span < (1 << 31) else 0
            out[lf["index"]] = (d, base, ln)
    return out


def emulate(its, user_arr, user_addr, packed_arr, packed_addr, direction, lists=None):
    """Run the descriptors on numpy byte arrays. Returns a coverage count of the packed
    array (every packed byte of the window must be touched exactly once)."""
    cover = np.zeros(packed_arr.shape[0], dtype=np.int32)

    def mv(ua, pa, n):
        uo = (ua - user_addr).astype(np.int64)
        po = (pa - packed_addr).astype(np.int64)
        for b in range(n):
            if direction == 0:
                packed_arr[po + b] = user_arr[uo + b]
            else:
                user_arr[uo + b] = packed_arr[po + b]
            np.add.at(cover, po + b, 1)

    for it in its:
        U = it.U
        if it.kind == ITEM_FRAG:
            mv(np.array([it.user], dtype=np.int64), np.array([it.packed], dtype=np.int64), int(it.nbytes))
            continue
        if it.kind in (ITEM_AFFINE, ITEM_LIST_UNI):
            u = np.arange(it.u0, it.u1, dtype=np.int64)
            blk = u // it.upb
            within = u - blk * it.upb
            if it.kind == ITEM_AFFINE:
                uo, po = _nest(it, blk)
                ua = it.user + uo + within * U
                pa = it.packed + po + within * U
            else:
                d, base, _ = lists[int(it.leaf)]
                i = blk % it.nblk
                outer = blk // it.nblk
                uo, po = _nest(it, outer)
                dd = d[i] - base if it.ldisp32 else d[i]
                ua = it.user + uo + dd + within * U
                pa = it.packed + po + (dd if it.same else i * it.ulen) + within * U
            mv(ua, pa, U)
            continue
        # LIST_VAR: one wave per 64-block group, inclusive scan, clip
        d, base, ln = lists[int(it.leaf)]
        ng = it.upb
        for gu in range(it.u0, it.u1):
            outer, g = divmod(gu, ng)
            uo, po = _nest(it, np.array([outer]))
            i = np.arange(g * 64, min(g * 64 + 64, it.nblk))
            l = ln[i].astype(np.int64)
            excl = np.concatenate([[0], np.cumsum(l)[:-1]])
            goff = int(np.sum(ln[:g * 64].astype(np.int64)))
            lx = outer * it.ulen + goff + excl
            s0 = np.maximum(lx, it.w0)
            s1 = np.minimum(lx + l, it.w1)
            for k in range(len(i)):
                if s1[k] > s0[k]:
                    off = s0[k] - lx[k]
                    dd = d[i[k]] - base if it.ldisp32 else d[i[k]]
                    ua = it.user + uo[0] + dd + off
                    pa = it.packed + po[0] + (dd if it.same else goff + excl[k]) + off
                    mv(np.array([ua]), np.array([pa]), int(s1[k] - s0[k]))
    return cover
