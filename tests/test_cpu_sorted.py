"""CPU replay of the address-ordered index-list engine (ompi_amd/csrc/ddt_sorted.hip).

The device builds its tables with atomics; this replays the same table definitions and
the two passes of pack and unpack with numpy index arithmetic, with the runs end to end in U
(the default since round 5) and padded to 64-byte segments that read a neighbouring run's LDS
bytes, and checks that every packed
element equals the direct gather user[disp[i]] (type-map order) and that unpack restores
exactly the touched elements.  It pins the layout math the kernels share, not the kernels.
"""
from __future__ import annotations

import numpy as np
import pytest

PAD = 0xFFFF


def build_tables(a, ch, seg):
    """a: element offsets of the blocks in type-map order (unique)."""
    n = a.size
    order = np.argsort(a, kind="stable")
    rank = np.empty(n, dtype=np.int64)
    rank[order] = np.arange(n)
    A = a[order]
    nc = nb = (n + ch - 1) // ch
    c = rank // ch
    k = np.arange(n) // ch
    ck = c * nb + k
    cnt = np.bincount(ck, minlength=nc * nb).reshape(nc, nb)
    # rank inside the (c, k) run: any consistent choice works (the device uses atomics);
    # replay it as type-map order inside the run
    srt = np.argsort(ck, kind="stable")
    first = np.zeros(nc * nb + 1, dtype=np.int64)
    first[1:] = np.cumsum(cnt.ravel())
    r = np.empty(n, dtype=np.int64)
    r[srt] = np.arange(n) - first[ck[srt]]
    off = np.zeros_like(cnt)
    off[:, 1:] = np.cumsum(cnt, axis=1)[:, :-1]
    pad = (cnt + seg - 1) // seg * seg
    ubT = np.zeros(nc * nb + 1, dtype=np.int64)
    ubT[1:] = np.cumsum(pad.T.ravel())
    slots = int(ubT[-1])
    ub = ubT[:-1].reshape(nb, nc).T
    bstart = np.append(ubT[:-1].reshape(nb, nc)[:, 0], slots)
    SL = np.empty(n, dtype=np.int64)
    SL[rank] = off[c, k] + r
    upos = np.full(slots, PAD, dtype=np.int64)
    upos[ub[c, k] + r] = np.arange(n) - k * ch
    assert SL.max() < ch and upos[upos != PAD].max() < ch
    return dict(A=A, SL=SL, cnt=cnt, off=off, ub=ub, bstart=bstart, upos=upos, nc=nc, nb=nb, slots=slots)


def pack(user, T, n, ch, seg):
    U = np.zeros(T["slots"], dtype=user.dtype)
    for c in range(T["nc"]):
        j0, m = c * ch, min(ch, n - c * ch)
        lds = np.full(ch + seg, -1, dtype=user.dtype)
        lds[T["SL"][j0:j0 + m]] = user[T["A"][j0:j0 + m]]
        for k in range(T["nb"]):
            cn = T["cnt"][c, k]
            if cn:
                pn = (cn + seg - 1) // seg * seg
                o, b = T["off"][c, k], T["ub"][c, k]
                U[b:b + pn] = lds[o:o + pn]
    out = np.zeros(n, dtype=user.dtype)
    for k in range(T["nb"]):
        s0, s1 = T["bstart"][k], T["bstart"][k + 1]
        lds = np.full(ch, -7, dtype=user.dtype)
        p = T["upos"][s0:s1]
        keep = p != PAD
        lds[p[keep]] = U[s0:s1][keep]
        m = min(ch, n - k * ch)
        out[k * ch:k * ch + m] = lds[:m]
    return out


def unpack(packed, user, T, n, ch, seg):
    U = np.zeros(T["slots"], dtype=packed.dtype)
    for k in range(T["nb"]):
        m = min(ch, n - k * ch)
        lds = packed[k * ch:k * ch + m]
        s0, s1 = T["bstart"][k], T["bstart"][k + 1]
        p = T["upos"][s0:s1]
        U[s0:s1] = np.where(p != PAD, lds[np.minimum(p, m - 1)], 0)
    for c in range(T["nc"]):
        j0, m = c * ch, min(ch, n - c * ch)
        lds = np.full(ch, -3, dtype=packed.dtype)
        for k in range(T["nb"]):
            cn = T["cnt"][c, k]
            o, b = T["off"][c, k], T["ub"][c, k]
            lds[o:o + cn] = U[b:b + cn]
        user[T["A"][j0:j0 + m]] = lds[T["SL"][j0:j0 + m]]


@pytest.mark.parametrize("padded", [False, True])
@pytest.mark.parametrize("esz,n,density", [(4, 3 * 512 + 77, 4), (8, 2000, 1), (16, 513, 64), (4, 5, 3)])
def test_sorted_engine_replay(esz, n, density, padded):
    # the device uses CH = 128 KiB / esz; a smaller CH keeps many chunks/buckets here
    ch = {4: 512, 8: 256, 16: 128}[esz]
    seg = 64 // esz if padded else 1
    rng = np.random.default_rng(esz * 7 + n)
    a = rng.permutation(density * n)[:n].astype(np.int64)
    user = rng.integers(1, 2 ** 31, density * n + 1).astype(np.int64)
    T = build_tables(a, ch, seg)
    got = pack(user, T, n, ch, seg)
    np.testing.assert_array_equal(got, user[a])
    back = np.full_like(user, -5)
    unpack(got, back, T, n, ch, seg)
    exp = np.full_like(user, -5)
    exp[a] = user[a]
    np.testing.assert_array_equal(back, exp)


def test_sorted_engine_size_limits():
    """The plan rule of ddt_plan.cpp (sorted_plan): runs average at least half a segment."""
    for esz in (4, 8, 16):
        ch = (128 << 10) // esz
        seg = 64 // esz
        nmax = 2 * ch * ch // seg
        # expected elements per (chunk, bucket) run at the limit
        runs = ((nmax + ch - 1) // ch) ** 2
        assert nmax / runs >= seg / 2
    # BASELINE config 4 (64 Mi floats) qualifies: 16 elements (one segment) per run
    assert (64 << 20) <= 2 * (32 << 10) ** 2 // 16


def chunk_of(b, n):
    """ddt_sorted.hip chunk_of with POL_XCD_SLAB: workgroup b (dealt to XCD b % 8) -> chunk."""
    x, i, per, rem = b & 7, b >> 3, n >> 3, n & 7
    return x * per + min(x, rem) + i


@pytest.mark.parametrize("n", list(range(1, 70)) + [2047, 2048, 2049, 4096 + 5])
def test_xcd_slab_chunk_map_is_a_bijection(n):
    """Every chunk is moved exactly once, and the chunks of one XCD (b % 8 equal) form one
    contiguous slab in workgroup order."""
    cs = [chunk_of(b, n) for b in range(n)]
    assert sorted(cs) == list(range(n))
    for x in range(8):
        mine = [chunk_of(b, n) for b in range(x, n, 8)]
        assert mine == list(range(mine[0], mine[0] + len(mine))) if mine else True
