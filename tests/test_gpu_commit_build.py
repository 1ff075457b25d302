"""The address-ordered tables are built where Open MPI pays its commit, not inside the first
pack of a message (opal_datatype_commit, opal_datatype_optimize.c:1739-1782).

A cfg4-shaped type -- an indexed list of 2 Mi one-float blocks at LCG displacements (the
address-ordered engine's domain, >= 1 Mi blocks) -- is committed with the engine's constructors
and, separately, handed to the bridge as Open MPI's committed description (two-block FLOAT4 pairs,
SURVEY App. A).  The engine's commit and the bridge's import (at prepare) build the tables; the
first asynchronous pack's host call then only enqueues: it must return in under 3 ms (the build
itself is ~10 ms of device work plus host round trips; 3 ms leaves room for box jitter, r5).  The packed bytes are checked.
"""
from __future__ import annotations

import time

import numpy as np
import pytest

from . import opal_shapes as S

pytestmark = pytest.mark.gpu

N = 2 << 20
SPAN_FLOATS = 1 << 24


def _lcg(n):
    out = np.empty(n, dtype=np.int64)
    x, a, c, m = 0x5EED, 1664525, 1013904223, 1 << 24
    for i in range(n):   # 2 Mi steps: ~1 s in Python, done once
        out[i] = x
        x = (a * x + c) % m
    return out


@pytest.fixture(scope="module")
def disps():
    d = _lcg(N)
    assert len(np.unique(d)) == N   # full period: unique, so unpack is well defined
    return d


def _want(user_host, d):
    return user_host.view(np.float32)[d].view(np.uint8)


def test_engine_commit_builds_the_tables(device, disps):
    import torch
    import ompi_amd
    from ompi_amd import recipe as ER
    user = torch.randint(1, 255, (SPAN_FLOATS * 4,), dtype=torch.uint8, device=device)
    packed = torch.zeros(N * 4, dtype=torch.uint8, device=device)
    t = ER.build_committed(("indexed_block", 1, disps.tolist(), ("basic", 15)))
    assert t.engine_info()["sorted"] == 1   # built at commit
    s = torch.cuda.Stream(device)
    c = ompi_amd.Convertor()
    c.set_stream(s, True)
    c.prepare_for_send(t, 1, user.data_ptr())
    t0 = time.perf_counter()
    rc, _, md = c.pack([(packed, N * 4)])
    host_s = time.perf_counter() - t0
    assert rc == 1 and md == N * 4
    torch.cuda.synchronize()
    np.testing.assert_array_equal(packed.cpu().numpy(), _want(user.cpu().numpy(), disps))
    assert host_s < 3e-3, f"first asynchronous pack took {host_s * 1e3:.2f} ms of host time"


@pytest.mark.parametrize("hook", [False, True], ids=["import_at_prepare", "commit_hook"])
def test_bridge_import_builds_the_tables(device, disps, hook):
    """With the commit hook (opal_hip_bridge_datatype_commit) the 1 Mi-entry description is
    imported inside the commit, so the prepare of the first message only hits the cache."""
    import torch
    order = np.arange(N)
    pairs = order[0::2]
    a, b = disps[pairs] * 4, disps[pairs + 1] * 4
    ents = np.zeros(N // 2, dtype=[("flags", "<u2"), ("type", "<u2"), ("count", "<u4"), ("blen", "<u8"),
                                   ("ext", "<i8"), ("disp", "<i8")])
    ents["flags"], ents["type"], ents["count"], ents["blen"] = 0x136 | 0x100, 15, 2, 1
    ents["ext"], ents["disp"] = b - a, a
    lo, hi = int(disps.min()) * 4, int(disps.max()) * 4 + 4
    ot = S.OpalType([ents.tobytes()], N * 4, lo, hi, lo, hi)
    ot.dt.desc.used = ot.dt.opt_desc.used = N // 2
    ot.raw = np.concatenate([np.frombuffer(ents.tobytes(), dtype=np.uint8),
                             np.frombuffer(S.end_loop(N // 2, N * 4, lo), dtype=np.uint8)])
    ot.dt.desc.desc = ot.dt.opt_desc.desc = ot.raw.ctypes.data
    ot.dt.desc.length = ot.dt.opt_desc.length = N // 2 + 1
    user = torch.randint(1, 255, (SPAN_FLOATS * 4,), dtype=torch.uint8, device=device)
    packed = torch.zeros(N * 4, dtype=torch.uint8, device=device)
    s = torch.cuda.Stream(device)
    base = S.stats()
    if hook:
        assert ot.commit_hook() == S.OPAL_SUCCESS
        assert S.stats()["imports"] - base["imports"] == 1
    conv = S.Convertor()
    t0 = time.perf_counter()
    assert conv.prepare(ot, 1, user.data_ptr(), send=True, stream=s.cuda_stream) == S.OPAL_SUCCESS
    prep_s = time.perf_counter() - t0
    assert S.stats()["imports"] - base["imports"] == 1
    if hook:
        assert prep_s < 5e-3, f"prepare after the commit hook took {prep_s * 1e3:.2f} ms"
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    rc, _, md = conv.pack([(packed.data_ptr(), N * 4)])
    host_s = time.perf_counter() - t0
    assert rc == 1 and md == N * 4
    torch.cuda.synchronize()
    np.testing.assert_array_equal(packed.cpu().numpy(), _want(user.cpu().numpy(), disps))
    assert host_s < 3e-3, f"first asynchronous bridge pack took {host_s * 1e3:.2f} ms of host time"
    ot.destruct()


@pytest.mark.parametrize("mode", ["global", "relaxed"])
def test_commit_during_foreign_capture(device, disps, mode):
    """a commit (or the bridge's first-attach import) of a table-building type while
    ANOTHER thread captures a graph (`mode` capture).  The table build allocates and waits on the
    library's private stream; it runs with the committing thread in relaxed capture mode and is
    skipped while the legacy stream reports a capture, so the foreign capture must end intact and
    its graph replay correctly; the type then packs bit-exactly (tables built now or at first
    move)."""
    import threading
    import torch
    import ompi_amd
    from ompi_amd import datatype as D
    x = torch.zeros(1024, device=device)
    sb = torch.cuda.Stream(device)
    g = torch.cuda.CUDAGraph()
    started, committed = threading.Event(), threading.Event()
    errors, types = [], []

    def capture():
        try:
            with torch.cuda.graph(g, stream=sb, capture_error_mode=mode):
                x.add_(1)
                started.set()
                committed.wait(120)
                x.add_(1)
        except Exception as ex:   # noqa: BLE001 -- reported below
            errors.append(repr(ex))
            started.set()

    def commit():
        try:
            started.wait(60)
            t = D.create_indexed_block(1, disps, D.predefined(15)).commit()
            types.append(t)
        except Exception as ex:   # noqa: BLE001
            errors.append(repr(ex))
        finally:
            committed.set()

    tb, ta = threading.Thread(target=capture), threading.Thread(target=commit)
    tb.start()
    ta.start()
    ta.join(180)
    tb.join(180)
    assert not errors, errors
    g.replay()
    torch.cuda.synchronize()
    assert float(x[0].item()) == 2.0
    user = torch.randint(1, 255, (SPAN_FLOATS * 4,), dtype=torch.uint8, device=device)
    packed = torch.zeros(N * 4, dtype=torch.uint8, device=device)
    assert ompi_amd.pack(user.data_ptr(), 1, types[0], packed, N * 4, 0) == N * 4
    torch.cuda.synchronize()
    np.testing.assert_array_equal(packed.cpu().numpy(), _want(user.cpu().numpy(), disps))
