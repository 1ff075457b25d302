"""Datatype lifetime on the GPU without device-wide waits (round 3).

The reference's opal_datatype_destruct (opal_datatype_create.c:61-91) frees host memory at
once.  The engine's plans live in HBM and queued kernels may still read them, so destroying a
type hands its memory to the engine's pool behind fence events on the streams that launched
it (ddt_pool.h) -- no hipDeviceSynchronize, no hipFree.  These tests destroy a type while its
pack is still queued and while another thread captures a graph, then check every byte.
"""
from __future__ import annotations

import threading

import numpy as np
import pytest

from . import recipes as R

pytestmark = pytest.mark.gpu

FLOAT4, FLOAT8 = 15, 16


def _pool():
    import ctypes
    import ompi_amd
    out = (ctypes.c_int64 * 6)()
    assert ompi_amd.lib().ddt_pool_info(out) == 0
    return dict(zip(("free_blocks", "free_bytes", "fenced_blocks", "fenced_bytes", "kept", "in_use"), list(out)))


def _dev(arr, device):
    import torch
    return torch.from_numpy(np.ascontiguousarray(arr)).to(device)


def _oracle_pack(b, host, origin, count=1):
    size = b.o.info()["size"] * count
    return np.frombuffer(b.o.pack(count, host, origin, 0, size, element_granular=False), dtype=np.uint8)


# T1 has plan memory of every kind: an index list and a descriptor set in HBM (the nine members'
# 2700 blocks commit to one run of FLOAT4 entries, which the import folds into one list)
_REC1 = ("struct", [1] * 9, [64 * i for i in range(9)],
         [("indexed_block", 2, [(37 * k) % 509 * 4 for k in range(300)], ("basic", FLOAT4))] * 9)
_REC2 = ("vector", 4096, 3, 7, ("basic", FLOAT4))


@pytest.mark.parametrize("mode", ["global", "relaxed"])
def test_destroy_while_queued_and_during_foreign_capture(device, mode):
    """Thread A queues T1's pack behind a 100 ms sleep on its stream, then -- while thread B
    captures a graph of T2 on another stream (torch.cuda.graph, `mode` capture) -- destroys
    T1 (the destroy records fence events; HIP allows that during another thread's global
    capture, scripts/probe_capture.cpp).  B's capture must end intact.  Then, with T1's pack
    still queued, a fresh T3 of the same shape is built and packed: T1's plan memory must
    wait for its fence (reused early, T3's uploads would overwrite the descriptors T1's
    queued pack still reads).  Every byte of T1, T3 and the replayed graph of T2 must match
    the oracle.  (Building a NEW plan during a foreign global capture is impossible in HIP:
    hipMalloc and stream synchronisation are refused there and invalidate the capture.)"""
    import torch
    import ompi_amd
    from ompi_amd import recipe as ER
    b1, b2, b3 = R.Built(_REC1), R.Built(_REC2), R.Built(_REC1)
    sizes, users, hosts, origins, outs = [], [], [], [], []
    for k, b in enumerate((b1, b2, b3)):
        info = b.o.info()
        span, origin = R.layout(info, 1)
        h = R.fill(span, 50 + k)
        hosts.append(h)
        origins.append(origin)
        users.append(_dev(h, device))
        sizes.append(info["size"])
        outs.append(torch.zeros(info["size"], dtype=torch.uint8, device=device))
    sa, sb = torch.cuda.Stream(device), torch.cuda.Stream(device)
    t1 = ER.build_committed(_REC1)
    t2 = ER.build_committed(_REC2)
    c1 = ompi_amd.Convertor()
    c1.set_stream(sa, True)
    c2 = ompi_amd.Convertor()
    for _ in range(3):   # warm: plans built, descriptor sets launched by pointer from HBM
        c1.prepare_for_send(t1, 1, users[0].data_ptr() + origins[0])
        c1.pack([(outs[0], sizes[0])])
        c2.prepare_for_send(t2, 1, users[1].data_ptr() + origins[1])
        c2.pack([(outs[1], sizes[1])])
    torch.cuda.synchronize()
    pi = t1.plan_info()
    assert pi["list_leaves"] >= 1 and pi["device_bytes"] > 0, pi
    for o in outs:
        o.zero_()
    torch.cuda.synchronize()
    # T1's pack queued behind a sleep: still to run when T1 is destroyed
    with torch.cuda.stream(sa):
        torch.cuda._sleep(int(2e8))
    c1.prepare_for_send(t1, 1, users[0].data_ptr() + origins[0])
    c1.pack([(outs[0], sizes[0])])
    before = _pool()
    started, destroyed = threading.Event(), threading.Event()
    errors = []
    g = torch.cuda.CUDAGraph()

    def capture():
        try:
            with torch.cuda.graph(g, stream=sb, capture_error_mode=mode):
                cs = torch.cuda.current_stream(device)
                c2.set_stream(cs, True)
                c2.prepare_for_send(t2, 1, users[1].data_ptr() + origins[1])
                c2.pack([(outs[1], sizes[1] // 2)])
                started.set()
                destroyed.wait(60)
                c2.set_position(sizes[1] // 2 // 4 * 4)
                c2.pack([(outs[1].data_ptr() + sizes[1] // 2 // 4 * 4, sizes[1] - sizes[1] // 2 // 4 * 4)])
        except Exception as ex:   # noqa: BLE001 -- reported below
            errors.append(repr(ex))
            started.set()

    def destroy():
        try:
            started.wait(60)
            c1.close()
            t1.destroy()   # the last references: ~Plan runs here, with T1's pack still queued
            mid = _pool()
            errors.append(("fenced", mid["fenced_blocks"] - before["fenced_blocks"]))
        except Exception as ex:   # noqa: BLE001
            errors.append(repr(ex))
        finally:
            destroyed.set()

    ta, tb = threading.Thread(target=destroy), threading.Thread(target=capture)
    tb.start()
    ta.start()
    ta.join(120)
    tb.join(120)
    fails = [e for e in errors if isinstance(e, str)]
    assert not fails, fails
    fenced = [e[1] for e in errors if isinstance(e, tuple) and e[0] == "fenced"]
    assert fenced and fenced[0] > 0, ("T1's memory should wait on its fence", fenced)
    # T1's pack is still queued behind the sleep: T3 (same plan sizes) must not get its memory
    t3 = ER.build_committed(_REC1)
    c3 = ompi_amd.Convertor()
    c3.set_stream(sa, True)
    for _ in range(2):
        c3.prepare_for_send(t3, 1, users[2].data_ptr() + origins[2])
        c3.pack([(outs[2], sizes[2])])
    torch.cuda.synchronize()
    np.testing.assert_array_equal(outs[0].cpu().numpy(), _oracle_pack(b1, hosts[0], origins[0]))
    np.testing.assert_array_equal(outs[2].cpu().numpy(), _oracle_pack(b3, hosts[2], origins[2]))
    outs[1].zero_()
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    np.testing.assert_array_equal(outs[1].cpu().numpy(), _oracle_pack(b2, hosts[1], origins[1]))
    t4 = ER.build_committed(_REC1)   # an allocation checks the fences: T1's blocks come free
    ompi_amd.pack(users[2].data_ptr() + origins[2], 1, t4, outs[2], sizes[2], 0)
    after = _pool()
    assert after["fenced_blocks"] <= before["fenced_blocks"], (before, after)


def test_trim_returns_cached_memory(device):
    """ddt_trim synchronises and hands every cached block back to HIP; types built afterwards
    work as before."""
    import torch
    import ompi_amd
    from ompi_amd import recipe as ER
    b = R.Built(_REC1)
    info = b.o.info()
    span, origin = R.layout(info, 1)
    host = R.fill(span, 9)
    user = _dev(host, device)
    out = torch.zeros(info["size"], dtype=torch.uint8, device=device)
    for _ in range(2):
        t = ER.build_committed(_REC1)
        ompi_amd.pack(user.data_ptr() + origin, 1, t, out, info["size"], 0)
        t.destroy()
    assert ompi_amd.lib().ddt_trim() == 0
    p = _pool()
    assert p["free_blocks"] == 0 and p["fenced_blocks"] == 0, p
    t = ER.build_committed(_REC1)
    out.zero_()
    ompi_amd.pack(user.data_ptr() + origin, 1, t, out, info["size"], 0)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(out.cpu().numpy(), _oracle_pack(b, host, origin))


def test_staging_fence_survives_a_stream_change(device):
    """an asynchronous unpack from pageable host memory (staged through the
    convertor's HBM buffer in two chunks: > 24 MiB) is queued on stream A behind a sleep; the
    convertor's stream is then set to NULL (what the bridge does after every call) and the
    convertor destroyed while A's kernels have not read the buffer yet.  Another convertor
    stages a different message of the same size at once on an idle stream: it must not be
    handed the buffer A still reads (the destructor fences it with the event recorded after
    the last reader, wherever that was), so both unpacks land bit-exact."""
    import torch
    import ompi_amd
    from ompi_amd import recipe as ER
    rec = ("vector", 1 << 22, 1, 2, ("basic", FLOAT8))   # 32 MiB packed
    b = R.Built(rec)
    info = b.o.info()
    size = info["size"]
    span, origin = R.layout(info, 1)
    t = ER.build_committed(rec)
    srcs = [np.ascontiguousarray(R.fill_fast(size, 70 + k)) for k in range(2)]
    outs = [torch.full((span,), 0xA5, dtype=torch.uint8, device=device) for _ in range(2)]
    sa, sc = torch.cuda.Stream(device), torch.cuda.Stream(device)
    torch.cuda.synchronize()
    c1 = ompi_amd.Convertor()
    c1.set_stream(sa, True)
    c1.prepare_for_recv(t, 1, outs[0].data_ptr() + origin)
    with torch.cuda.stream(sa):
        torch.cuda._sleep(int(4e8))
    rc, _, md = c1.unpack([(srcs[0].ctypes.data, size)])
    assert md == size
    c1.set_stream(None, False)
    before = _pool()
    c1.close()
    mid = _pool()
    assert mid["fenced_blocks"] > before["fenced_blocks"], (before, mid)
    c2 = ompi_amd.Convertor()
    c2.set_stream(sc, True)
    c2.prepare_for_recv(t, 1, outs[1].data_ptr() + origin)
    c2.unpack([(srcs[1].ctypes.data, size)])
    torch.cuda.synchronize()
    for k in range(2):
        want = np.full(span, 0xA5, dtype=np.uint8)
        b.o.unpack(1, want, origin, 0, srcs[k].tobytes())
        np.testing.assert_array_equal(outs[k].cpu().numpy(), want)
    c2.close()


def test_large_external32_scratch_goes_back_to_hip(device):
    """external32 scratch above 256 MiB is a block of the call's own and goes back to
    HIP when the call ends, not into the engine's cache (where a co-resident allocator could
    not have it)."""
    import torch
    import ompi_amd
    from ompi_amd import recipe as ER
    n = (288 << 20) // 8
    t = ER.build_committed(("contig", n, ("basic", FLOAT8)))
    src = torch.arange(n, dtype=torch.float64, device=device)
    ext = torch.zeros(n * 8, dtype=torch.uint8, device=device)
    before = _pool()
    ompi_amd.pack_external(src, 1, t, ext, n * 8)
    torch.cuda.synchronize()
    after = _pool()
    cached = lambda p: p["free_bytes"] + p["fenced_bytes"]   # noqa: E731
    assert cached(after) - cached(before) < (256 << 20), (before, after)
    want = src.cpu().numpy().astype(">f8").view(np.uint8)
    np.testing.assert_array_equal(ext.cpu().numpy(), want)
