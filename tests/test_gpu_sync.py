"""Synchronous completion on a device-written host word (round 6; ddt_kernels.hip
ddt_signal_kernel, ddt_convertor.cpp complete_sync).

MPI_Pack / MPI_Unpack and a convertor without the async flag must return with the data in place
(/root/reference/ompi/mpi/c/pack.c.in:129-150; opal_convertor_pack is synchronous for the
accelerator movers, opal_datatype_pack_accelerator.c).  The engine returns once a signal kernel
queued behind the move has stored its count to pinned host memory.  Right after return, work
that was never ordered after the call -- a kernel on another stream, a D2H copy on a third --
must see the final bytes: affine leaves, line-dense records and index lists alike.  The fallback
(spin timeout, signal off) must be just as correct.
"""
from __future__ import annotations

import ctypes

import numpy as np
import pytest

from . import recipes as R

pytestmark = pytest.mark.gpu


def _info():
    from ompi_amd._lib import lib
    out = (ctypes.c_int64 * 3)()
    assert lib().ddt_sync_info(out) == 0
    return list(out)


CASES = {
    # the y face of a 64^3 double field: affine rows
    "affine": (("resized", ("vector", 64, 64, 64 * 64, ("basic", 16)), 0, 64 ** 3 * 8), 3),
    # struct{double,int[3]} records at a 32-byte pitch: line-dense records (cfg5's shape)
    "dense": (("hvector", 4096, 1, 32, ("struct", [1, 3], [0, 8], [("basic", 16), ("basic", 6)])), 2),
    # random 4-byte displacements: an index list
    "list": None,
}


def _case(name):
    if name == "list":
        rng = np.random.default_rng(7)
        disps = rng.permutation(1 << 18)[:30000].astype(np.int64)
        return ("indexed_block", 1, disps.tolist(), ("basic", 15)), 2
    return CASES[name]


def _run(device, name, seed):
    """MPI_Pack then MPI_Unpack (both synchronous, on the legacy stream); right after each
    returns, a clone on an unrelated stream and a D2H copy on another read the result."""
    import torch
    import ompi_amd
    rec, count = _case(name)
    b = R.Built(rec)
    e = b.engine()
    info = b.o.info()
    size = info["size"] * count
    span, origin = R.layout(info, count)
    host = R.fill(span, seed)
    user = torch.from_numpy(host).to(device)
    uptr = user.data_ptr() + origin
    packed = torch.full((size,), 0xA5, dtype=torch.uint8, device=device)
    s2, s3 = torch.cuda.Stream(device), torch.cuda.Stream(device)
    sink = torch.empty(size, dtype=torch.uint8).pin_memory()
    torch.cuda.synchronize()
    assert ompi_amd.pack(uptr, count, e, packed, size, 0) == size
    with torch.cuda.stream(s2):           # no event, no stream ordering against the pack
        seen = packed.clone()
    with torch.cuda.stream(s3):
        sink.copy_(packed, non_blocking=True)
    torch.cuda.synchronize()
    ref = np.frombuffer(b.o.pack(count, host, origin, 0, size, element_granular=False), dtype=np.uint8)
    np.testing.assert_array_equal(seen.cpu().numpy(), ref)
    np.testing.assert_array_equal(sink.numpy(), ref)
    # MPI_Unpack into a 0x5A-filled buffer, read the same way right after return
    out = torch.full((span,), 0x5A, dtype=torch.uint8, device=device)
    sink2 = torch.empty(span, dtype=torch.uint8).pin_memory()
    torch.cuda.synchronize()
    assert ompi_amd.unpack(packed, size, 0, out.data_ptr() + origin, count, e) == size
    with torch.cuda.stream(s2):
        seen2 = out.clone()
    with torch.cuda.stream(s3):
        sink2.copy_(out, non_blocking=True)
    torch.cuda.synchronize()
    exp = np.full(span, 0x5A, dtype=np.uint8)
    b.o.unpack(count, exp, origin, 0, ref.tobytes())
    np.testing.assert_array_equal(seen2.cpu().numpy(), exp)
    np.testing.assert_array_equal(sink2.numpy(), exp)


@pytest.mark.parametrize("name", ["affine", "dense", "list"])
def test_sync_calls_return_with_the_data_in_place(device, name):
    before = _info()
    for seed in range(3):
        _run(device, name, 100 + seed)
    after = _info()
    # every synchronous call completed on the signal (none fell back)
    assert after[0] - before[0] >= 6 and after[1] == before[1], (before, after)


@pytest.mark.parametrize("name", ["affine", "list"])
def test_sync_fallbacks_are_correct(device, name):
    """The spin gives up at once (sigspin_us 0: the call blocks in hipStreamSynchronize after
    ~1000 polls) or the signal is off: the same bytes, counted as fallbacks / plain syncs."""
    import ompi_amd
    L = ompi_amd.lib()
    try:
        L.ddt_tune(b"sigspin_us", 0)
        b0 = _info()
        for seed in range(2):
            _run(device, name, 200 + seed)
        b1 = _info()
        assert b1[0] + b1[1] - b0[0] - b0[1] >= 4, (b0, b1)
        L.ddt_tune(b"sigspin_us", 20000)
        L.ddt_tune(b"sigsync", 0)
        _run(device, name, 300)
        b2 = _info()
        assert b2[2] - b1[2] >= 2 and b2[0] == b1[0], (b1, b2)
    finally:
        L.ddt_tune(b"sigsync", 1)
        L.ddt_tune(b"sigspin_us", 20000)


def test_sync_from_many_threads(device):
    """Sixteen signal slots, more threads than slots: every thread's synchronous packs are in
    place on return (a thread finding no free slot falls back to a plain stream sync)."""
    import threading
    import torch
    import ompi_amd
    rec, count = _case("affine")
    b = R.Built(rec)
    e = b.engine()
    info = b.o.info()
    size = info["size"] * count
    span, origin = R.layout(info, count)
    host = R.fill(span, 77)
    user = torch.from_numpy(host).to(device)
    ref = np.frombuffer(b.o.pack(count, host, origin, 0, size, element_granular=False), dtype=np.uint8)
    errors = []

    def work(i):
        try:
            torch.cuda.set_device(device)
            packed = torch.zeros(size, dtype=torch.uint8, device=device)
            for _ in range(20):
                packed.zero_()
                torch.cuda.current_stream(device).synchronize()
                ompi_amd.pack(user.data_ptr() + origin, count, e, packed, size, 0)
                got = packed.cpu().numpy()   # the legacy stream's D2H right after return
                if not np.array_equal(got, ref):
                    errors.append(i)
                    return
        except Exception as ex:  # surface to the main thread
            errors.append(repr(ex))

    th = [threading.Thread(target=work, args=(i,)) for i in range(20)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    assert not errors, errors
