"""Argument-free launches (ddt_move.hip.h ddt_move_slot_kernel, ddt_plan.cpp slot_bind; round 5).

A descriptor set launched twice in a row on the same buffers is bound to a launch record in
device memory and later launches on those buffers take no kernel arguments.  Every launch must
still move exactly the oracle's bytes: new contents each call, buffers that change after a bind,
more hot sets than slots, a second stream, slots released with their type and bound again.
"""
from __future__ import annotations

import gc

import numpy as np
import pytest

from . import recipes as R

pytestmark = pytest.mark.gpu


def _slots():
    import ctypes
    from ompi_amd._lib import lib
    out = (ctypes.c_int64 * 4)()
    assert lib().ddt_slot_info(out) == 0
    return list(out)


@pytest.fixture(autouse=True)
def _no_bindings():
    """Every test starts with all slots free: ddt_trim ends the bindings earlier tests left."""
    import torch
    from ompi_amd._lib import lib
    torch.cuda.synchronize()
    assert lib().ddt_trim() == 0
    st = _slots()
    assert st[0] == 0 and st[1] == 0, st
    yield


NSLOT = 32   # launch records per direction (ddt_device.h)


def _face(n, which):
    import bench
    return bench.face_recipes(n=n)[which]


class _Msg:
    """One type on fixed device buffers, packed / unpacked again and again through one
    asynchronous convertor pair on `stream`."""

    def __init__(self, recipe, count, device, stream, seed):
        import torch
        import ompi_amd
        self.b = R.Built(recipe)
        self.e = self.b.engine()
        info = self.b.o.info()
        self.count = count
        self.size = info["size"] * count
        self.span, self.origin = R.layout(info, count)
        self.device = device
        self.user = torch.zeros(self.span + 16, dtype=torch.uint8, device=device)
        self.out = torch.zeros(self.span + 16, dtype=torch.uint8, device=device)
        self.packed = torch.zeros(self.size, dtype=torch.uint8, device=device)
        self.stream = stream
        self.cp, self.cu = ompi_amd.Convertor(), ompi_amd.Convertor()
        for c in (self.cp, self.cu):
            c.set_stream(stream, True)
        self.rng = np.random.default_rng(seed)

    def step(self, packed=None):
        """New user contents, pack, unpack into a 0xA5-filled buffer; both checked."""
        import torch
        packed = self.packed if packed is None else packed
        host = self.rng.integers(1, 255, self.span, dtype=np.uint8)
        torch.cuda.synchronize()
        self.user[:self.span].copy_(torch.from_numpy(host))
        self.out.fill_(0xA5)
        torch.cuda.synchronize()
        uptr = self.user.data_ptr() + self.origin
        self.cp.prepare_for_send(self.e, self.count, uptr)
        rc, _, md = self.cp.pack([(packed.data_ptr(), self.size)])
        assert rc == 1 and md == self.size
        self.cu.prepare_for_recv(self.e, self.count, self.out.data_ptr() + self.origin)
        rc, _, md = self.cu.unpack([(packed.data_ptr(), self.size)])
        assert rc == 1 and md == self.size
        torch.cuda.synchronize()
        ref = np.frombuffer(self.b.o.pack(self.count, host, self.origin, 0, self.size, element_granular=False),
                            dtype=np.uint8)
        np.testing.assert_array_equal(packed.cpu().numpy(), ref)
        exp = np.full(self.span, 0xA5, dtype=np.uint8)
        self.b.o.unpack(self.count, exp, self.origin, 0, ref.tobytes())
        np.testing.assert_array_equal(self.out[:self.span].cpu().numpy(), exp)


def test_hot_faces_bind_slots_and_move_the_oracle_bytes(device):
    import torch
    s = torch.cuda.Stream(device)
    before = _slots()
    msgs = [_Msg(_face(32, w), 3, device, s, 10 + i) for i, w in enumerate("xyz")]
    for _ in range(5):
        for m in msgs:
            m.step()
    after = _slots()
    # three sets per direction bound (pack and unpack sets are distinct: their task orders differ)
    assert after[0] - before[0] == 3 and after[1] - before[1] == 3, (before, after)
    # launches 3..5 of each of the 6 sets ran without arguments
    assert after[3] - before[3] >= 6 * 3, (before, after)


def test_changed_buffers_fall_back_and_return(device):
    import torch
    s = torch.cuda.Stream(device)
    m = _Msg(_face(32, "y"), 2, device, s, 21)
    for _ in range(3):
        m.step()
    other = torch.zeros_like(m.packed)
    n0 = _slots()[3]
    m.step(packed=other)           # a different packed buffer: launches with arguments
    assert _slots()[3] == n0
    m.step()                       # the bound buffers again: argument-free, both directions
    assert _slots()[3] == n0 + 2


def test_more_hot_sets_than_slots(device):
    """More hot types of one direction than slots: NSLOT bind, the rest keep launching with
    arguments; all move the right bytes."""
    import torch
    from ompi_amd._lib import lib
    s = torch.cuda.Stream(device)
    msgs = [_Msg(("resized", ("vector", 64, 1 + (i % 3), 8 + i, ("basic", 16)), 0, 8 * (8 + i) * 64), 2,
                 device, s, 40 + i) for i in range(NSLOT + 6)]
    for _ in range(3):
        for m in msgs:
            m.step()
    st = _slots()
    assert st[0] == NSLOT and st[1] == NSLOT, st
    assert lib().ddt_slot_state(0, NSLOT) == -1 and lib().ddt_slot_state(0, NSLOT - 1) & 1
    for m in msgs:
        m.step()


def test_idle_bindings_are_evicted_for_a_new_hot_set(device):
    """NSLOT sets bind every pack slot and go idle; a further set's bind attempts age them and,
    after kEvictIdle ticks, end the least recent binding (behind fences): the new set binds and
    launches argument-free; the evicted set falls back to arguments and stays correct."""
    import torch
    s = torch.cuda.Stream(device)
    # one 8-byte element per 64+ bytes: the unit loop (line-dense records take no slots)
    idle = [_Msg(("resized", ("vector", 16, 1, 8 + i, ("basic", 16)), 0, 8 * (8 + i) * 16), 1, device, s, 70 + i)
            for i in range(NSLOT)]
    for _ in range(3):
        for m in idle:
            m.step()
    assert _slots()[0] == NSLOT
    hot = _Msg(("resized", ("vector", 16, 1, 8 + NSLOT + 3, ("basic", 16)), 0, 8 * (8 + NSLOT + 3) * 16), 1,
               device, s, 90)
    n0 = _slots()[3]
    for _ in range(140):   # 2 calls per step: >= 256 bind attempts in the unpack and pack families
        hot.step()
    assert _slots()[3] > n0, _slots()   # the hot set launched from a slot at last
    for m in idle:
        m.step()


def test_second_stream_uses_a_bound_slot(device):
    import torch
    s1, s2 = torch.cuda.Stream(device), torch.cuda.Stream(device)
    m = _Msg(_face(32, "z"), 2, device, s1, 31)
    for _ in range(3):
        m.step()
    for c in (m.cp, m.cu):
        c.set_stream(s2, True)
    n0 = _slots()[3]
    m.step()                       # the record is in device memory: s2 launches from the slot too
    assert _slots()[3] == n0 + 2


def test_slots_are_released_with_their_type_and_bound_again(device):
    import torch
    s = torch.cuda.Stream(device)
    base = _slots()
    m = _Msg(_face(32, "x"), 2, device, s, 51)
    for _ in range(3):
        m.step()
    bound = _slots()
    assert bound[0] == base[0] + 1 and bound[1] == base[1] + 1
    del m
    gc.collect()
    torch.cuda.synchronize()
    freed = _slots()
    assert freed[0] == base[0] and freed[1] == base[1], (base, freed)
    m2 = _Msg(_face(32, "y"), 2, device, s, 52)
    for _ in range(4):
        m2.step()
    assert _slots()[0] == base[0] + 1


def test_slots_off(device):
    import torch
    import ompi_amd
    L = ompi_amd.lib()
    L.ddt_tune(b"slots", 0)
    try:
        s = torch.cuda.Stream(device)
        m = _Msg(_face(32, "y"), 2, device, s, 61)
        n0 = _slots()[3]
        for _ in range(4):
            m.step()
        assert _slots()[3] == n0
    finally:
        L.ddt_tune(b"slots", 1)


def test_large_launches_keep_their_arguments(device):
    """Only launches of at most slot_max_kb packed KiB bind (a slot kernel's extra record load
    costs a large latency-bound launch more than the host saves)."""
    import torch
    import ompi_amd
    L = ompi_amd.lib()
    L.ddt_tune(b"slot_max_kb", 16)
    try:
        s = torch.cuda.Stream(device)
        m = _Msg(_face(32, "y"), 3, device, s, 81)   # 24 KiB packed
        n0 = _slots()
        for _ in range(4):
            m.step()
        assert _slots()[2:] == n0[2:]
    finally:
        L.ddt_tune(b"slot_max_kb", 4096)


def test_random_interleaving_of_types_buffers_streams_and_trims(device):
    """A random schedule over twelve small affine types: each step packs and unpacks one type on
    one of two buffer sets and one of two streams, now and then destroys a type and builds it
    again, or trims; every step moves the oracle's bytes (bindings bind, fall back, end and bind
    again underneath)."""
    import random
    import torch
    from ompi_amd._lib import lib
    rng = random.Random(1234)
    streams = [torch.cuda.Stream(device), torch.cuda.Stream(device)]

    def recipe(i):
        if i % 3 == 0:
            return _face(16 + 8 * (i % 2), "xyz"[i % 3])
        return ("resized", ("vector", 24 + i, 1 + i % 2, 6 + i, ("basic", 16 if i % 2 else 6)), 0, 8 * (6 + i) * (24 + i))

    msgs = [_Msg(recipe(i), 1 + i % 3, device, streams[i % 2], 300 + i) for i in range(12)]
    alt = [torch.zeros_like(m.packed) for m in msgs]
    for step in range(240):
        i = rng.randrange(12)
        m = msgs[i]
        st = streams[rng.randrange(2)]   # one stream per step: the unpack reads what the pack wrote
        for c in (m.cp, m.cu):
            c.set_stream(st, True)
        m.step(packed=alt[i] if rng.random() < 0.2 else None)
        r = rng.random()
        if r < 0.03:
            msgs[i] = _Msg(recipe(i), 1 + i % 3, device, streams[i % 2], 500 + step)
            alt[i] = torch.zeros_like(msgs[i].packed)
        elif r < 0.05:
            torch.cuda.synchronize()
            assert lib().ddt_trim() == 0
    st = _slots()
    assert st[3] > 0 and st[0] <= 8 and st[1] <= 8, st


@pytest.mark.parametrize("mode", ["global", "relaxed"])
def test_binding_during_foreign_capture(device, mode):
    """A set's descriptor upload and its slot bind (event queries, a private-stream upload and
    wait) happen while ANOTHER thread captures a graph: they run in relaxed capture mode, so the
    foreign capture ends intact and replays; the packs are bit-exact."""
    import threading
    import torch
    import ompi_amd
    x = torch.zeros(1024, device=device)
    sb, sa = torch.cuda.Stream(device), torch.cuda.Stream(device)
    g = torch.cuda.CUDAGraph()
    b = R.Built(_face(32, "y"))
    e = b.engine()
    info = b.o.info()
    count, size = 2, info["size"] * 2
    span, origin = R.layout(info, count)
    host = np.random.default_rng(7).integers(1, 255, span, dtype=np.uint8)
    user = torch.from_numpy(host).to(device)
    packed = torch.zeros(size, dtype=torch.uint8, device=device)
    torch.cuda.synchronize()
    started, done = threading.Event(), threading.Event()
    errors = []
    n0 = _slots()

    def capture():
        try:
            with torch.cuda.graph(g, stream=sb, capture_error_mode=mode):
                x.add_(1)
                started.set()
                done.wait(120)
                x.add_(1)
        except Exception as ex:   # noqa: BLE001 -- reported below
            errors.append(repr(ex))
            started.set()

    def packs():
        try:
            started.wait(60)
            c = ompi_amd.Convertor()
            c.set_stream(sa, True)
            for _ in range(4):
                c.prepare_for_send(e, count, user.data_ptr() + origin)
                rc, _, md = c.pack([(packed.data_ptr(), size)])
                assert rc == 1 and md == size
        except Exception as ex:   # noqa: BLE001
            errors.append(repr(ex))
        finally:
            done.set()

    tb, ta = threading.Thread(target=capture), threading.Thread(target=packs)
    tb.start()
    ta.start()
    ta.join(180)
    tb.join(180)
    assert not errors, errors
    g.replay()
    torch.cuda.synchronize()
    assert float(x[0].item()) == 2.0
    ref = np.frombuffer(b.o.pack(count, host, origin, 0, size, element_granular=False), dtype=np.uint8)
    np.testing.assert_array_equal(packed.cpu().numpy(), ref)
    assert _slots()[3] > n0[3]   # the fourth pack ran from its slot


def test_a_set_that_moves_to_other_buffers_rebinds(device):
    """Bound on buffers A, then used on buffers B: the second call on B binds B beside A (a
    double-buffered exchange); C binds a third binding (up to 8 per set, r6: threads sharing a
    type bring their own buffers); with all 8 in use a ninth pair of buffers launches with
    arguments, and every call moves the right bytes."""
    import torch
    s = torch.cuda.Stream(device)
    m = _Msg(_face(32, "z"), 2, device, s, 91)
    for _ in range(3):
        m.step()
    assert _slots()[0] == 1 and _slots()[1] == 1
    b, c = torch.zeros_like(m.packed), torch.zeros_like(m.packed)
    n0 = _slots()[3]
    m.step(packed=b)     # first call on B: with arguments
    assert _slots()[3] == n0
    m.step(packed=b)     # second: binds B, argument-free
    m.step()             # A is still bound
    st = _slots()
    assert st[3] == n0 + 4 and st[0] == 2 and st[1] == 2, st
    m.step(packed=c)
    m.step(packed=c)     # binds C beside A and B
    st2 = _slots()
    assert st2[3] == st[3] + 2 and st2[0] == 3 and st2[1] == 3, st2
    more = [torch.zeros_like(m.packed) for _ in range(6)]
    for p in more:       # D..I: five more bind (8 in all), the sixth finds every binding in use
        m.step(packed=p)
        m.step(packed=p)
    st3 = _slots()
    assert st3[0] == 8 and st3[1] == 8, st3
    n1 = st3[3]
    m.step(packed=more[-1])   # the ninth pair: no binding was free, launched with arguments
    assert _slots()[3] == n1
    m.step()                  # A is still bound
    assert _slots()[3] == n1 + 2


def test_double_buffered_exchange_alternates_two_bindings(device):
    """Send buffers alternating A, B, A, B ... (a double-buffered halo): from the third call on
    every launch is argument-free."""
    import torch
    s = torch.cuda.Stream(device)
    m = _Msg(_face(32, "y"), 2, device, s, 93)
    b = torch.zeros_like(m.packed)
    for i in range(4):
        m.step(packed=b if i % 2 else None)
    n0 = _slots()[3]
    for i in range(6):
        m.step(packed=b if i % 2 else None)
    assert _slots()[3] == n0 + 12


def test_threads_bind_launch_and_evict_concurrently(device):
    """Four threads, each with its own stream and three small types, packing and unpacking at
    once (ctypes releases the GIL in the calls): bindings, argument-free launches and releases
    race under the table lock; every step of every thread moves the oracle's bytes."""
    import threading
    import torch
    errors = []

    def worker(t):
        try:
            s = torch.cuda.Stream(device)
            msgs = [_Msg(("resized", ("vector", 20 + 3 * t + i, 1 + i % 2, 7 + t + i, ("basic", 16)), 0,
                          8 * (7 + t + i) * (20 + 3 * t + i)), 1 + i, device, s, 1000 + 10 * t + i)
                    for i in range(3)]
            for k in range(25):
                msgs[k % 3].step()
        except Exception as ex:   # noqa: BLE001 -- reported below
            errors.append(repr(ex))

    ts = [threading.Thread(target=worker, args=(t,)) for t in range(4)]
    for th in ts:
        th.start()
    for th in ts:
        th.join(300)
    assert not errors, errors[:3]
    assert _slots()[3] > 0


def test_ending_binding_waits_for_a_capturing_stream(device):
    """a binding whose end cannot record its fences (its stream is capturing) stays
    taken and "ending" -- never rebound, never freed without fences -- and a later bind attempt
    (after the capture) records them and frees the slot."""
    import torch
    from ompi_amd._lib import lib
    s = torch.cuda.Stream(device)
    m = _Msg(_face(32, "y"), 2, device, s, 81)
    for _ in range(3):
        m.step()
    ks = [k for k in range(NSLOT) if lib().ddt_slot_state(0, k) & 1]
    assert len(ks) == 1, [lib().ddt_slot_state(0, k) for k in range(NSLOT)]
    k = ks[0]
    keep = (m.user, m.out, m.packed)   # the buffers outlive the capture (torch's allocator)
    x = torch.zeros(16, device=device)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s, capture_error_mode="relaxed"):
        x.add_(1)
        del m   # type, plan and convertors go while their stream captures: no fence can be recorded
        gc.collect()
        during = lib().ddt_slot_state(0, k)
    assert during & 3 == 3, during          # still taken, ending: no bind may reuse it
    assert during >> 8 >= 1                 # its streams kept for the retry
    g.replay()
    torch.cuda.synchronize()
    assert lib().ddt_slot_state(0, k) & 3 == 3
    # a new hot set's bind attempts retry the fences (the stream no longer captures)
    m2 = _Msg(_face(32, "z"), 2, device, s, 82)
    for _ in range(3):
        m2.step()
    torch.cuda.synchronize()
    assert lib().ddt_slot_state(0, k) & 2 == 0, lib().ddt_slot_state(0, k)
    assert float(x[0]) == 1.0
    del keep
