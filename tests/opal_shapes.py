"""Open MPI's own objects, built in memory the way Open MPI builds them, for driving the
fAdvance bridge (bridge/opal_datatype_hip_bridge.c) exactly as the reference drives its
movers.  Test infrastructure only.

* ctypes mirrors of opal_datatype_t, dt_elem_desc_t and opal_convertor_t (the layout of
  include/opal_layout.h; `check_layout` compares them with the compiled bridge);
* committed descriptions as arrays of 32-byte entries with the END_LOOP sentinel at
  [used] (opal_datatype_optimize.c:454-465): hand-written ones (SURVEY.md Appendix A
  records the reference's opt_desc for the BASELINE shapes) and flat ones, one DATA
  entry per run of the oracle's type map;
* restatements of the convertor entry points the bridge sits behind:
  OPAL_CONVERTOR_PREPARE + opal_convertor_prepare_for_{send,recv}
  (opal_convertor.c:526-591, :616-696), opal_convertor_pack / _unpack (:255-349) and
  opal_convertor_set_position (opal_convertor.h:357-394).  Like
  pack_description_sweep.c:877-965, the movers are swapped after prepare
  (opal_hip_bridge_attach).
"""
from __future__ import annotations

import ctypes
import struct

import numpy as np

from ompi_amd._lib import IOVec

c_size_t, c_ssize_t = ctypes.c_size_t, ctypes.c_ssize_t

# opal_convertor.h:55-76, opal_datatype.h:79-142
F_PREDEFINED, F_COMMITTED, F_CONTIGUOUS, F_NO_GAPS, F_DATA = 0x2, 0x4, 0x10, 0x20, 0x100
CONVERTOR_DATATYPE_MASK = 0x0000FFFF
CONVERTOR_RECV, CONVERTOR_SEND = 0x00400000, 0x00800000
CONVERTOR_HOMOGENEOUS, CONVERTOR_NO_OP, CONVERTOR_COMPLETED = 0x01000000, 0x02000000, 0x04000000
CONVERTOR_HAS_REMOTE_SIZE = 0x08000000
CONVERTOR_ACCELERATOR, CONVERTOR_ACCELERATOR_ASYNC = 0x10000000, 0x20000000
OPAL_SUCCESS, OPAL_ERR_NOT_SUPPORTED = 0, -8

# OPAL predefined sizes (opal_datatype_module.c:143-180, LP64)
BASIC_SIZE = {4: 1, 5: 2, 6: 4, 7: 8, 8: 16, 9: 1, 10: 2, 11: 4, 12: 8, 13: 16, 14: 2, 15: 4, 16: 8,
              17: 16, 18: 16, 19: 4, 20: 8, 21: 16, 22: 32, 23: 1, 24: 4, 25: 8, 26: 8, 27: 32}


class OpalObject(ctypes.Structure):
    _fields_ = [("obj_class", ctypes.c_void_p), ("obj_reference_count", ctypes.c_int32)]


class DtTypeDesc(ctypes.Structure):
    _fields_ = [("length", c_size_t), ("used", c_size_t), ("desc", ctypes.c_void_p)]


class OpalDatatype(ctypes.Structure):
    _fields_ = [("super", OpalObject), ("flags", ctypes.c_uint32), ("bdt_used", ctypes.c_uint32),
                ("size", c_size_t), ("true_lb", c_ssize_t), ("true_ub", c_ssize_t),
                ("lb", c_ssize_t), ("ub", c_ssize_t), ("nbElems", c_size_t),
                ("id", ctypes.c_uint16), ("align", ctypes.c_uint16), ("stack_depth", ctypes.c_uint32),
                ("name", ctypes.c_char * 64), ("desc", DtTypeDesc), ("opt_desc", DtTypeDesc),
                ("ptypes", ctypes.c_void_p)]


class DtStack(ctypes.Structure):
    _fields_ = [("index", ctypes.c_int32), ("type", ctypes.c_int16), ("padding", ctypes.c_int16),
                ("count", c_size_t), ("disp", c_ssize_t)]


class AccelStream(ctypes.Structure):
    _fields_ = [("super", OpalObject), ("stream", ctypes.c_void_p)]


ADVANCE = ctypes.CFUNCTYPE(ctypes.c_int32, ctypes.c_void_p, ctypes.POINTER(IOVec),
                           ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(c_size_t))
POSITION = ctypes.CFUNCTYPE(ctypes.c_int32, ctypes.c_void_p, ctypes.POINTER(c_size_t))


class OpalConvertor(ctypes.Structure):
    _fields_ = [("super", OpalObject), ("pDesc", ctypes.c_void_p), ("use_desc", ctypes.c_void_p),
                ("count", c_size_t), ("remote_size", c_size_t), ("master", ctypes.c_void_p),
                ("fAdvance", ctypes.c_void_p),
                ("bConverted", c_size_t), ("partial_length", c_size_t), ("local_size", c_size_t),
                ("pBaseBuf", ctypes.c_void_p), ("pStack", ctypes.c_void_p), ("cbmemcpy", ctypes.c_void_p),
                ("flags", ctypes.c_uint32), ("stack_pos", ctypes.c_uint32), ("stack_size", ctypes.c_uint32),
                ("remoteArch", ctypes.c_uint32),
                ("sizes", ctypes.c_void_p), ("fPosition", ctypes.c_void_p),
                ("static_stack", DtStack * 5), ("stream", ctypes.c_void_p)]


def bridge_lib():
    """libddt_hip.so with the bridge entry points typed."""
    from ompi_amd import lib
    L = lib()
    if not getattr(L, "_bridge_typed", False):
        vp = ctypes.c_void_p
        sig = {
            "opal_pack_hip": (ctypes.c_int32, [vp, ctypes.POINTER(IOVec), ctypes.POINTER(ctypes.c_uint32),
                                               ctypes.POINTER(c_size_t)]),
            "opal_unpack_hip": (ctypes.c_int32, [vp, ctypes.POINTER(IOVec), ctypes.POINTER(ctypes.c_uint32),
                                                 ctypes.POINTER(c_size_t)]),
            "opal_position_hip": (ctypes.c_int32, [vp, ctypes.POINTER(c_size_t)]),
            "opal_hip_bridge_attach": (ctypes.c_int, [vp]),
            "opal_hip_bridge_datatype_destruct": (None, [vp]),
            "opal_hip_bridge_datatype_commit": (ctypes.c_int, [vp]),
            "opal_hip_bridge_finalize": (None, []),
            "opal_hip_bridge_stats": (None, [ctypes.POINTER(c_size_t)]),
            "opal_hip_bridge_layout": (None, [ctypes.POINTER(c_size_t)]),
        }
        for n, (r, a) in sig.items():
            f = getattr(L, n)
            f.restype, f.argtypes = r, a
        L._bridge_typed = True
    return L


def check_layout():
    out = (c_size_t * 8)()
    bridge_lib().opal_hip_bridge_layout(out)
    mine = [ctypes.sizeof(OpalDatatype), OpalDatatype.opt_desc.offset, ctypes.sizeof(OpalConvertor),
            OpalConvertor.bConverted.offset, OpalConvertor.flags.offset, OpalConvertor.fPosition.offset,
            OpalConvertor.stream.offset, 32]
    return list(out), mine


def stats():
    out = (c_size_t * 4)()
    bridge_lib().opal_hip_bridge_stats(out)
    return {"entries": out[0], "imports": out[1], "hits": out[2], "stale": out[3]}


# ------------------------------------------------------------------ descriptions
def data(tid, count, blocklen, extent, disp, flags=F_DATA | F_CONTIGUOUS):
    """DATA entry (ddt_elem_desc_t, opal_datatype_internal.h:130-136); blocklen in elements."""
    return struct.pack("<HHIQqq", flags | F_DATA, tid, count, blocklen, extent, disp)


def loop(loops, items, extent, flags=0):
    """LOOP entry (ddt_loop_desc_t :147-153): `items` counts itself and its body."""
    return struct.pack("<HHIIIQq", flags, 0, items, loops, 0, (1 << 64) - 1, extent)


def end_loop(items, size, first_elem_disp, flags=0):
    """END_LOOP entry (ddt_endloop_desc_t :156-162)."""
    return struct.pack("<HHIIIQq", flags, 1, items, 0xFFFFFFFF, 0, size, first_elem_disp)


class OpalType:
    """A committed opal_datatype_t whose desc is `entries` and whose opt_desc is
    `opt_entries` (default: the same array), each followed by its END_LOOP sentinel
    (opal_datatype_optimize.c:454-465: items = used, the first element's displacement, size)."""

    def __init__(self, entries, size, lb, ub, true_lb, true_ub, flags=0, name=b"ddt", opt_entries=None,
                 first_disp=0):
        entries = list(entries)
        self.raw = np.frombuffer(b"".join(entries + [end_loop(len(entries), size, first_disp)]),
                                 dtype=np.uint8).copy()
        self.dt = OpalDatatype()
        d = self.dt
        d.super.obj_reference_count = 1
        d.flags = flags | F_COMMITTED | F_DATA
        d.size, d.lb, d.ub, d.true_lb, d.true_ub = size, lb, ub, true_lb, true_ub
        d.name = name[:63]
        d.desc.length, d.desc.used, d.desc.desc = len(entries) + 1, len(entries), self.raw.ctypes.data
        if opt_entries is None:
            self.opt_raw = self.raw
            d.opt_desc.length, d.opt_desc.used, d.opt_desc.desc = d.desc.length, d.desc.used, d.desc.desc
        else:
            opt_entries = list(opt_entries)
            self.opt_raw = np.frombuffer(b"".join(opt_entries + [end_loop(len(opt_entries), size, first_disp)]),
                                         dtype=np.uint8).copy()
            d.opt_desc.length, d.opt_desc.used = len(opt_entries) + 1, len(opt_entries)
            d.opt_desc.desc = self.opt_raw.ctypes.data

    @property
    def ptr(self):
        return ctypes.addressof(self.dt)

    @property
    def extent(self):
        return self.dt.ub - self.dt.lb

    def destruct(self):
        bridge_lib().opal_hip_bridge_datatype_destruct(self.ptr)

    def commit_hook(self):
        """What opal_datatype_commit calls last in the patched tree."""
        return bridge_lib().opal_hip_bridge_datatype_commit(self.ptr)


def flat_from_oracle(otype, flags=0):
    """One DATA entry per run of the oracle's type map (a valid, unoptimised description:
    opal_datatype_add emits DATA entries with CREATE_ELEM's count=1 collapse,
    opal_datatype_internal.h:195-209).  Installed as opt_desc it is a description whose
    elements are the type map's own, not the committed carriers: tests of the import only."""
    info = otype.info()
    ents = []
    for disp, ln, esize, tid in otype.typed_runs():
        bs = BASIC_SIZE[tid]
        ents.append(data(tid, 1, ln // bs, ln, disp))
    fl = flags
    if info["flags"] & F_CONTIGUOUS:
        fl |= F_CONTIGUOUS
    if info["flags"] & F_NO_GAPS:
        fl |= F_NO_GAPS
    return OpalType(ents, info["size"], info["lb"], info["ub"], info["true_lb"], info["true_ub"], fl)


def pack_entry(e):
    """A 7-tuple (flags, type, count|items, loops, blocklen|size, extent, disp|first_elem_disp)
    as the 32-byte dt_elem_desc_t."""
    fl, ty, a, lo, b, x, d = e
    if fl & F_DATA:
        return struct.pack("<HHIQqq", fl, ty, a, b, x, d)
    if ty == 0:
        return struct.pack("<HHIIIQq", fl, 0, a, lo, 0, b & ((1 << 64) - 1), x)
    return struct.pack("<HHIIIQq", fl, 1, a, lo & 0xFFFFFFFF, 0, b, d)


def unpack_entries(raw: bytes):
    """32-byte dt_elem_desc_t entries -> 7-tuples (the inverse of pack_entry)."""
    out = []
    for i in range(len(raw) // 32):
        p = raw[32 * i:32 * i + 32]
        fl, ty = struct.unpack_from("<HH", p)
        if fl & F_DATA:
            c, b, x, d = struct.unpack_from("<IQqq", p, 4)
            out.append((fl, ty, c, 0, b, x, d))
        elif ty == 0:
            it, lo, _, un, x = struct.unpack_from("<IIIQq", p, 4)
            out.append((fl, ty, it, lo, un if un < (1 << 63) else -1, x, 0))
        else:
            it, un, _, sz, fd = struct.unpack_from("<IIIQq", p, 4)
            out.append((fl, ty, it, un, sz, 0, fd))
    return out


def from_oracle(otype, flags=0):
    """The opal_datatype_t Open MPI commits for the oracle's type: desc as opal_datatype_add
    builds it, opt_desc as opal_datatype_commit optimizes it (both restated in
    oracle/ddt_oracle.c), OPTIMIZED_RESTRICTED when a region was re-typed.  This is what the
    bridge meets inside Open MPI: use_desc = &opt_desc (opal_convertor.c:533)."""
    info = otype.info()
    fl = flags | (info["flags"] & (F_CONTIGUOUS | F_NO_GAPS)) | (0x10000 if otype.restricted() else 0)
    desc = [pack_entry(e) for e in otype.desc()]
    opt = otype.opt_desc(sentinel=True)
    first = opt[-1][6] if opt else 0
    return OpalType(desc, info["size"], info["lb"], info["ub"], info["true_lb"], info["true_ub"], fl,
                    opt_entries=[pack_entry(e) for e in opt[:-1]], first_disp=first)


# ------------------------------------------------------------------ the convertor
class Convertor:
    """An opal_convertor_t prepared by the restated prepare_for_{send,recv}; `device`
    stands for check_addr's answer (opal_convertor.c:593-608)."""

    def __init__(self):
        self.c = OpalConvertor()
        self.c.super.obj_reference_count = 1
        self.c.pStack = ctypes.addressof(self.c.static_stack)
        self.c.stack_size = 5
        self.c.flags = F_NO_GAPS | CONVERTOR_COMPLETED   # opal_convertor_construct state
        self.stream_obj = None

    @property
    def ptr(self):
        return ctypes.addressof(self.c)

    def prepare(self, otype: OpalType, count: int, buf: int, send: bool, device=True,
                stream=None):
        c, d = self.c, otype.dt
        self.otype = otype
        c.flags &= (CONVERTOR_SEND | CONVERTOR_RECV | CONVERTOR_HOMOGENEOUS | CONVERTOR_ACCELERATOR
                    | CONVERTOR_ACCELERATOR_ASYNC)
        c.flags &= ~(CONVERTOR_SEND | CONVERTOR_RECV | CONVERTOR_ACCELERATOR)
        c.flags |= CONVERTOR_SEND if send else CONVERTOR_RECV
        if device:
            c.flags |= CONVERTOR_ACCELERATOR
        if stream is not None:   # pml_ob1_recvfrag.c:761-769: stream attached, ASYNC set
            # the rocm component's stream object holds a pointer to a malloc'ed hipStream_t
            # cell, not the handle itself (accelerator_rocm_module.c:80, :176-182)
            self.stream_cell = ctypes.c_void_p(stream)
            self.stream_obj = AccelStream()
            self.stream_obj.stream = ctypes.addressof(self.stream_cell)
            c.stream = ctypes.addressof(self.stream_obj)
            c.flags |= CONVERTOR_ACCELERATOR_ASYNC
        # OPAL_CONVERTOR_PREPARE (opal_convertor.c:526-591)
        c.local_size = count * d.size
        c.pBaseBuf = buf
        c.count = count
        c.pDesc = otype.ptr
        c.bConverted = 0
        c.use_desc = otype.ptr + OpalDatatype.opt_desc.offset
        c.fPosition = None
        c.fAdvance = None
        if count == 0 or d.size == 0:
            c.flags |= F_NO_GAPS | CONVERTOR_COMPLETED | CONVERTOR_HAS_REMOTE_SIZE
            c.local_size = c.remote_size = 0
            return OPAL_SUCCESS
        c.flags |= CONVERTOR_DATATYPE_MASK & d.flags
        c.flags |= CONVERTOR_NO_OP | CONVERTOR_HOMOGENEOUS
        c.remote_size = c.local_size
        if (c.flags & F_NO_GAPS) or ((c.flags & F_CONTIGUOUS) and count == 1):
            return OPAL_SUCCESS   # NO_OP: opal_convertor_pack copies it with cbmemcpy
        c.flags &= ~CONVERTOR_NO_OP
        # dispatch (:633-635, :677-679) chose the accelerator movers; swap them like
        # pack_description_sweep.c:877-965 does
        return bridge_lib().opal_hip_bridge_attach(self.ptr)

    # opal_convertor_pack / opal_convertor_unpack (opal_convertor.c:255-349)
    def _advance(self, iovs, pack):
        c = self.c
        arr = (IOVec * max(len(iovs), 1))()
        for i, (p, n) in enumerate(iovs):
            arr[i].iov_base, arr[i].iov_len = p, n
        out = ctypes.c_uint32(len(iovs))
        md = c_size_t(0)
        if c.flags & CONVERTOR_NO_OP:
            return self._no_op(arr, out, md, pack)
        if c.flags & CONVERTOR_COMPLETED:   # OPAL_CONVERTOR_SET_STATUS_BEFORE_PACK_UNPACK
            return 1, [], 0
        fn = ADVANCE(c.fAdvance)
        rc = fn(self.ptr, arr, ctypes.byref(out), ctypes.byref(md))
        return rc, [(arr[i].iov_base, arr[i].iov_len) for i in range(out.value)], md.value

    def _no_op(self, arr, out, md, pack):
        import torch
        c = self.c
        pending = c.local_size - c.bConverted
        base = c.pBaseBuf + c.bConverted + self.otype.dt.true_lb
        used, total = 0, 0
        for i in range(out.value):
            n = min(arr[i].iov_len, pending - total)
            src, dst = (base + total, arr[i].iov_base) if pack else (arr[i].iov_base, base + total)
            _dev_copy(dst, src, n)
            arr[i].iov_len = n
            total += n
            used = i + 1
            if total == pending:
                break
        torch.cuda.synchronize()
        c.bConverted += total
        if c.bConverted == c.local_size:
            c.flags |= CONVERTOR_COMPLETED
            return 1, [(arr[i].iov_base, arr[i].iov_len) for i in range(used)], total
        return 0, [(arr[i].iov_base, arr[i].iov_len) for i in range(used)], total

    def pack(self, iovs):
        return self._advance(iovs, True)

    def unpack(self, iovs):
        return self._advance(iovs, False)

    def set_position(self, position: int) -> int:
        """opal_convertor_set_position (opal_convertor.h:357-394)."""
        c = self.c
        packed = c.local_size
        if packed <= position:
            c.flags |= CONVERTOR_COMPLETED
            c.bConverted = packed
            return packed
        if position == c.bConverted:
            return position
        c.flags &= ~CONVERTOR_COMPLETED
        if not c.fPosition:
            c.bConverted = position
            return position
        p = c_size_t(position)
        rc = POSITION(c.fPosition)(self.ptr, ctypes.byref(p))
        assert rc == OPAL_SUCCESS
        return p.value


def _dev_copy(dst: int, src: int, n: int):
    """cbmemcpy = opal_convertor_accelerator_memcpy (opal_convertor.c:46-63): a device copy."""
    if n <= 0:
        return
    import torch
    from torch.utils import dlpack  # noqa: F401
    s = _wrap(src, n)
    d = _wrap(dst, n)
    d.copy_(s)


def _wrap(ptr: int, n: int):
    """A uint8 CUDA tensor view of device memory at `ptr` (no copy)."""
    import torch

    class _Arr:
        __cuda_array_interface__ = {"shape": (n,), "typestr": "|u1", "data": (ptr, False), "version": 3}
    return torch.as_tensor(_Arr(), device="cuda")
