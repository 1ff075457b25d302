"""Host-side mirror of the Open MPI datatype constructors over libddt_hip.so.

Function names and argument meaning follow ``ompi/datatype/ompi_datatype.h:217-284``
(``ompi_datatype_create_vector(count, bLength, stride, oldType, &newType)`` becomes
``create_vector(count, blocklen, stride, old)``); every call goes straight to the C ABI.
"""
from __future__ import annotations

import ctypes
from typing import Optional, Sequence

import numpy as np

from ._lib import check, lib

# OPAL predefined ids (opal/datatype/opal_datatype_internal.h:71-99)
LB, UB = 2, 3
INT1, INT2, INT4, INT8, INT16 = 4, 5, 6, 7, 8
UINT1, UINT2, UINT4, UINT8, UINT16 = 9, 10, 11, 12, 13
FLOAT2, FLOAT4, FLOAT8, FLOAT12, FLOAT16 = 14, 15, 16, 17, 18
SHORT_FLOAT_COMPLEX, FLOAT_COMPLEX, DOUBLE_COMPLEX, LONG_DOUBLE_COMPLEX = 19, 20, 21, 22
BOOL, WCHAR, LONG, UNSIGNED_LONG, FLOAT128_COMPLEX = 23, 24, 25, 26, 27

FLAG_PREDEFINED = 0x0002
FLAG_COMMITTED = 0x0004
FLAG_CONTIGUOUS = 0x0010
FLAG_NO_GAPS = 0x0020
FLAG_USER_LB = 0x0040
FLAG_USER_UB = 0x0080
FLAG_DATA = 0x0100

ORDER_C = 0
ORDER_FORTRAN = 1


class Datatype:
    """A committed-or-not engine datatype (opaque ``ddt_datatype_t*``)."""

    __slots__ = ("handle", "owned", "name", "subtypes")

    def __init__(self, handle: int, owned: bool = True, name: str = "derived"):
        if not handle:
            raise ValueError("null datatype handle")
        self.handle = ctypes.c_void_p(handle)
        self.owned = owned
        self.name = name
        self.subtypes = ()   # recipe.build_committed: the sub-types it was built from

    # --- lifetime ---------------------------------------------------------
    def commit(self) -> "Datatype":
        check(lib().ddt_type_commit(self.handle), "ddt_type_commit")
        return self

    def destroy(self) -> None:
        if self.owned and self.handle:
            h = ctypes.c_void_p(self.handle.value)
            check(lib().ddt_type_destroy(ctypes.byref(h)), "ddt_type_destroy")
            self.handle = ctypes.c_void_p(0)
            self.owned = False

    def __del__(self):  # best effort, never raise from a finalizer
        try:
            self.destroy()
        except Exception:
            pass

    # --- queries ----------------------------------------------------------
    def info(self) -> dict:
        out = (ctypes.c_int64 * 8)()
        check(lib().ddt_type_info(self.handle, out), "ddt_type_info")
        keys = ("size", "lb", "ub", "true_lb", "true_ub", "align", "flags", "nbElems")
        return dict(zip(keys, list(out)))

    def commit_info(self) -> dict:
        """opal_datatype_t's committed stack_depth and bdt_used (opal_datatype.h:175-187), the
        optimizer flags and whether the type is committed (ddt_type_commit_info)."""
        out = (ctypes.c_int64 * 4)()
        check(lib().ddt_type_commit_info(self.handle, out), "ddt_type_commit_info")
        return dict(zip(("stack_depth", "bdt_used", "opt_flags", "committed"), list(out)))

    def consolidate(self, count: int) -> "Optional[Datatype]":
        """ompi_datatype_consolidate_create: contiguous(count, self) with the opt_desc of
        opal_datatype_optimize_from_contiguous, committed; None where MPI_Pack keeps (count, self)."""
        out = ctypes.c_void_p()
        check(lib().ddt_type_consolidate(self.handle, count, ctypes.byref(out)), "ddt_type_consolidate")
        return Datatype(out.value, owned=True, name=f"consolidated({count})") if out.value else None

    @property
    def size(self) -> int:
        return self.info()["size"]

    @property
    def lb(self) -> int:
        return self.info()["lb"]

    @property
    def extent(self) -> int:
        i = self.info()
        return i["ub"] - i["lb"]

    @property
    def true_lb(self) -> int:
        return self.info()["true_lb"]

    @property
    def true_extent(self) -> int:
        i = self.info()
        return i["true_ub"] - i["true_lb"]

    @property
    def flags(self) -> int:
        return int(lib().ddt_type_flags(self.handle))

    def plan_info(self) -> dict:
        out = (ctypes.c_int64 * 4)()
        check(lib().ddt_type_plan_info(self.handle, out), "ddt_type_plan_info")
        return dict(zip(("leaves", "device_bytes", "list_leaves", "max_dims"), list(out)))

    def get_elements(self, ucount: int):
        """MPI_Get_elements (ompi_datatype_get_elements): basic elements in `ucount` packed
        bytes, or None (MPI_UNDEFINED) when the bytes end inside an element."""
        n = ctypes.c_size_t()
        rc = lib().ddt_get_elements(self.handle, ucount, ctypes.byref(n))
        if rc == -11:
            return None
        check(rc, "ddt_get_elements")
        return int(n.value)

    def engine_info(self) -> dict:
        """State of the address-ordered index-list engine (ddt_type_engine_info)."""
        out = (ctypes.c_int64 * 4)()
        check(lib().ddt_type_engine_info(self.handle, out), "ddt_type_engine_info")
        return dict(zip(("sorted", "device_bytes", "chunks", "slots"), list(out)))

    def to_opal_desc(self) -> bytes:
        """The uncommitted type map as Open MPI dt_elem_desc_t entries (ddt_type_to_opal_desc)."""
        n = lib().ddt_type_to_opal_desc(self.handle, None, 0)
        if n >= 0:
            need = n
        else:
            need = -n
        buf = ctypes.create_string_buffer(max(need, 1) * 32)
        got = check(lib().ddt_type_to_opal_desc(self.handle, buf, need), "ddt_type_to_opal_desc")
        return buf.raw[:got * 32]

    def to_opal_opt_desc(self):
        """(entries, flags): the committed opt_desc as Open MPI would derive it
        (ddt_type_to_opal_opt_desc; flags & 0x10000 = OPAL_DATATYPE_OPTIMIZED_RESTRICTED)."""
        fl = ctypes.c_uint32(0)
        n = lib().ddt_type_to_opal_opt_desc(self.handle, None, 0, ctypes.byref(fl))
        need = n if n >= 0 else -n
        buf = ctypes.create_string_buffer(max(need, 1) * 32)
        got = check(lib().ddt_type_to_opal_opt_desc(self.handle, buf, need, ctypes.byref(fl)),
                    "ddt_type_to_opal_opt_desc")
        return buf.raw[:got * 32], int(fl.value)

    def cache_info(self) -> dict:
        """Descriptor-set cache of the plan (ddt_type_cache_info)."""
        out = (ctypes.c_int64 * 4)()
        check(lib().ddt_type_cache_info(self.handle, out), "ddt_type_cache_info")
        return dict(zip(("cached", "retiring", "pinned", "device"), list(out)))

    def snap_position(self, position: int) -> int:
        """Predefined-element boundary at or below a packed position: where a send convertor's
        set_position lands (opal_convertor_position_generic, opal_convertor.c:458-470)."""
        s = ctypes.c_size_t()
        check(lib().ddt_type_snap_position(self.handle, position, ctypes.byref(s)),
              "ddt_type_snap_position")
        return int(s.value)

    def __repr__(self):
        return f"Datatype({self.name}, {self.info()})"


def predefined(type_id: int, name: str = "") -> Datatype:
    h = lib().ddt_predefined(type_id)
    if not h:
        raise ValueError(f"no predefined type {type_id}")
    return Datatype(h, owned=False, name=name or f"opal{type_id}")


def _new(fn_name: str, *args) -> Datatype:
    out = ctypes.c_void_p()
    check(getattr(lib(), fn_name)(*args, ctypes.byref(out)), fn_name)
    return Datatype(out.value, owned=True, name=fn_name.replace("ddt_type_create_", ""))


def _sizes(a: Sequence[int]) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(a, dtype=np.uint64))


def _disps(a: Sequence[int]) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(a, dtype=np.int64))


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


# --- constructors (ompi_datatype_create_*) ------------------------------------
def create_contiguous(count: int, old: Datatype) -> Datatype:
    return _new("ddt_type_create_contiguous", count, old.handle)


def create_vector(count: int, blocklen: int, stride: int, old: Datatype) -> Datatype:
    return _new("ddt_type_create_vector", count, blocklen, stride, old.handle)


def create_hvector(count: int, blocklen: int, stride_bytes: int, old: Datatype) -> Datatype:
    return _new("ddt_type_create_hvector", count, blocklen, stride_bytes, old.handle)


def create_indexed(blocklens: Sequence[int], disps: Sequence[int], old: Datatype) -> Datatype:
    b, d = _sizes(blocklens), _disps(disps)
    assert b.shape == d.shape
    return _new("ddt_type_create_indexed", len(b), _ptr(b), _ptr(d), old.handle)


def create_hindexed(blocklens: Sequence[int], disps_bytes: Sequence[int], old: Datatype) -> Datatype:
    b, d = _sizes(blocklens), _disps(disps_bytes)
    assert b.shape == d.shape
    return _new("ddt_type_create_hindexed", len(b), _ptr(b), _ptr(d), old.handle)


def create_indexed_block(blocklen: int, disps: Sequence[int], old: Datatype) -> Datatype:
    d = _disps(disps)
    return _new("ddt_type_create_indexed_block", len(d), blocklen, _ptr(d), old.handle)


def create_hindexed_block(blocklen: int, disps_bytes: Sequence[int], old: Datatype) -> Datatype:
    d = _disps(disps_bytes)
    return _new("ddt_type_create_hindexed_block", len(d), blocklen, _ptr(d), old.handle)


def create_struct(blocklens: Sequence[int], disps: Sequence[int], types: Sequence[Datatype]) -> Datatype:
    b, d = _sizes(blocklens), _disps(disps)
    arr = (ctypes.c_void_p * len(types))(*[t.handle.value for t in types])
    return _new("ddt_type_create_struct", len(b), _ptr(b), _ptr(d), ctypes.cast(arr, ctypes.c_void_p))


def create_subarray(sizes: Sequence[int], subsizes: Sequence[int], starts: Sequence[int],
                    order: int, old: Datatype) -> Datatype:
    s, ss, st = _sizes(sizes), _sizes(subsizes), _sizes(starts)
    return _new("ddt_type_create_subarray", len(s), _ptr(s), _ptr(ss), _ptr(st), order, old.handle)


DISTRIBUTE_BLOCK, DISTRIBUTE_CYCLIC, DISTRIBUTE_NONE, DISTRIBUTE_DFLT_DARG = 0, 1, 2, -1


def create_darray(size: int, rank: int, gsizes: Sequence[int], distribs: Sequence[int],
                  dargs: Sequence[int], psizes: Sequence[int], order: int, old: Datatype) -> Datatype:
    """MPI_Type_create_darray (ompi_datatype_create_darray.c:187-312)."""
    g = _sizes(gsizes)
    di = np.ascontiguousarray(np.asarray(distribs, dtype=np.int32))
    da = np.ascontiguousarray(np.asarray(dargs, dtype=np.int32))
    ps = np.ascontiguousarray(np.asarray(psizes, dtype=np.int32))
    return _new("ddt_type_create_darray", size, rank, len(g), _ptr(g), _ptr(di), _ptr(da), _ptr(ps),
                order, old.handle)


def create_resized(old: Datatype, lb: int, extent: int) -> Datatype:
    return _new("ddt_type_create_resized", old.handle, lb, extent)


def duplicate(old: Datatype) -> Datatype:
    out = ctypes.c_void_p()
    check(lib().ddt_type_dup(old.handle, ctypes.byref(out)), "ddt_type_dup")
    return Datatype(out.value, owned=True, name="dup")


def from_opal_desc(desc: bytes, size: int, lb: int, ub: int, true_lb: int, true_ub: int) -> Datatype:
    """Import a committed Open MPI ``dt_elem_desc_t`` array (32-byte entries)."""
    assert len(desc) % 32 == 0
    buf = ctypes.create_string_buffer(desc, len(desc))
    out = ctypes.c_void_p()
    check(lib().ddt_type_from_opal_desc(buf, len(desc) // 32, size, lb, ub, true_lb, true_ub,
                                        ctypes.byref(out)), "ddt_type_from_opal_desc")
    return Datatype(out.value, owned=True, name="opal_desc")


class _Predefs:
    """Lazily created MPI predefined handles (ompi_datatype_module.c mapping)."""

    _map = {
        "MPI_CHAR": INT1, "MPI_SIGNED_CHAR": INT1, "MPI_UNSIGNED_CHAR": UINT1, "MPI_BYTE": UINT1,
        "MPI_SHORT": INT2, "MPI_UNSIGNED_SHORT": UINT2, "MPI_INT": INT4, "MPI_UNSIGNED": UINT4,
        "MPI_LONG": LONG, "MPI_UNSIGNED_LONG": UNSIGNED_LONG, "MPI_LONG_LONG": INT8,
        "MPI_INT8_T": INT1, "MPI_INT16_T": INT2, "MPI_INT32_T": INT4, "MPI_INT64_T": INT8,
        "MPI_UINT8_T": UINT1, "MPI_UINT16_T": UINT2, "MPI_UINT32_T": UINT4, "MPI_UINT64_T": UINT8,
        # x86-64: long double has 64 mantissa digits in 16 bytes -> FLOAT12
        # (ompi_datatype_internal.h:637-638, opal_datatype_constructors.h:267-270)
        "MPI_FLOAT": FLOAT4, "MPI_DOUBLE": FLOAT8, "MPI_LONG_DOUBLE": FLOAT12,
        "MPI_C_FLOAT_COMPLEX": FLOAT_COMPLEX, "MPI_C_DOUBLE_COMPLEX": DOUBLE_COMPLEX,
        "MPI_C_LONG_DOUBLE_COMPLEX": LONG_DOUBLE_COMPLEX,
        "MPI_C_BOOL": BOOL, "MPI_WCHAR": WCHAR,
        # MPI-1 bound markers (ompi_datatype_module.c:92-93; opal_datatype_add.c:158-186)
        "MPI_LB": LB, "MPI_UB": UB,
    }

    def __getattr__(self, name):
        if name not in self._map:
            raise AttributeError(name)
        dt = predefined(self._map[name], name)
        setattr(self, name, dt)
        return dt


MPI = _Predefs()
