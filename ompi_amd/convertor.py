"""Host-side mirror of the Open MPI convertor (opal/datatype/opal_convertor.h) over
libddt_hip.so, plus the MPI_Pack / MPI_Unpack front end.

Buffers are passed as raw addresses or as objects with ``data_ptr()`` (torch tensors:
device memory and streams are PyTorch's plumbing; the data movement is the HIP engine).
"""
from __future__ import annotations

import ctypes
from typing import List, Sequence, Tuple

from ._lib import IOVec, check, lib
from .datatype import Datatype


def addr(x) -> int:
    if x is None:
        return 0
    if hasattr(x, "data_ptr"):
        return int(x.data_ptr())
    if isinstance(x, int):
        return x
    raise TypeError(f"cannot take the address of {type(x)}")


def stream_handle(s) -> int:
    if s is None:
        return 0
    if hasattr(s, "cuda_stream"):
        return int(s.cuda_stream)
    return int(s)


class Convertor:
    """opal_convertor_t: prepare once, then pack/unpack iovec fragments from the current position."""

    def __init__(self):
        self.h = ctypes.c_void_p(lib().ddt_convertor_create())
        if not self.h:
            raise MemoryError("ddt_convertor_create")

    def close(self):
        if self.h:
            lib().ddt_convertor_destroy(self.h)
            self.h = ctypes.c_void_p(0)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def prepare_for_send(self, dt: Datatype, count: int, buf) -> "Convertor":
        check(lib().ddt_convertor_prepare_for_send(self.h, dt.handle, count, addr(buf)),
              "ddt_convertor_prepare_for_send")
        return self

    def prepare_for_recv(self, dt: Datatype, count: int, buf) -> "Convertor":
        check(lib().ddt_convertor_prepare_for_recv(self.h, dt.handle, count, addr(buf)),
              "ddt_convertor_prepare_for_recv")
        return self

    def prepare_for_raw(self, dt: Datatype, count: int, buf) -> "Convertor":
        """prepare_for_send without the device check: raw export needs no data."""
        check(lib().ddt_convertor_prepare_for_raw(self.h, dt.handle, count, addr(buf)),
              "ddt_convertor_prepare_for_raw")
        return self

    def clone(self, position: int | None = None, copy_stack: bool = False) -> "Convertor":
        """opal_convertor_clone / clone_with_position: a new convertor on the same message."""
        c = Convertor()
        if position is None:
            check(lib().ddt_convertor_clone(self.h, c.h, int(copy_stack)), "ddt_convertor_clone")
        else:
            p = ctypes.c_size_t(position)
            check(lib().ddt_convertor_clone_with_position(self.h, c.h, int(copy_stack), ctypes.byref(p)),
                  "ddt_convertor_clone_with_position")
        return c

    def need_buffers(self) -> bool:
        """opal_convertor_need_buffers: False when the user buffer is the packed stream."""
        return bool(lib().ddt_convertor_need_buffers(self.h))

    def current_pointer(self) -> int:
        p = ctypes.c_void_p()
        check(lib().ddt_convertor_get_current_pointer(self.h, ctypes.byref(p)), "get_current_pointer")
        return int(p.value or 0)

    def offset_pointer(self, offset: int) -> int:
        p = ctypes.c_void_p()
        check(lib().ddt_convertor_get_offset_pointer(self.h, offset, ctypes.byref(p)), "get_offset_pointer")
        return int(p.value or 0)

    @property
    def unpacked_size(self) -> int:
        s = ctypes.c_size_t()
        check(lib().ddt_convertor_get_unpacked_size(self.h, ctypes.byref(s)), "get_unpacked_size")
        return int(s.value)

    def cleanup(self) -> "Convertor":
        """opal_convertor_cleanup: reusable, unprepared and completed."""
        check(lib().ddt_convertor_cleanup(self.h), "ddt_convertor_cleanup")
        return self

    def raw(self, max_iov: int):
        """opal_convertor_raw: (1 if the whole message is described else 0,
        [(address, length)] of user memory in type-map order, bytes described)."""
        arr = (IOVec * max(max_iov, 1))()
        n = ctypes.c_uint32(max_iov)
        length = ctypes.c_size_t(0)
        rc = check(lib().ddt_convertor_raw(self.h, arr, ctypes.byref(n), ctypes.byref(length)),
                   "ddt_convertor_raw")
        return rc, [(int(arr[i].iov_base or 0), int(arr[i].iov_len)) for i in range(n.value)], \
            int(length.value)

    def set_stream(self, stream, async_: bool = True) -> None:
        check(lib().ddt_convertor_set_stream(self.h, stream_handle(stream), int(async_)),
              "ddt_convertor_set_stream")

    def _advance(self, fn, iovs: Sequence[Tuple[object, int]]):
        n = len(iovs)
        arr = (IOVec * max(n, 1))()
        for i, (b, ln) in enumerate(iovs):
            arr[i].iov_base = addr(b)
            arr[i].iov_len = int(ln)
        out_size = ctypes.c_uint32(n)
        max_data = ctypes.c_size_t(0)
        rc = check(fn(self.h, arr, ctypes.byref(out_size), ctypes.byref(max_data)), fn.__name__)
        lens: List[int] = [int(arr[i].iov_len) for i in range(out_size.value)]
        return rc, lens, int(max_data.value)

    def pack(self, iovs: Sequence[Tuple[object, int]]):
        """opal_convertor_pack: returns (1 if complete else 0, bytes per iovec used, total)."""
        return self._advance(lib().ddt_convertor_pack, iovs)

    def unpack(self, iovs: Sequence[Tuple[object, int]]):
        """opal_convertor_unpack."""
        return self._advance(lib().ddt_convertor_unpack, iovs)

    def set_position(self, position: int) -> int:
        p = ctypes.c_size_t(position)
        check(lib().ddt_convertor_set_position(self.h, ctypes.byref(p)), "ddt_convertor_set_position")
        return int(p.value)

    @property
    def packed_size(self) -> int:
        s = ctypes.c_size_t()
        check(lib().ddt_convertor_get_packed_size(self.h, ctypes.byref(s)), "get_packed_size")
        return int(s.value)

    @property
    def position(self) -> int:
        s = ctypes.c_size_t()
        check(lib().ddt_convertor_get_position(self.h, ctypes.byref(s)), "get_position")
        return int(s.value)

    @property
    def completed(self) -> bool:
        return bool(lib().ddt_convertor_is_completed(self.h))


# ------------------------------------------------------------------ MPI front end
def pack_size(incount: int, dt: Datatype) -> int:
    s = ctypes.c_size_t()
    check(lib().ddt_pack_size(incount, dt.handle, ctypes.byref(s)), "ddt_pack_size")
    return int(s.value)


def pack(inbuf, incount: int, dt: Datatype, outbuf, outsize: int, position: int = 0) -> int:
    """MPI_Pack: returns the new position."""
    p = ctypes.c_size_t(position)
    check(lib().ddt_pack(addr(inbuf), incount, dt.handle, addr(outbuf), outsize, ctypes.byref(p)),
          "ddt_pack")
    return int(p.value)


def unpack(inbuf, insize: int, position: int, outbuf, outcount: int, dt: Datatype) -> int:
    """MPI_Unpack: returns the new position."""
    p = ctypes.c_size_t(position)
    check(lib().ddt_unpack(addr(inbuf), insize, ctypes.byref(p), addr(outbuf), outcount, dt.handle),
          "ddt_unpack")
    return int(p.value)


def pack_window(dt: Datatype, count: int, buf, offset: int, dst, max_len: int, stream=None) -> int:
    """UCX generic-datatype pack (pml_ucx_datatype.c:72-88): bytes [offset, offset+max_len)."""
    n = ctypes.c_size_t()
    check(lib().ddt_pack_window(dt.handle, count, addr(buf), offset, addr(dst), max_len,
                                ctypes.byref(n), stream_handle(stream)), "ddt_pack_window")
    return int(n.value)


def unpack_window(dt: Datatype, count: int, buf, offset: int, src, length: int, stream=None) -> None:
    check(lib().ddt_unpack_window(dt.handle, count, addr(buf), offset, addr(src), length,
                                  stream_handle(stream)), "ddt_unpack_window")


def copy_content_same_ddt(dt: Datatype, count: int, dst, src, stream=None) -> None:
    """opal_datatype_copy_content_same_ddt: typed device-to-device copy in one launch."""
    check(lib().ddt_copy_content_same_ddt(dt.handle, count, addr(dst), addr(src),
                                          stream_handle(stream)), "ddt_copy_content_same_ddt")


def sndrcv(sbuf, scount: int, stype, rbuf, rcount: int, rtype, stream=None) -> None:
    """ompi_datatype_sndrcv: local send/recv between typed device buffers; a type of None
    marks that side as MPI_PACKED bytes."""
    check(lib().ddt_sndrcv(addr(sbuf), scount, stype.handle if stype is not None else None,
                           addr(rbuf), rcount, rtype.handle if rtype is not None else None,
                           stream_handle(stream)), "ddt_sndrcv")


# ------------------------------------------------------------------ external32
def pack_external_size(incount: int, dt: Datatype, datarep: str = "external32") -> int:
    """MPI_Pack_external_size."""
    s = ctypes.c_ssize_t()
    check(lib().ddt_pack_external_size(datarep.encode(), incount, dt.handle, ctypes.byref(s)),
          "ddt_pack_external_size")
    return int(s.value)


def pack_external(inbuf, incount: int, dt: Datatype, outbuf, outsize: int, position: int = 0,
                  datarep: str = "external32") -> int:
    """MPI_Pack_external (big-endian external32 stream): returns the new position."""
    p = ctypes.c_ssize_t(position)
    check(lib().ddt_pack_external(datarep.encode(), addr(inbuf), incount, dt.handle, addr(outbuf),
                                  outsize, ctypes.byref(p)), "ddt_pack_external")
    return int(p.value)


def unpack_external(inbuf, insize: int, position: int, outbuf, outcount: int, dt: Datatype,
                    datarep: str = "external32") -> int:
    """MPI_Unpack_external: returns the new position."""
    p = ctypes.c_ssize_t(position)
    check(lib().ddt_unpack_external(datarep.encode(), addr(inbuf), insize, ctypes.byref(p),
                                    addr(outbuf), outcount, dt.handle), "ddt_unpack_external")
    return int(p.value)
