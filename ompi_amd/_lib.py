"""ctypes binding of libddt_hip.so (the C ABI declared in include/ddt_hip.h).

The library is built in-tree by ``__graft_entry__.build()`` (ompi_amd/csrc/Makefile).
There is no fallback: if the shared object is missing, importing the product raises.
"""
from __future__ import annotations

import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# DDT_LIB_PATH selects another build of the same library (e.g. the host-ASAN build of
# scripts/asan_cpu_tests.sh); the default is the in-tree gfx950 build.
LIB_PATH = os.environ.get("DDT_LIB_PATH") or os.path.join(HERE, "libddt_hip.so")

c_size_t = ctypes.c_size_t
c_ssize_t = ctypes.c_ssize_t
c_int = ctypes.c_int
c_int32 = ctypes.c_int32
c_uint32 = ctypes.c_uint32
c_int64 = ctypes.c_int64
c_void_p = ctypes.c_void_p
P = ctypes.POINTER


class IOVec(ctypes.Structure):
    _fields_ = [("iov_base", c_void_p), ("iov_len", c_size_t)]


# name -> (restype, argtypes); every entry is declared in include/ddt_hip.h
SIGNATURES = {
    "ddt_predefined": (c_void_p, [c_int]),
    "ddt_type_create_contiguous": (c_int, [c_size_t, c_void_p, P(c_void_p)]),
    "ddt_type_create_vector": (c_int, [c_size_t, c_size_t, c_ssize_t, c_void_p, P(c_void_p)]),
    "ddt_type_create_hvector": (c_int, [c_size_t, c_size_t, c_ssize_t, c_void_p, P(c_void_p)]),
    "ddt_type_create_indexed": (c_int, [c_size_t, c_void_p, c_void_p, c_void_p, P(c_void_p)]),
    "ddt_type_create_hindexed": (c_int, [c_size_t, c_void_p, c_void_p, c_void_p, P(c_void_p)]),
    "ddt_type_create_indexed_block": (c_int, [c_size_t, c_size_t, c_void_p, c_void_p, P(c_void_p)]),
    "ddt_type_create_hindexed_block": (c_int, [c_size_t, c_size_t, c_void_p, c_void_p, P(c_void_p)]),
    "ddt_type_create_struct": (c_int, [c_size_t, c_void_p, c_void_p, c_void_p, P(c_void_p)]),
    "ddt_type_create_subarray": (c_int, [c_int, c_void_p, c_void_p, c_void_p, c_int, c_void_p,
                                         P(c_void_p)]),
    "ddt_type_create_darray": (c_int, [c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                                       c_int, c_void_p, P(c_void_p)]),
    "ddt_type_create_resized": (c_int, [c_void_p, c_ssize_t, c_ssize_t, P(c_void_p)]),
    "ddt_type_dup": (c_int, [c_void_p, P(c_void_p)]),
    "ddt_type_commit": (c_int, [c_void_p]),
    "ddt_type_destroy": (c_int, [P(c_void_p)]),
    "ddt_type_size": (c_int, [c_void_p, P(c_size_t)]),
    "ddt_type_get_extent": (c_int, [c_void_p, P(c_ssize_t), P(c_ssize_t)]),
    "ddt_type_get_true_extent": (c_int, [c_void_p, P(c_ssize_t), P(c_ssize_t)]),
    "ddt_type_flags": (c_uint32, [c_void_p]),
    "ddt_type_info": (c_int, [c_void_p, P(c_int64)]),
    "ddt_type_commit_info": (c_int, [c_void_p, P(c_int64)]),
    "ddt_type_consolidate": (c_int, [c_void_p, c_size_t, P(c_void_p)]),
    "ddt_type_from_opal_desc": (c_int, [c_void_p, c_size_t, c_size_t, c_ssize_t, c_ssize_t,
                                        c_ssize_t, c_ssize_t, P(c_void_p)]),
    "ddt_type_to_opal_desc": (c_int64, [c_void_p, c_void_p, c_size_t]),
    "ddt_type_prepare_device": (c_int, [c_void_p]),
    "ddt_type_to_opal_opt_desc": (c_int64, [c_void_p, c_void_p, c_size_t, ctypes.POINTER(ctypes.c_uint32)]),
    "ddt_convertor_create": (c_void_p, []),
    "ddt_convertor_destroy": (None, [c_void_p]),
    "ddt_convertor_prepare_for_send": (c_int, [c_void_p, c_void_p, c_size_t, c_void_p]),
    "ddt_convertor_prepare_for_recv": (c_int, [c_void_p, c_void_p, c_size_t, c_void_p]),
    "ddt_convertor_pack": (c_int32, [c_void_p, P(IOVec), P(c_uint32), P(c_size_t)]),
    "ddt_convertor_unpack": (c_int32, [c_void_p, P(IOVec), P(c_uint32), P(c_size_t)]),
    "ddt_pack_external_size": (c_int, [ctypes.c_char_p, c_size_t, c_void_p, P(c_ssize_t)]),
    "ddt_pack_external": (c_int, [ctypes.c_char_p, c_void_p, c_size_t, c_void_p, c_void_p,
                                  c_ssize_t, P(c_ssize_t)]),
    "ddt_unpack_external": (c_int, [ctypes.c_char_p, c_void_p, c_ssize_t, P(c_ssize_t), c_void_p,
                                    c_size_t, c_void_p]),
    "ddt_convertor_prepare_for_raw": (c_int, [c_void_p, c_void_p, c_size_t, c_void_p]),
    "ddt_convertor_raw": (c_int32, [c_void_p, P(IOVec), P(c_uint32), P(c_size_t)]),
    "ddt_convertor_set_position": (c_int, [c_void_p, P(c_size_t)]),
    "ddt_type_snap_position": (c_int, [c_void_p, c_size_t, P(c_size_t)]),
    "ddt_convertor_get_packed_size": (c_int, [c_void_p, P(c_size_t)]),
    "ddt_convertor_get_position": (c_int, [c_void_p, P(c_size_t)]),
    "ddt_convertor_is_completed": (c_int, [c_void_p]),
    "ddt_convertor_clone": (c_int, [c_void_p, c_void_p, c_int]),
    "ddt_convertor_clone_with_position": (c_int, [c_void_p, c_void_p, c_int, P(c_size_t)]),
    "ddt_convertor_need_buffers": (c_int, [c_void_p]),
    "ddt_convertor_get_current_pointer": (c_int, [c_void_p, P(c_void_p)]),
    "ddt_convertor_get_offset_pointer": (c_int, [c_void_p, c_size_t, P(c_void_p)]),
    "ddt_convertor_get_unpacked_size": (c_int, [c_void_p, P(c_size_t)]),
    "ddt_convertor_cleanup": (c_int, [c_void_p]),
    "ddt_convertor_set_stream": (c_int, [c_void_p, c_void_p, c_int]),
    "ddt_pack": (c_int, [c_void_p, c_size_t, c_void_p, c_void_p, c_size_t, P(c_size_t)]),
    "ddt_unpack": (c_int, [c_void_p, c_size_t, P(c_size_t), c_void_p, c_size_t, c_void_p]),
    "ddt_pack_size": (c_int, [c_size_t, c_void_p, P(c_size_t)]),
    "ddt_pack_window": (c_int, [c_void_p, c_size_t, c_void_p, c_size_t, c_void_p, c_size_t,
                                P(c_size_t), c_void_p]),
    "ddt_unpack_window": (c_int, [c_void_p, c_size_t, c_void_p, c_size_t, c_void_p, c_size_t,
                                  c_void_p]),
    "ddt_copy_content_same_ddt": (c_int, [c_void_p, c_size_t, c_void_p, c_void_p, c_void_p]),
    "ddt_sndrcv": (c_int, [c_void_p, c_size_t, c_void_p, c_void_p, c_size_t, c_void_p, c_void_p]),
    "ddt_type_plan_info": (c_int, [c_void_p, P(c_int64)]),
    "ddt_get_elements": (c_int, [c_void_p, c_size_t, P(c_size_t)]),
    "ddt_type_engine_info": (c_int, [c_void_p, P(c_int64)]),
    "ddt_type_cache_info": (c_int, [c_void_p, P(c_int64)]),
    "ddt_trim": (c_int, []),
    "ddt_pool_info": (c_int, [P(c_int64)]),
    "ddt_slot_info": (c_int, [P(c_int64)]),
    "ddt_slot_state": (c_int, [c_int, c_int]),
    "ddt_sync_info": (c_int, [P(c_int64)]),
    "ddt_type_plan_leaves": (c_int64, [c_void_p, P(c_int64), c_size_t]),
    "ddt_debug_items": (c_int, [c_void_p, c_size_t, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                                ctypes.c_uint64, c_int, c_void_p, c_size_t, P(c_size_t), P(c_size_t)]),
    "ddt_type_plan_list": (c_int64, [c_void_p, c_size_t, c_void_p, c_void_p, c_size_t]),
    "ddt_debug_host_window": (c_int, [c_void_p, c_size_t, P(ctypes.c_uint64)]),
    "ddt_tune": (c_int, [ctypes.c_char_p, ctypes.c_long]),
    "ddt_selftest": (c_int, []),
    "ddt_version": (ctypes.c_char_p, []),
    "ddt_build_id": (ctypes.c_char_p, []),
    "ddt_last_error": (ctypes.c_char_p, []),
}

_lib = None


def lib():
    """Load libddt_hip.so once; raise if it has not been built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`"
                " (there is no CPU fallback)")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


class DDTError(RuntimeError):
    def __init__(self, code: int, what: str):
        msg = lib().ddt_last_error().decode(errors="replace")
        super().__init__(f"{what} failed with code {code}: {msg}")
        self.code = code


def check(rc: int, what: str) -> int:
    if rc < 0:
        raise DDTError(rc, what)
    return rc
