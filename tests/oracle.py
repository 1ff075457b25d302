"""ctypes wrapper of the CPU oracle (oracle/ddt_oracle.c) -- test infrastructure only.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load this.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
ORACLE_LIB = os.path.join(ORACLE_DIR, "_build", "libddt_oracle.so")

_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)
    return ORACLE_LIB


def lib():
    global _lib
    if _lib is None:
        src = os.path.join(ORACLE_DIR, "ddt_oracle.c")
        if not os.path.exists(ORACLE_LIB) or (
                os.path.exists(src) and os.path.getmtime(src) > os.path.getmtime(ORACLE_LIB)):
            build()
        L = ctypes.CDLL(ORACLE_LIB)
        vp, i64, i = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int
        sig = {
            "ort_basic": (vp, [i]), "ort_empty": (vp, []), "ort_dup": (vp, [vp]),
            "ort_free": (None, [vp]),
            "ort_contiguous": (vp, [i64, vp]),
            "ort_vector": (vp, [i64, i64, i64, vp]), "ort_hvector": (vp, [i64, i64, i64, vp]),
            "ort_indexed": (vp, [i64, vp, vp, vp]), "ort_hindexed": (vp, [i64, vp, vp, vp]),
            "ort_indexed_block": (vp, [i64, i64, vp, vp]),
            "ort_hindexed_block": (vp, [i64, i64, vp, vp]),
            "ort_struct": (vp, [i64, vp, vp, vp]),
            "ort_subarray": (vp, [i, vp, vp, vp, i, vp]),
            "ort_darray": (vp, [i, i, i, vp, vp, vp, vp, i, vp]),
            "ort_resized": (vp, [vp, i64, i64]),
            "ort_info": (None, [vp, vp]), "ort_run_at": (None, [vp, i64, vp]),
            "ort_run_tid": (i64, [vp, i64]),
            "ort_pack": (i64, [vp, i64, vp, i64, vp, i64]),
            "ort_pack_bytes": (i64, [vp, i64, vp, i64, vp, i64]),
            "ort_set_position": (i64, [vp, i64, i64, i]),
            "ort_unpack": (i64, [vp, i64, vp, i64, vp, i64]),
            "ort_run_mt": (i64, [vp, i64, vp, vp, i, i]),
            "ort_raw": (i64, [vp, i64, i64, i64, i64, vp, vp, vp]),
            "ort_external": (i64, [vp, i64, vp, vp, i]),
            "ort_external_size": (i64, [vp]),
            "ort_commit": (None, [vp]),
            "ort_opt_used": (i64, [vp]), "ort_opt_at": (None, [vp, i64, vp]),
            "ort_opt_flags": (ctypes.c_uint32, [vp]),
            "ort_desc_used": (i64, [vp]), "ort_desc_at": (None, [vp, i64, vp]),
            "ort_commit_info": (None, [vp, vp]),
            "ort_optimize_config": (None, [i64, i64, i64, i]),
            "ort_consolidate": (vp, [vp, i64, i64]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def _arr(a, dt):
    a = np.ascontiguousarray(np.asarray(a, dtype=dt))
    return a, a.ctypes.data_as(ctypes.c_void_p)


class OType:
    """An oracle type (flattened MPI type map)."""

    def __init__(self, h):
        if not h:
            raise ValueError("oracle returned null")
        self.h = ctypes.c_void_p(h)

    def __del__(self):
        try:
            if self.h:
                lib().ort_free(self.h)
        except Exception:
            pass

    def info(self) -> dict:
        out = (ctypes.c_int64 * 8)()
        lib().ort_info(self.h, out)
        keys = ("size", "lb", "ub", "true_lb", "true_ub", "align", "flags", "nruns")
        return dict(zip(keys, list(out)))

    def runs(self):
        n = self.info()["nruns"]
        out = (ctypes.c_int64 * 3)()
        res = []
        for r in range(n):
            lib().ort_run_at(self.h, r, out)
            res.append((out[0], out[1], out[2]))
        return res

    def typed_runs(self):
        """[(disp, len, esize, opal id)] of the flattened type map, in type-map order."""
        return [r + (int(lib().ort_run_tid(self.h, i)),) for i, r in enumerate(self.runs())]

    # --- descriptions (Open MPI's dt_elem_desc_t entries, as 7-tuples
    #     (flags, type, count|items, loops, blocklen|size, extent, disp|first_elem_disp)) ---
    def desc(self):
        """opal_datatype_t::desc as opal_datatype_add builds it (no sentinel)."""
        out = (ctypes.c_int64 * 7)()
        res = []
        for i in range(int(lib().ort_desc_used(self.h))):
            lib().ort_desc_at(self.h, i, out)
            res.append(tuple(out))
        return res

    def opt_desc(self, sentinel: bool = False):
        """opal_datatype_t::opt_desc after opal_datatype_commit (the optimizer restated in
        oracle/ddt_oracle.c); with `sentinel` the END_LOOP at [used] is included."""
        out = (ctypes.c_int64 * 7)()
        n = int(lib().ort_opt_used(self.h))
        res = []
        for i in range(n + (1 if sentinel and n else 0)):
            lib().ort_opt_at(self.h, i, out)
            res.append(tuple(out))
        return res

    def commit_info(self) -> dict:
        """stack_depth / bdt_used after commit (opal_datatype_optimize.c:1777,
        opal_datatype_add.c:306) and the two descriptions' lengths."""
        out = (ctypes.c_int64 * 4)()
        lib().ort_commit_info(self.h, out)
        return dict(zip(("stack_depth", "bdt_used", "desc_used", "opt_used"), list(out)))

    def restricted(self) -> bool:
        """OPAL_DATATYPE_OPTIMIZED_RESTRICTED after commit (a mixed-type region was re-typed)."""
        return bool(lib().ort_opt_flags(self.h) & 0x10000)

    @property
    def size(self):
        return self.info()["size"]

    @property
    def extent(self):
        i = self.info()
        return i["ub"] - i["lb"]

    # --- data movement (numpy byte arrays; base = address of the type origin) ---
    def pack(self, count: int, user: np.ndarray, origin: int, position: int, length: int,
             element_granular: bool = True) -> bytes:
        out = np.zeros(max(length, 1), dtype=np.uint8)
        base = user.ctypes.data + origin
        fn = lib().ort_pack if element_granular else lib().ort_pack_bytes
        n = fn(self.h, count, ctypes.c_void_p(base), position, out.ctypes.data_as(ctypes.c_void_p),
               length)
        return out[:n].tobytes()

    def unpack(self, count: int, user: np.ndarray, origin: int, position: int, data: bytes) -> int:
        src = np.frombuffer(data, dtype=np.uint8).copy()
        base = user.ctypes.data + origin
        return lib().ort_unpack(self.h, count, ctypes.c_void_p(base), position,
                                src.ctypes.data_as(ctypes.c_void_p), len(data))

    def set_position(self, count: int, position: int, send: bool = True) -> int:
        """Where opal_convertor_set_position leaves a fresh convertor of `count` instances
        (send convertors snap to the predefined-element boundary, opal_convertor.c:458-470)."""
        return int(lib().ort_set_position(self.h, count, position, int(send)))

    def pack_all(self, count: int, user: np.ndarray, origin: int) -> bytes:
        total = count * self.size
        return self.pack(count, user, origin, 0, total, element_granular=False)

    def raw(self, count: int, base: int, position: int, cap: int):
        """opal_convertor_raw from `position`: ([(addr, len)], bytes described)."""
        addr = np.zeros(max(cap, 1), dtype=np.int64)
        ln = np.zeros(max(cap, 1), dtype=np.int64)
        n = ctypes.c_int64()
        got = lib().ort_raw(self.h, count, base, position, cap, addr.ctypes.data, ln.ctypes.data,
                            ctypes.byref(n))
        return [(int(addr[i]), int(ln[i])) for i in range(n.value)], int(got)

    def external_size(self) -> int:
        """external32 bytes of one instance, -1 if a type has no fixed external form."""
        return int(lib().ort_external_size(self.h))

    def pack_external(self, count: int, user: np.ndarray, origin: int):
        """MPI_Pack_external of `count` instances (bytes), or None when unsupported."""
        es = self.external_size()
        if es < 0:
            return None
        out = np.zeros(max(es * count, 1), dtype=np.uint8)
        lib().ort_external(self.h, count, ctypes.c_void_p(user.ctypes.data + origin),
                           out.ctypes.data, 1)
        return out[:es * count].tobytes()

    def unpack_external(self, count: int, user: np.ndarray, origin: int, data: bytes) -> int:
        buf = np.frombuffer(data, dtype=np.uint8).copy()
        return int(lib().ort_external(self.h, count, ctypes.c_void_p(user.ctypes.data + origin),
                                      buf.ctypes.data, 0))

    def run_mt(self, count, user_ptr: int, buf_ptr: int, nthreads: int, unpack: bool) -> int:
        return lib().ort_run_mt(self.h, count, ctypes.c_void_p(user_ptr), ctypes.c_void_p(buf_ptr),
                                nthreads, int(unpack))


def basic(type_id: int) -> OType:
    return OType(lib().ort_basic(type_id))


def contiguous(count, old):
    return OType(lib().ort_contiguous(count, old.h))


def consolidate(old, count, threshold=250):
    """ompi_datatype_consolidate_create: contiguous(count, old) with the opt_desc of
    opal_datatype_optimize_from_contiguous, or None where the reference keeps (count, old)."""
    h = lib().ort_consolidate(old.h, count, threshold)
    return OType(h) if h else None


def vector(count, blen, stride, old):
    return OType(lib().ort_vector(count, blen, stride, old.h))


def hvector(count, blen, stride, old):
    return OType(lib().ort_hvector(count, blen, stride, old.h))


def indexed(blens, disps, old):
    b, bp = _arr(blens, np.int64)
    d, dp = _arr(disps, np.int64)
    return OType(lib().ort_indexed(len(b), bp, dp, old.h))


def hindexed(blens, disps, old):
    b, bp = _arr(blens, np.int64)
    d, dp = _arr(disps, np.int64)
    return OType(lib().ort_hindexed(len(b), bp, dp, old.h))


def indexed_block(blen, disps, old):
    d, dp = _arr(disps, np.int64)
    return OType(lib().ort_indexed_block(len(d), blen, dp, old.h))


def hindexed_block(blen, disps, old):
    d, dp = _arr(disps, np.int64)
    return OType(lib().ort_hindexed_block(len(d), blen, dp, old.h))


def struct(blens, disps, types):
    b, bp = _arr(blens, np.int64)
    d, dp = _arr(disps, np.int64)
    arr = (ctypes.c_void_p * len(types))(*[t.h.value for t in types])
    return OType(lib().ort_struct(len(b), bp, dp, ctypes.cast(arr, ctypes.c_void_p)))


def darray(size, rank, gsizes, distribs, dargs, psizes, order, old):
    g, gp = _arr(gsizes, np.int64)
    di, dip = _arr(distribs, np.int32)
    da, dap = _arr(dargs, np.int32)
    ps, psp = _arr(psizes, np.int32)
    return OType(lib().ort_darray(size, rank, len(g), gp, dip, dap, psp, order, old.h))


def subarray(sizes, subsizes, starts, order, old):
    s, sp = _arr(sizes, np.int64)
    ss, ssp = _arr(subsizes, np.int64)
    st, stp = _arr(starts, np.int64)
    return OType(lib().ort_subarray(len(s), sp, ssp, stp, order, old.h))


def resized(old, lb, extent):
    return OType(lib().ort_resized(old.h, lb, extent))


def dup(old):
    return OType(lib().ort_dup(old.h))


def optimize_config(growth: int = 10, unroll_items: int = 8, unroll_bytes: int = 128,
                    preserve_type: bool = True) -> None:
    """The optimizer's MCA parameters for later commits (opal_datatype_module.c:85-90)."""
    lib().ort_optimize_config(growth, unroll_items, unroll_bytes, int(bool(preserve_type)))
