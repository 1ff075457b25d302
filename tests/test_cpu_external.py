"""external32: MPI_Pack_external / MPI_Unpack_external.

The oracle (ort_external) restates the external32 convertor of the reference element by
element (opal_copy_functions_heterogeneous.c).  It is pinned here against:
  * the reference's own known answers (ompi/test/datatype/external32.c: htonl/htons of
    int32/int16 contiguous data and of vector(2,1,2) of int);
  * Python's `struct` module with big-endian formats, which is an independent statement of
    the external32 layout (MPI-4.1 §5.14 sizes: long = 4 bytes).
The engine's external sizes are compared with the oracle's on fuzzed types; the GPU
conversion itself is compared in test_gpu_parity.py.
"""
from __future__ import annotations

import random
import struct

import numpy as np
import pytest

import ompi_amd
from tests import oracle as O
from tests import recipes as R


def test_reference_external32_contiguous_int32_int16():
    # external32.c:183-205 and :207-227
    u = np.array([1234, 5678], dtype=np.int32).view(np.uint8).copy()
    got = O.basic(6).pack_external(2, u, 0)
    assert got == struct.pack(">ii", 1234, 5678)
    back = np.full(8, 0xFF, dtype=np.uint8)
    O.basic(6).unpack_external(2, back, 0, got)
    assert back.view(np.int32).tolist() == [1234, 5678]
    u16 = np.array([1234, 5678], dtype=np.int16).view(np.uint8).copy()
    assert O.basic(5).pack_external(2, u16, 0) == struct.pack(">hh", 1234, 5678)


def test_reference_external32_vector_of_int():
    # external32.c:229-266: vector(2, 1, 2, MPI_INT) over {1234, 0, 5678}
    t = O.vector(2, 1, 2, O.basic(6))
    u = np.array([1234, 0, 5678], dtype=np.int32).view(np.uint8).copy()
    got = t.pack_external(1, u, 0)
    assert got == struct.pack(">ii", 1234, 5678)
    back = np.array([-1, -1, -1], dtype=np.int32).view(np.uint8).copy()
    t.unpack_external(1, back, 0, got)
    assert back.view(np.int32).tolist() == [1234, -1, 5678]


def test_struct_against_python_struct_module():
    # struct { int32 a; double b; int16 c[3]; long d; uint64 e; float complex f; bool g }
    # laid out by hand with C alignment; external32 = '>i d 3h i Q 2f ?' (long -> 4 bytes)
    fields = [(6, 1, 0), (16, 1, 8), (5, 3, 16), (25, 1, 24), (12, 1, 32), (20, 1, 40), (23, 1, 48)]
    t = O.struct([n for _, n, _ in fields], [d for _, _, d in fields],
                 [O.basic(tid) for tid, _, _ in fields])
    vals = [(-7, 3.25, (1, -2, 300), -123456789, 2 ** 63 + 5, (1.5, -2.0), True),
            (2 ** 31 - 1, -0.0, (-32768, 0, 32767), 2 ** 40 + 17, 1, (0.0, 1e30), False)]
    ext = info_ext = t.info()["ub"] - t.info()["lb"]
    buf = bytearray(ext * len(vals))
    want = b""
    for i, (a, b, c, d, e, f, g) in enumerate(vals):
        base = i * ext
        struct.pack_into("<i", buf, base + 0, a)
        struct.pack_into("<d", buf, base + 8, b)
        struct.pack_into("<3h", buf, base + 16, *c)
        struct.pack_into("<q", buf, base + 24, d)
        struct.pack_into("<Q", buf, base + 32, e)
        struct.pack_into("<2f", buf, base + 40, *f)
        struct.pack_into("<?", buf, base + 48, g)
        d32 = (d + 2 ** 31) % 2 ** 32 - 2 ** 31   # MPI_LONG travels as its low 32 bits
        want += struct.pack(">id3hiQ2f?", a, b, *c, d32, e, *f, g)
    user = np.frombuffer(bytes(buf), dtype=np.uint8).copy()
    assert info_ext == 56
    got = t.pack_external(len(vals), user, 0)
    assert got == want
    assert t.external_size() == len(want) // len(vals) == 4 + 8 + 6 + 4 + 8 + 8 + 1
    # unpack: sign extension of the 4-byte long
    back = np.zeros_like(user)
    t.unpack_external(len(vals), back, 0, got)
    d0 = struct.unpack_from("<q", back.tobytes(), 24)[0]
    d1 = struct.unpack_from("<q", back.tobytes(), 56 + 24)[0]
    assert d0 == -123456789 and d1 == 17


def test_unsigned_long_zero_extends():
    t = O.basic(26)
    u = np.frombuffer(struct.pack("<Q", 0xFFFFFFFF80000001), dtype=np.uint8).copy()
    got = t.pack_external(1, u, 0)
    assert got == struct.pack(">I", 0x80000001)
    back = np.zeros(8, dtype=np.uint8)
    t.unpack_external(1, back, 0, got)
    assert struct.unpack("<Q", back.tobytes())[0] == 0x80000001


def _quad_be(sign: int, exp: int, frac112: int) -> bytes:
    """IEEE binary128, big-endian (the external32 long double, ompi_datatype_external32.c:95-99)."""
    return ((sign << 127) | (exp << 112) | frac112).to_bytes(16, "big")


def test_long_double_complex_converts_x87_to_ieee_quad():
    """LONG_DOUBLE_COMPLEX (COPY_2SAMETYPE_HETEROGENEOUS_INTERNAL(..., 1),
    opal_copy_functions_heterogeneous.c:779-842): each x87 component becomes a big-endian
    IEEE quad on pack (exact); unpack converts back, and the component's 6 padding bytes
    keep the swapped quad's bytes 10..15 (the in-place f128_to_ldbl store, :558-590)."""
    vals = np.array([1.0, -2.5, 0.1, np.finfo(np.longdouble).tiny / 4, np.inf, -0.0],
                    dtype=np.longdouble)
    assert vals.dtype.itemsize == 16   # x86-64 long double: 80 bits in 16 bytes
    user = vals.view(np.uint8).copy()
    t = O.basic(22)
    ext = t.pack_external(3, user, 0)
    assert t.external_size() == 32 and len(ext) == 96
    assert ext[0:16] == _quad_be(0, 16383, 0)                     # 1.0
    assert ext[16:32] == _quad_be(1, 16384, 1 << 110)             # -2.5 = -1.25 x 2^1
    # 0.1 as x87: mantissa 0xCCCCCCCCCCCCCCCD x 2^-67 -> quad fraction = (m - 2^63) << 49
    m = int.from_bytes(vals[2:3].view(np.uint8)[:8].tobytes(), "little")
    assert ext[32:48] == _quad_be(0, 16383 - 4, (m - (1 << 63)) << 49)
    assert ext[48:64] == _quad_be(0, 0, (1 << 61) << 49)         # x87 denormal 2^-16384
    assert ext[64:80] == _quad_be(0, 0x7FFF, 0)                   # inf
    assert ext[80:96] == _quad_be(1, 0, 0)                        # -0.0
    back = np.zeros(96, dtype=np.uint8)
    t.unpack_external(3, back, 0, ext)
    for i in range(6):
        comp, q = back[16 * i:16 * i + 16].tobytes(), ext[16 * i:16 * i + 16][::-1]
        assert comp[:10] == user[16 * i:16 * i + 10].tobytes()
        assert comp[10:] == q[10:]


def test_long_double_unpack_rounds_to_nearest_even():
    """A quad with more precision than x87 holds (f128_to_ldbl, libgcc __trunctfxf2): the 49
    dropped fraction bits round to nearest, ties to even, carrying into the exponent."""
    t = O.basic(22)
    cases = [((1 << 112) - 1, 1 << 63, 16384),     # all ones: rounds up into the next binade
             (1 << 48, 1 << 63, 16383),             # tie, even mantissa: stays
             ((1 << 49) | (1 << 48), (1 << 63) | 2, 16383)]   # tie, odd mantissa: rounds up
    for frac, want_m, want_e in cases:
        q = _quad_be(0, 16383, frac)
        back = np.zeros(32, dtype=np.uint8)
        t.unpack_external(1, back, 0, q + q)
        assert int.from_bytes(back[:8].tobytes(), "little") == want_m
        assert int.from_bytes(back[8:10].tobytes(), "little") == want_e


def test_long_double_and_float128_swap_whole():
    """FLOAT12 (MPI_LONG_DOUBLE) and FLOAT16 (_Float128) use the copy functions without the
    long-double flag (opal_copy_functions_heterogeneous.c:1033-1034, :1058-1059): 16 bytes
    reversed, no format change."""
    raw = np.arange(32, dtype=np.uint8)
    for tid in (17, 18):
        t = O.basic(tid)
        ext = t.pack_external(2, raw, 0)
        assert ext == raw[:16].tobytes()[::-1] + raw[16:].tobytes()[::-1]
        assert ompi_amd.pack_external_size(2, __import__("ompi_amd").datatype.predefined(tid)) == 32


def test_float128_complex_has_no_external_form():
    """FLOAT128_COMPLEX: the reference routes its quad components through ldbl_to_f128 as if
    they were long doubles (:1082-1083); the engine refuses it rather than guess."""
    assert O.basic(27).external_size() == -1
    from ompi_amd import datatype as D
    with pytest.raises(ompi_amd.DDTError) as ei:
        ompi_amd.pack_external_size(1, D.predefined(D.FLOAT128_COMPLEX))
    assert ei.value.code == -10


@pytest.mark.parametrize("seed", range(3))
def test_engine_external_size_matches_oracle(seed):
    rng = random.Random(7300 + seed)
    for _ in range(150):
        b = R.Built(R.random_recipe(rng, basics=R.EXT_BASICS))
        count = rng.choice([0, 1, 3])
        es = ompi_amd.pack_external_size(count, b.engine())
        assert es == b.o.external_size() * count, b.recipe


def test_oracle_external_roundtrip_fuzz():
    rng = random.Random(7400)
    for n in range(120):
        b = R.Built(R.random_recipe(rng, basics=R.EXT_BASICS))
        info = b.o.info()
        if info["size"] == 0:
            continue
        count = rng.choice([1, 2])
        span, origin = R.layout(info, count)
        user = R.fill(span, n)
        ext = b.o.pack_external(count, user, origin)
        assert len(ext) == b.o.external_size() * count
        # the native stream and the external stream hold the same elements: for types
        # without LONG or converted long doubles the byte multisets agree
        if b.o.external_size() == info["size"] and 22 not in {r[3] for r in b.o.typed_runs()}:
            native = b.o.pack(count, user, origin, 0, info["size"] * count, element_granular=False)
            assert sorted(native) == sorted(ext)
