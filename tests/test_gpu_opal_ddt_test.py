"""opal_datatype_test.c restated on device buffers (test/datatype/opal_datatype_test.c:568-809,
types from test/datatype/opal_ddt_lib.c).

The reference's opal-level driver copies each type through a send convertor and a receive
convertor in fixed-size pieces (local_copy_with_convertor, :322) and through a send convertor of
one type and a receive convertor of another (local_copy_with_convertor_2datatypes, :207-320: the
two must finish on the same piece, :261-265), optionally resetting both convertors to 0 and back
to the running length after every piece (RESET_CONVERTORS, :285-297, which must land exactly on
that length).  Here every piece moves device memory through the engine's convertors and the
receive buffer must end equal to the oracle's unpack of the oracle's pack (the reference
convertor's bytes).  test_gpu_parity.test_reference_ddt_test_c covers ddt_test.c, the ompi-level
twin of this driver; this file adds the types and pairs only opal_datatype_test.c runs.
"""
from __future__ import annotations

import numpy as np
import pytest

from . import recipes as R
from .test_gpu_parity import _dev, _host

pytestmark = pytest.mark.gpu

INT1, INT4, FLOAT4, FLOAT8 = 4, 6, 15, 16
F8 = ("basic", FLOAT8)

# opal_ddt_lib.c:201-232 create_strange_dt: {double @0, char @8} resized to sizeof(sdata_intern)
# (12 bytes, so the doubles sit at 4-byte phases), 10 of them contiguous
STRANGE = ("contig", 10, ("resized", ("struct", [1, 1], [0, 8], [F8, ("basic", INT1)]), 0, 12))
# :260-272 create_struct_constant_gap_resized_ddt: doubles @8 and @16 of a 24-byte structure
CONSTANT_GAP = ("resized", ("struct", [1, 1], [8, 16], [F8, F8]), 0, 24)
# :59-69 test_create_twice_two_doubles
TWICE_TWO = ("vector", 2, 2, 5, F8)
# :95-109 test_create_blacs_type: 18 int blocks of 13..1
BLACS_LEN = [13, 13, 13, 13, 13, 13, 12, 11, 10, 9, 8, 7, 6, 5, 4, 3, 2, 1]
BLACS_IDX = [x // 4 for x in (1144, 1232, 1320, 1408, 1496, 1584, 1676, 1768, 1860, 1952, 2044, 2136,
                              2228, 2320, 2412, 2504, 2596, 2688)]
BLACS = ("indexed", BLACS_LEN, BLACS_IDX, ("basic", INT4))
# :135-159 test_struct: {2 floats @0, {double, char} @16, 3 chars @26} (dumped only there; packed here)
TEST_STRUCT = ("struct", [2, 1, 3], [0, 16, 26],
               [("basic", FLOAT4), ("struct", [1, 1], [0, 8], [F8, ("basic", INT1)]), ("basic", INT1)])
# :532-558 upper_matrix(100): row i holds 100 - i doubles from the diagonal
UPPER = ("indexed", [100 - i for i in range(100)], [i * 101 for i in range(100)], F8)


def _copy(send, scount, recv, rcount, chunk, device, reset=None):
    """local_copy_with_convertor_2datatypes (:207-320) on device memory; with send == recv the
    same walk as local_copy_with_convertor (:322)."""
    import torch
    import ompi_amd
    bs, br = R.Built(send), R.Built(recv)
    si, ri = bs.o.info(), br.o.info()
    size = si["size"] * scount
    assert ri["size"] * rcount == size
    sspan, sorig = R.layout(si, scount)
    rspan, rorig = R.layout(ri, rcount)
    host = R.fill(sspan, 91)
    src = _dev(host, device)
    dst = torch.zeros(rspan, dtype=torch.uint8, device=device)   # :239 the receiver starts zeroed
    tmp = torch.empty(chunk, dtype=torch.uint8, device=device)
    cs = ompi_amd.Convertor().prepare_for_send(bs.engine(), scount, src.data_ptr() + sorig)
    cr = ompi_amd.Convertor().prepare_for_recv(br.engine(), rcount, dst.data_ptr() + rorig)
    done1 = done2 = 0
    length = 0
    while not (done1 and done2):
        assert not (done1 or done2), "the send and the receive must finish on the same piece (:261-265)"
        md = 0
        if not done1:
            done1, _, md = cs.pack([(tmp, chunk)])
        if not done2:
            done2, _, got = cr.unpack([(tmp, md)])
            assert got == md
        length += md
        # RESET_CONVERTORS (on by default, opal_ddt_lib.c:27): local_copy_with_convertor resets
        # the send convertor while it is not done (:389-401), the two-type copy both (:285-297)
        for c in ((cs, cr) if reset == "both" else (cs,) if reset == "send" and not done1 else ()):
            assert c.set_position(0) == 0
            assert c.set_position(length) == length
    assert length == size
    stream = bs.o.pack(scount, host, sorig, 0, size, element_granular=False)
    exp = np.zeros(rspan, dtype=np.uint8)
    br.o.unpack(rcount, exp, rorig, 0, stream)
    np.testing.assert_array_equal(_host(dst), exp)


# (name, type, count, pieces) as opal_datatype_test.c:579-793 runs local_copy_with_convertor
SAME_TYPE = [
    ("contig_int1_x10", ("contig", 10, ("basic", INT1)), 100, [956]),                    # :580-584
    ("strange", STRANGE, 1, [956]),                                                       # :589-593
    ("upper_matrix_100", UPPER, 1, [48]),                                                 # :598-602
    ("float8", F8, 4500, [12]),                                                           # :666-669
    ("vector_450_10_11", ("vector", 450, 10, 11, F8), 1, [12, 82, 6000, 36000]),         # :721-732
    ("constant_gap_resized_100", CONSTANT_GAP, 100, [11, 82]),                           # :740-747
    ("constant_gap_resized_1500", CONSTANT_GAP, 1500, [6000]),                           # :748
    ("constant_gap_resized_10000", CONSTANT_GAP, 10000, [36000]),                        # :750
    ("twice_two_doubles", TWICE_TWO, 4500, [12]),                                         # :769-773
    ("blacs", BLACS, 4500, [956, 16 * 1024, 64 * 1024]),                                  # :780-789
    ("test_struct", TEST_STRUCT, 100, [100]),
]


@pytest.mark.parametrize("name,dt,count,pieces", SAME_TYPE, ids=[s[0] for s in SAME_TYPE])
def test_local_copy_with_convertor(device, name, dt, count, pieces):
    for p in pieces:
        _copy(dt, count, dt, count, p, device, reset="send")


# local_copy_with_convertor_2datatypes calls (:669-789), send type == receive type, the pieces
# the reference pairs with them; and the one pair of different types, blacs1 -> blacs2 (:796-800)
TWO_TYPES = [
    ("float8", F8, 4500, F8, 4500, 12),
    ("vector_450_10_11_12", ("vector", 450, 10, 11, F8), 1, ("vector", 450, 10, 11, F8), 1, 12),
    ("vector_450_10_11_6000", ("vector", 450, 10, 11, F8), 1, ("vector", 450, 10, 11, F8), 1, 6000),
    ("constant_gap_81", CONSTANT_GAP, 100, CONSTANT_GAP, 100, 81),
    ("constant_gap_666", CONSTANT_GAP, 1500, CONSTANT_GAP, 1500, 666),
    ("constant_gap_1111", CONSTANT_GAP, 10000, CONSTANT_GAP, 10000, 1111),
    ("struct_char_double", ("struct", [1, 1], [0, 8], [("basic", INT1), F8]), 4500,
     ("struct", [1, 1], [0, 8], [("basic", INT1), F8]), 4500, 12),
    ("twice_two_doubles", TWICE_TWO, 4500, TWICE_TWO, 4500, 12),
    ("blacs_956", BLACS, 4500, BLACS, 4500, 956),
    ("blacs_64k", BLACS, 4500, BLACS, 4500, 64 * 1024),
    ("blacs1_to_blacs2", ("vector", 7, 1, 3, ("basic", INT4)), 1, ("vector", 7, 1, 2, ("basic", INT4)), 1, 100),
    # a send and a receive type of the same signature but different shapes, in pieces
    ("vector_to_contig", ("vector", 450, 10, 11, F8), 1, ("contig", 4500, F8), 1, 82),
    ("constant_gap_to_vector", CONSTANT_GAP, 1500, ("vector", 1500, 2, 3, F8), 1, 666),
]


@pytest.mark.parametrize("reset", [None, "both"])
@pytest.mark.parametrize("name,st,sc,rt,rc,chunk", TWO_TYPES, ids=[t[0] for t in TWO_TYPES])
def test_local_copy_with_convertor_2datatypes(device, name, st, sc, rt, rc, chunk, reset):
    _copy(st, sc, rt, rc, chunk, device, reset=reset)
