"""ddt_raw.c restated (ompi/test/datatype/ddt_raw.c:128-346, types from ddt_lib.c).

The reference's raw test extracts every datatype of its list through `opal_convertor_raw` with a
budget of 5 iovecs per call (`local_copy_ddt_raw`, :99-143; `test_upper`, :52-89 for the 500x500
upper triangle) until the convertor completes, and passes when the lengths of the extracted
regions add up to count x size (:136-141).  Here the engine's `ddt_convertor_raw` does the same
walk; it must cover count x size exactly, stop every call at 5 iovecs, and give, call for call,
the iovec list the oracle's `opal_convertor_raw` restatement gives (`ort_raw`,
opal_convertor_raw.c:65-283).  No data moves, so this runs on CPU.
"""
from __future__ import annotations

import pytest

import ompi_amd
from tests import recipes as R

INT1, INT4, INT8, FLOAT4, FLOAT8 = 4, 6, 7, 15, 16
F8, I4 = ("basic", FLOAT8), ("basic", INT4)
BASE = 1 << 40
IOV_NUM = 5   # ddt_raw.c:147


def upper_matrix(n):   # ddt_lib.c:124-147
    return ("indexed", [n - i for i in range(n)], [i * n + i for i in range(n)], F8)


def strange():   # ddt_lib.c:379-449 with USE_RESIZED: sdata_intern {i1, gap, i2}, sstrange {counter, v[10], last}
    pdt1 = ("resized", ("indexed_block", 1, [0, 2], I4), 0, 12)
    pdt2 = ("resized", ("struct", [1, 10, 1], [0, 4, 124], [I4, pdt1, I4]), 0, 128)
    return ("contig", 10, pdt2)


BLACS_LEN = [13, 13, 13, 13, 13, 13, 12, 11, 10, 9, 8, 7, 6, 5, 4, 3, 2, 1]
BLACS_IDX = [x // 4 for x in (1144, 1232, 1320, 1408, 1496, 1584, 1676, 1768, 1860, 1952, 2044, 2136,
                              2228, 2320, 2412, 2504, 2596, 2688)]

# (name, recipe, count) in the order ddt_raw.c's main runs local_copy_ddt_raw / test_upper
CASES = [
    ("inversed_vector_int_10", ("vector", 10, 1, 2, I4), 100),                       # :160-164
    ("strange", strange(), 1),                                                          # :167-171
    ("upper_matrix_100", upper_matrix(100), 1),                                         # :175-179
    ("upper_matrix_500", upper_matrix(500), 1),                                         # :183 test_upper(500)
    ("double_x4500", F8, 4500),                                                         # :231-235
    ("contig_4500_x1", ("contig", 4500, F8), 1),                                        # :240-244
    ("contig_450_x10", ("contig", 450, F8), 10),                                        # :245-249
    ("contig_45_x100", ("contig", 45, F8), 100),                                        # :250-254
    ("contig_100_x45", ("contig", 100, F8), 45),                                        # :255-259
    ("contig_10_x450", ("contig", 10, F8), 450),                                        # :260-264
    ("contig_1_x4500", ("contig", 1, F8), 4500),                                        # :265-269
    ("vector_450_10_11", ("vector", 450, 10, 11, F8), 1),                               # :275-283
    ("struct_char_double", ("struct", [1, 1], [0, 8], [("basic", INT1), F8]), 4500),    # :289-293 (ddt_lib.c:220-238)
    ("twice_two_doubles", ("vector", 2, 2, 5, F8), 4500),                               # :298-302
    ("blacs", ("indexed", BLACS_LEN, BLACS_IDX, I4), 4500),                             # :307-314
    ("blacs1_int", ("vector", 7, 1, 3, I4), 1),                                         # :319-323
]


@pytest.mark.parametrize("name,recipe,count", CASES, ids=[c[0] for c in CASES])
def test_ddt_raw_c(name, recipe, count):
    b = R.Built(recipe)
    info = b.o.info()
    total = info["size"] * count
    base = BASE + R.layout(info, count)[1]
    c = ompi_amd.Convertor()
    c.prepare_for_raw(b.engine(), count, base)
    pos, calls, covered = 0, 0, 0
    while True:
        rc, iovs, n = c.raw(IOV_NUM)
        ref, rn = b.o.raw(count, base, pos, IOV_NUM)
        assert iovs == ref and n == rn, (name, calls, pos)
        assert len(iovs) <= IOV_NUM and sum(ln for _, ln in iovs) == n
        covered += n
        pos += n
        calls += 1
        if rc == 1:
            break
        assert iovs, "no progress"
    # ddt_raw.c:136-141: "Not all raw description was been extracted" unless this is 0
    assert covered == total, (name, covered, total)
    assert c.position == total
