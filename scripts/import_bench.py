#!/usr/bin/env python3
"""Host time of ddt_type_from_opal_desc (the bridge's one-time import of a committed opt_desc) on a
cfg4-shaped description: N DATA entries FLOAT4 count 2 blen 1 (the optimizer's indexed pairs,
opal_datatype_optimize.c:1179-1185), unique random displacements.  CPU only.
Usage: python scripts/import_bench.py N"""
import ctypes, time, sys
import numpy as np
sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from ompi_amd._lib import lib
L = lib()
N = int(sys.argv[1])
# cfg4's committed description: N DATA entries FLOAT4 count 2 blen 1, extent = d2 - d1 (LCG pairs)


# vectorised LCG is awkward; use a permutation of a 2^28 range instead (unique displacements)
rng = np.random.default_rng(1)
d = (rng.choice(1 << 28, size=2 * N, replace=False).astype(np.int64)) * 4
dt = np.dtype([("flags", "<u2"), ("type", "<u2"), ("count", "<u4"), ("blen", "<u8"), ("extent", "<i8"), ("disp", "<i8")])
desc = np.zeros(N + 1, dtype=dt)
desc["flags"][:N] = 0x100 | 0x10
desc["type"][:N] = 15
desc["count"][:N] = 2
desc["blen"][:N] = 1
desc["extent"][:N] = d[1::2] - d[0::2]
desc["disp"][:N] = d[0::2]
desc["type"][N] = 1   # END_LOOP sentinel
lo, hi = int(d.min()), int(d.max()) + 4
out = ctypes.c_void_p()
t0 = time.perf_counter()
rc = L.ddt_type_from_opal_desc(desc.ctypes.data, N, 8 * N, lo, hi, lo, hi, ctypes.byref(out))
t1 = time.perf_counter()
print(f"N={N} entries: rc={rc} import {t1 - t0:.3f} s ({N / (t1 - t0) / 1e6:.1f} M entries/s)")
