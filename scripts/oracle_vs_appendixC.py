#!/usr/bin/env python3
"""The CPU baseline anchored to the reference's own timings (round 3).

SURVEY.md Appendix C timed the reference convertor (opal/datatype built from its sources in
the survey's container) on the BASELINE shapes, pack and unpack separately, 1 thread and 8
threads (position-sharded).  This script times the oracle (oracle/ddt_oracle.c, the C
restatement bench.py's cpu_baseline runs) on the same shapes in the same kind of container
(8 CPUs), the same way: whole-message pack, then unpack, GiB/s of packed bytes, median of
repeated trials.  It prints one JSON line per shape with the reference's figures beside the
oracle's and their ratio.  Test infrastructure only (loads the oracle).

Differences in the inputs, stated per line: cfg4 uses SURVEY §8d's LCG displacements (the
survey's probe used an xorshift with duplicates); cfg5 is timed on a 16 Mi-record prefix
(the full 128 Mi records need an 8 GiB run table in the oracle's flat representation).
"""
from __future__ import annotations

import json
import os
import statistics
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from tests import recipes as R  # noqa: E402
import bench  # noqa: E402

GiB = float(1 << 30)
D8, F4 = ("basic", 16), ("basic", 15)
N3 = 512

# (name, recipe, count, reference 1T pack, 1T unpack, 8T pack, 8T unpack) -- SURVEY.md App. C
SHAPES = [
    ("cfg1 vector(1024,1,2) dbl x2048", ("vector", 1024, 1, 2, D8), 2048, 4.78, 3.88, 18.88, 20.77),
    ("cfg2 x-face vector(65536,1,256)", ("vector", 65536, 1, 256, D8), 1, 0.44, 0.33, 1.26, 1.04),
    ("cfg2 y-face vector(256,256,65536)", ("vector", 256, 256, 65536, D8), 1, 6.24, 3.30, 2.85, 3.08),
    ("cfg3 subarray face dim0", ("subarray", [N3] * 3, [1, N3, N3], [N3 - 1, 0, 0], 0, F4), 1, 8.24, 5.74, 4.19, 5.35),
    ("cfg3 subarray face dim1", ("subarray", [N3] * 3, [N3, 1, N3], [0, N3 - 1, 0], 0, F4), 1, 3.95, 3.13, 4.06, 5.00),
    ("cfg3 subarray face dim2", ("subarray", [N3] * 3, [N3, N3, 1], [0, 0, N3 - 1], 0, F4), 1, 0.19, 0.15, 0.90, 0.48),
]


def time_shape(name, recipe, count, ref, trials_s=3.0, note=""):
    b = R.Built(recipe)
    info = b.o.info()
    S = info["size"] * count
    span, origin = R.layout(info, count)
    user = R.fill_fast(span, 7)
    buf = np.zeros(S, dtype=np.uint8)
    ptr = user.ctypes.data + origin
    out = {"shape": name, "packed_bytes": S, "note": note}
    for th in (1, 8):
        for op, unpack in (("pack", False), ("unpack", True)):
            b.o.run_mt(count, ptr, buf.ctypes.data, th, unpack)   # warm (page faults)
            ts, t0 = [], time.perf_counter()
            while (time.perf_counter() - t0 < trials_s and len(ts) < 200) or len(ts) < 3:
                a = time.perf_counter()
                b.o.run_mt(count, ptr, buf.ctypes.data, th, unpack)
                ts.append(time.perf_counter() - a)
            out[f"oracle_{th}T_{op}_GiBs"] = round(S / statistics.median(ts) / GiB, 3)
    keys = ["1T_pack", "1T_unpack", "8T_pack", "8T_unpack"]
    for k, r in zip(keys, ref):
        out[f"reference_{k}_GiBs"] = r
        out[f"ratio_{k}"] = round(out[f"oracle_{k}_GiBs"] / r, 2)
    print(json.dumps(out), flush=True)
    return out


def main():
    only = sys.argv[1:]
    for name, rec, count, *ref in SHAPES:
        if not only or any(o in name for o in only):
            time_shape(name, rec, count, ref)
    if not only or any("cfg4" in o for o in only):
        d = bench.lcg_disps(64 << 20)
        time_shape("cfg4 indexed 64M disps into 1 GiB float", ("indexed_block", 1, d, F4), 1,
                   (0.16, 0.14, 0.75, 0.67), trials_s=6.0,
                   note="LCG displacements (SURVEY 8d), the reference probe used xorshift with duplicates")
    if not only or any("cfg5" in o for o in only):
        st = ("struct", [1, 3], [0, 8], [D8, ("basic", 6)])
        time_shape("cfg5 hvector(16Mi,1,32B) of struct{dbl,int[3]}", ("hvector", 16 << 20, 1, 32, st), 1,
                   (4.98, 4.19, 21.72, 21.32), note="16 Mi-record prefix of the 128 Mi records")


if __name__ == "__main__":
    main()
