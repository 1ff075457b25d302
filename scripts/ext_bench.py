#!/usr/bin/env python3
"""SURVEY.md §8f row 4 measured: MPI_Pack_external / MPI_Unpack_external (external32, big
endian) of the BASELINE configs' types with device buffers -- a native pack into HBM scratch
plus the conversion kernel (ddt_ext_kernel), synchronous like the reference -- beside the
native pack / unpack of the same message; and the raw iovec export rate
(opal_convertor_raw: iovecs per second).  Not the driver's bench."""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
import ompi_amd  # noqa: E402
from ompi_amd import recipe as ER  # noqa: E402

GiB = float(1 << 30)


def wall(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - a)
    return statistics.median(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="cfg1,cfg2,cfg3,cfg5")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    for name in args.configs.split(","):
        recipe, count, desc = bench.make_workload(name)
        dt = ER.build_committed(recipe)
        info = dt.info()
        S = info["size"] * count
        span, origin = bench.layout(info, count)
        user = torch.randint(1, 255, (span,), dtype=torch.uint8, device=dev)
        back = torch.zeros(span, dtype=torch.uint8, device=dev)
        es = ompi_amd.pack_external_size(count, dt)
        ext = torch.empty(es, dtype=torch.uint8, device=dev)
        pk = torch.empty(S, dtype=torch.uint8, device=dev)
        t_pe = wall(lambda: ompi_amd.pack_external(user.data_ptr() + origin, count, dt, ext.data_ptr(), es, 0))
        t_ue = wall(lambda: ompi_amd.unpack_external(ext.data_ptr(), es, 0, back.data_ptr() + origin, count, dt))
        t_p = wall(lambda: ompi_amd.pack(user.data_ptr() + origin, count, dt, pk.data_ptr(), S, 0))
        t_u = wall(lambda: ompi_amd.unpack(pk.data_ptr(), S, 0, back.data_ptr() + origin, count, dt))
        print(json.dumps({"config": name, "workload": desc["workload"], "packed_bytes": S, "external_bytes": es,
                          "pack_external_us": round(t_pe * 1e6, 1), "unpack_external_us": round(t_ue * 1e6, 1),
                          "pack_us": round(t_p * 1e6, 1), "unpack_us": round(t_u * 1e6, 1),
                          "pack_external_GiBs": round(es / t_pe / GiB, 1),
                          "unpack_external_GiBs": round(es / t_ue / GiB, 1)}), flush=True)
        del user, back, ext, pk


if __name__ == "__main__":
    main()
