#!/usr/bin/env python3
"""The drop-in path measured: BASELINE config 2 (the 256^3 double halo, 16 fields) packed and
unpacked through Open MPI's own convertor slots -- opal-shaped opal_datatype_t /
opal_convertor_t objects (tests/opal_shapes.py) whose fAdvance / fPosition the bridge serves
(bridge/opal_datatype_hip_bridge.c) -- beside the engine's own convertor API, on the same
buffers.  Also the host time of one fragment call through each (a PML's prepare_src loop).
Not the driver's bench."""
from __future__ import annotations

import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import ompi_amd  # noqa: E402
from ompi_amd import recipe as ER  # noqa: E402
from tests import opal_shapes as S  # noqa: E402


def halo_desc(n=256):
    row, plane, field = 8 * n, 8 * n * n, 8 * n * n * n
    ents = [S.data(16, n * n, 1, row, 0), S.data(16, n * n, 1, row, row - 8),
            S.data(16, n, n, plane, 0), S.data(16, n, n, plane, (n - 1) * row),
            S.data(16, 1, n * n, plane, 0), S.data(16, 1, n * n, plane, (n - 1) * plane)]
    return S.OpalType(ents, 6 * 8 * n * n, 0, field, 0, field)


def main():
    dev = torch.device("cuda:0")
    fields, steps = 16, 50
    rec, field = bench.halo_recipe()
    dt = ER.build_committed(rec)
    S_bytes = dt.info()["size"] * fields
    user = torch.randint(1, 255, (fields * field,), dtype=torch.uint8, device=dev)
    pk_e = torch.empty(S_bytes, dtype=torch.uint8, device=dev)
    pk_b = torch.empty(S_bytes, dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream(dev)
    ot = halo_desc()

    ce, cue = ompi_amd.Convertor(), ompi_amd.Convertor()
    for c in (ce, cue):
        c.set_stream(st, True)

    def engine_step():
        ce.prepare_for_send(dt, fields, user)
        ce.pack([(pk_e, S_bytes)])
        cue.prepare_for_recv(dt, fields, user)
        cue.unpack([(pk_e, S_bytes)])

    cb, cub = S.Convertor(), S.Convertor()

    def bridge_step():
        cb.prepare(ot, fields, user.data_ptr(), send=True, stream=st.cuda_stream)
        cb.pack([(pk_b.data_ptr(), S_bytes)])
        cub.prepare(ot, fields, user.data_ptr(), send=False, stream=st.cuda_stream)
        cub.unpack([(pk_b.data_ptr(), S_bytes)])

    out = {}
    for name, fn in (("engine_convertor", engine_step), ("opal_bridge", bridge_step)):
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(steps):
            fn()
        e1.record(st)
        torch.cuda.synchronize()
        t = e0.elapsed_time(e1) / 1e3 / steps
        out[name] = {"step_us": round(t * 1e6, 1), "GiBs": round(2 * S_bytes / t / 2 ** 30, 1)}
    out["same_bytes"] = bool(torch.equal(pk_e, pk_b))

    # host time of one 64 KiB fragment call (prepare + set_position + pack, asynchronous)
    frag = 64 << 10
    def host_us(fn, reps=2000):
        ts = []
        for i in range(reps):
            a = time.perf_counter()
            fn(i)
            ts.append(time.perf_counter() - a)
            if i % 64 == 63:
                torch.cuda.synchronize()
        torch.cuda.synchronize()
        return round(statistics.median(ts) * 1e6, 2)

    def e_frag(i):
        ce.prepare_for_send(dt, fields, user)
        ce.set_position((i % 700) * frag)
        ce.pack([(pk_e.data_ptr() + (i % 700) * frag, frag)])

    def b_frag(i):
        cb.prepare(ot, fields, user.data_ptr(), send=True, stream=st.cuda_stream)
        cb.set_position((i % 700) * frag)
        cb.pack([(pk_b.data_ptr() + (i % 700) * frag, frag)])

    out["fragment_call_host_us"] = {"engine_convertor": host_us(e_frag), "opal_bridge": host_us(b_frag),
                                    "fragment_bytes": frag,
                                    "note": "python/ctypes harness included in both; the difference is the bridge"}
    ot.destruct()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
