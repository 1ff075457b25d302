#!/usr/bin/env python3
"""Small launches where MPI halos live: one face type of the 256^3 double grid
over 16 fields (8 MiB packed; 1 field = 512 KiB), pack then unpack, through the engine and through
the face's bare kernel (ompi_amd/csrc/ddt_floor.hip), K launches each enqueued while the stream is
held by a sleep kernel, so the HIP events see device time only (no host enqueue).  Run under
`rocprofv3 --kernel-trace --stats` the same loop separates each kernel's own duration from the
launch and completion around it (the event time).  One JSON line per (face, fields, path)."""
from __future__ import annotations

import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import ompi_amd  # noqa: E402
from ompi_amd import recipe as ER  # noqa: E402
import bench  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    K = int(os.environ.get("K", "50"))
    fields_list = [int(x) for x in os.environ.get("FIELDS", "1,16").split(",")]
    field = 256 ** 3 * 8
    user = torch.empty(max(fields_list) * field, dtype=torch.uint8, device=dev)
    user.fill_(0x5A)
    stream = torch.cuda.current_stream(dev)
    L, Part = bench.floor_lib()
    recs = bench.face_recipes()
    # the event floor: the same event pair around one empty kernel
    tiny = torch.zeros(1, device=dev)
    evs = [tuple(torch.cuda.Event(enable_timing=True) for _ in range(2)) for _ in range(K)]
    torch.cuda._sleep(int(2e8))
    for a, b in evs:
        a.record(stream)
        tiny.add_(1)
        b.record(stream)
    torch.cuda.synchronize()
    print(json.dumps({"path": "empty torch kernel", "device_us": round(float(np.median(
        [a.elapsed_time(b) for a, b in evs])) * 1e3, 2)}), flush=True)
    for face in ("y", "z", "x"):
        for fields in fields_list:
            t = ER.build_committed(recs[face])
            S = t.info()["size"] * fields
            pk = torch.empty(S, dtype=torch.uint8, device=dev)
            c = ompi_amd.Convertor()
            c.set_stream(stream, True)
            kind, es, ls, ss, base, lw = bench.face_floor_part(face, fields)
            part = Part(kind, es, ls[0], ls[1], ls[2], lw, ss[0], ss[1], ss[2], base, 0)

            def engine(d):
                if d == 0:
                    c.prepare_for_send(t, fields, user.data_ptr())
                    c.pack([(pk, S)])
                else:
                    c.prepare_for_recv(t, fields, user.data_ptr())
                    c.unpack([(pk, S)])

            def bare(d):
                L.ddt_floor_launch(ctypes.c_void_p(user.data_ptr()), ctypes.c_void_p(pk.data_ptr()),
                                   ctypes.byref(part), d, ctypes.c_void_p(stream.cuda_stream))
            src = user[:S]

            def copy(d):
                # the same bytes as one contiguous device copy (the blit floor of a launch)
                if d == 0:
                    pk.copy_(src)
                else:
                    src.copy_(pk)
            for name, fn in (("engine", engine), ("bare", bare), ("contiguous copy", copy)):
                for _ in range(3):
                    fn(0)
                    fn(1)
                torch.cuda.synchronize()
                ev = [tuple(torch.cuda.Event(enable_timing=True) for _ in range(4)) for _ in range(K)]
                torch.cuda._sleep(int(4e8))
                for a, b, cc, d in ev:
                    a.record(stream)
                    fn(0)
                    b.record(stream)
                    cc.record(stream)
                    fn(1)
                    d.record(stream)
                torch.cuda.synchronize()
                tp = float(np.median([a.elapsed_time(b) for a, b, _, _ in ev])) * 1e3
                tu = float(np.median([cc.elapsed_time(d) for _, _, cc, d in ev])) * 1e3
                print(json.dumps({"face": face, "fields": fields, "path": name, "bytes": S,
                                  "pack_us": round(tp, 2), "unpack_us": round(tu, 2),
                                  "frac": round(4 * S / ((tp + tu) * 1e-6) / 8e12, 4)}), flush=True)
            del pk


if __name__ == "__main__":
    main()
