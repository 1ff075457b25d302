#!/usr/bin/env python3
"""Per-face pack/unpack time against the number of fields in one launch (round 2).

Each face type of the 256^3 double grid alone, count = F fields, pack then unpack, K steps
enqueued while the stream is held by a sleep kernel, so the HIP events see device time only
(no host enqueue cost).  A linear fit of time against F separates the per-field cost from
the fixed cost of a launch -- the bench's 16 fields sit where the fixed part matters."""
from __future__ import annotations

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
    recs = bench.face_recipes()
    field = 256 ** 3 * 8
    fields_list = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "1,4,16,64,256").split(",")]
    steps = 10
    user = torch.empty(max(fields_list) * field, dtype=torch.uint8, device=dev)
    user.fill_(0x5A)
    stream = torch.cuda.current_stream(dev)
    # floor: the same event pair around one tiny torch kernel
    tiny = torch.zeros(64, device=dev)
    evs = [tuple(torch.cuda.Event(enable_timing=True) for _ in range(2)) for _ in range(20)]
    torch.cuda._sleep(int(1e8))
    for a, b in evs:
        a.record(stream)
        tiny.add_(1.0)
        b.record(stream)
    torch.cuda.synchronize()
    print(json.dumps({"floor": "one tiny torch kernel between events",
                      "us": round(float(np.median([a.elapsed_time(b) for a, b in evs])) * 1e3, 2)}), flush=True)
    faces = sys.argv[2].split(",") if len(sys.argv) > 2 else ("x", "y", "z")
    # round 3: "read" = bench.face_throughput's cold-clean protocol (a 1 GiB read before each
    # operation, outside the events), so a pack does not pay the previous unpack's write-backs
    flush = sys.argv[3] if len(sys.argv) > 3 else "none"
    scribble = torch.full((1 << 27,), 3, dtype=torch.int64, device=dev) if flush == "read" else None
    print(json.dumps({"protocol": "pack+unpack loop" if scribble is None else
                      "cold-clean: 1 GiB read before every operation, outside the events"}), flush=True)
    for k in faces:
        ft = ER.build_committed(recs[k])
        rows = []
        for F in fields_list:
            fS = ft.info()["size"] * F
            fp = torch.empty(fS, dtype=torch.uint8, device=dev)
            c = ompi_amd.Convertor()
            c.set_stream(stream, True)
            for _ in range(2):
                c.prepare_for_send(ft, F, user.data_ptr())
                c.pack([(fp, fS)])
                c.prepare_for_recv(ft, F, user.data_ptr())
                c.unpack([(fp, fS)])
            torch.cuda.synchronize()
            evs = [tuple(torch.cuda.Event(enable_timing=True) for _ in range(3)) for _ in range(steps)]
            torch.cuda._sleep(int(2e8))   # hold the stream while the host enqueues
            ev2 = [torch.cuda.Event(enable_timing=True) for _ in range(steps)]
            for (a, b, e), b2 in zip(evs, ev2):
                if scribble is not None:
                    scribble.sum()
                a.record(stream)
                c.prepare_for_send(ft, F, user.data_ptr())
                c.pack([(fp, fS)])
                b.record(stream)
                if scribble is not None:
                    scribble.sum()
                b2.record(stream)
                c.prepare_for_recv(ft, F, user.data_ptr())
                c.unpack([(fp, fS)])
                e.record(stream)
            torch.cuda.synchronize()
            tp = float(np.median([a.elapsed_time(b) for a, b, _ in evs])) * 1e3
            tu = float(np.median([b2.elapsed_time(e) for (_, _, e), b2 in zip(evs, ev2)])) * 1e3
            rows.append((F, tp, tu))
            lines = ft.info()["size"] * F // 8 if k == "x" else None
            print(json.dumps({"face": k, "fields": F, "packed_MiB": fS / 2**20, "pack_us": round(tp, 2),
                              "unpack_us": round(tu, 2),
                              **({"pack_G_lines_per_s": round(lines / tp / 1e3, 1),
                                  "unpack_G_lines_per_s": round(lines / tu / 1e3, 1)} if lines else {}),
                              "frac": round(4 * fS / ((tp + tu) * 1e-6) / 8e12, 4)}), flush=True)
            del fp
        F = np.array([r[0] for r in rows], dtype=float)
        for j, name in ((1, "pack"), (2, "unpack")):
            y = np.array([r[j] for r in rows])
            slope, icpt = np.polyfit(F, y, 1)
            print(json.dumps({"face": k, "fit": name, "us_per_field": round(slope, 3),
                              "fixed_us": round(icpt, 2)}), flush=True)


if __name__ == "__main__":
    main()
