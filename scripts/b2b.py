#!/usr/bin/env python3
"""bench.back_to_back alone: one JSON line per field count, K operations of
one face type between ONE event pair (eager with the stream held, host-paced, HIP graph)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402

if __name__ == "__main__":
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    K = int(os.environ.get("K", "200"))
    import ompi_amd
    # VARIANTS="k=v;k=v|k=v": one run per '|'-separated ddt_tune set (reset in between)
    for var in os.environ.get("VARIANTS", "").split("|"):
        ompi_amd.lib().ddt_tune(b"reset", 0)
        for kv in filter(None, var.split(";")):
            k, v = kv.split("=")
            ompi_amd.lib().ddt_tune(k.encode(), int(v))
        faces = tuple(os.environ.get("FACES", "xyz"))
        for f in [int(x) for x in os.environ.get("FIELDS", "16,1").split(",")]:
            r = bench.back_to_back(dev, f, K=K, faces=faces, with_copy=not var)
            r["variant"] = var
            print(json.dumps(r), flush=True)
