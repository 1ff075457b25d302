#!/usr/bin/env python3
"""SURVEY.md §8f row 2 measured: the device typed copy (opal_datatype_copy_content_same_ddt,
ddt_copy_content_same_ddt: ONE launch moving the type map from one user buffer to another)
against the pack + unpack pair through an HBM packed stream, on the BASELINE configs' own
types.  Algorithmic bytes: the typed copy reads and writes S once (2S); the pair moves 4S.
The typed copy is synchronous like the reference's (the data is in place when it returns), so
its wall time per call includes a stream synchronisation; `--only copy` under
`rocprofv3 --kernel-trace --stats` gives the kernel alone.  Not the driver's bench."""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
import ompi_amd  # noqa: E402
from ompi_amd import convertor as CV  # noqa: E402
from ompi_amd import recipe as ER  # noqa: E402

GiB = float(1 << 30)


def timed(fn, stream, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(stream)
    for _ in range(reps):
        fn()
    b.record(stream)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / 1e3 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="cfg1,cfg2,cfg3,cfg5")
    ap.add_argument("--only", default="", choices=["", "copy"], help="copy: typed copies only (for rocprofv3)")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream(dev)
    for name in args.configs.split(","):
        recipe, count, desc = bench.make_workload(name)
        dt = ER.build_committed(recipe)
        info = dt.info()
        S = info["size"] * count
        span, origin = bench.layout(info, count)
        src = torch.randint(1, 255, (span,), dtype=torch.uint8, device=dev)
        dst = torch.zeros(span, dtype=torch.uint8, device=dev)
        pk = torch.empty(S, dtype=torch.uint8, device=dev)
        cp, cu = ompi_amd.Convertor(), ompi_amd.Convertor()
        for c in (cp, cu):
            c.set_stream(st, True)

        def copy():
            CV.copy_content_same_ddt(dt, count, dst.data_ptr() + origin, src.data_ptr() + origin, st)

        def pair():
            cp.prepare_for_send(dt, count, src.data_ptr() + origin)
            cp.pack([(pk, S)])
            cu.prepare_for_recv(dt, count, dst.data_ptr() + origin)
            cu.unpack([(pk, S)])

        t_copy = timed(copy, st)
        if args.only == "copy":
            print(json.dumps({"config": name, "typed_copy_call_us": round(t_copy * 1e6, 1)}), flush=True)
            continue
        t_pair = timed(pair, st)
        # the copy must move exactly the type map: dst == what the pair produces
        dst.zero_()
        copy()
        ref = dst.clone()
        dst.zero_()
        pair()
        torch.cuda.synchronize()
        same = bool(torch.equal(ref, dst))
        print(json.dumps({"config": name, "workload": desc["workload"], "packed_bytes": S,
                          "typed_copy_call_us": round(t_copy * 1e6, 1), "pack_unpack_us": round(t_pair * 1e6, 1),
                          "typed_copy_call_GiBs": round(S / t_copy / GiB, 1),
                          "pair_GiBs": round(2 * S / t_pair / GiB, 1),
                          "copy_matches_pack_unpack": same}), flush=True)
        del src, dst, pk


if __name__ == "__main__":
    main()
