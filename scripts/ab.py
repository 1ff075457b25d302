#!/usr/bin/env python3
"""Interleaved A/B of engine tuning variants in ONE process (cdna guide §5.4 rule 24):
per variant and round, a fresh committed type, then pack and unpack timed separately
with HIP events.  Usage: python scripts/ab.py --config cfg2 --variants nt=-1,nt=0,nt=1"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import ompi_amd  # noqa: E402
from ompi_amd import recipe as ER  # noqa: E402
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--variants", default="nt=-1,nt=0,nt=1")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--mode", default="pair", choices=["pair", "pack", "unpack"],
                    help="pair = pack then unpack per step; pack/unpack = that direction only")
    ap.add_argument("--unpack-rev", action="store_true",
                    help="timing only: unpack with a type that writes the same bytes in reverse order "
                         "(fields, faces and rows reversed; xx and cfg2), to test Infinity Cache reuse")
    ap.add_argument("--prewarm", type=float, default=0.0, help="seconds of HBM copies first")
    ap.add_argument("--count", type=int, default=0, help="override the instance (field) count")
    ap.add_argument("--flush", default="none", choices=["read", "write", "none"],
                    help="touch a 1 GiB scribble before each operation, outside the events "
                         "(bench.face_throughput's protocol)")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    faces = bench.face_recipes()
    n, field = 256, 256 ** 3 * 8
    xf, yf = faces["x"][1], faces["y"][1]
    faces["xx"] = ("resized", ("struct", [1, 1], [0, (n - 1) * 8], [xf, xf]), 0, field)
    faces["yz"] = ("resized", ("struct", [1, 1, 1, 1], [0, (n - 1) * n * 8, 0, (n - 1) * n * n * 8],
                               [yf, yf, faces["z"][1], faces["z"][1]]), 0, field)
    n3, f3 = 512, 512 ** 3 * 4
    for i, (sub, st) in enumerate((([1, n3, n3], [n3 - 1, 0, 0]), ([n3, 1, n3], [0, n3 - 1, 0]),
                                   ([n3, n3, 1], [0, 0, n3 - 1]))):
        faces[f"c3d{i}"] = ("resized", ("subarray", [n3] * 3, sub, st, 0, ("basic", 15)), 0, f3)
    if args.config.startswith("c3d"):
        recipe, count = faces[args.config], 8
    elif args.config in faces:
        recipe, count = faces[args.config], 16
    else:
        recipe, count, _ = bench.make_workload(args.config)
    if args.count:
        count = args.count
    rev_recipe = None
    if args.unpack_rev:
        d8 = ("basic", 16)
        xr = ("hvector", n * n, 1, -n * 8, d8)                       # x face, rows last to first
        yr = ("hvector", n, n, -n * n * 8, d8)                       # y face, planes last to first
        zr = ("contig", n * n, d8)
        last_row = (n * n - 1) * n * 8
        if args.config == "xx":
            one = ("struct", [1, 1], [(n - 1) * 8 + last_row, last_row], [xr, xr])
        else:
            lp = (n - 1) * n * n * 8
            one = ("struct", [1] * 6,
                   [(n - 1) * n * n * 8, 0, (n - 1) * n * 8 + lp, lp, (n - 1) * 8 + last_row, last_row],
                   [zr, zr, yr, yr, xr, xr])
        rev_recipe = ("struct", [1], [15 * field], [("hvector", 16, 1, -field, one)])
    variants = [dict(kv.split("=") for kv in v.split(";")) for v in args.variants.split(",")]
    probe = ER.build_committed(recipe)
    info = probe.info()
    S = info["size"] * count
    span, origin = bench.layout(info, count)
    user = torch.randint(1, 255, (span,), dtype=torch.uint8, device=dev)
    packed = torch.empty(S, dtype=torch.uint8, device=dev)
    uptr = user.data_ptr() + origin
    L = ompi_amd.lib()
    if args.prewarm > 0:
        import time
        a = torch.empty(1 << 30, dtype=torch.uint8, device=dev)
        b = torch.empty_like(a)
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < args.prewarm:
            b.copy_(a)
            torch.cuda.synchronize()
        del a, b
    scribble = torch.full((1 << 27,), 3, dtype=torch.int64, device=dev) if args.flush != "none" else None

    def touch(i):
        if args.flush == "write":
            scribble.fill_(i)
        elif args.flush == "read":
            scribble.sum()

    res = {json.dumps(v): {"pack": [], "unpack": []} for v in variants}
    for _ in range(args.rounds):
        for v in variants:
            L.ddt_tune(b"reset", 0)
            for k, val in v.items():
                L.ddt_tune(k.encode(), int(val))
            dt = ER.build_committed(recipe)
            udt, ucount = (ER.build_committed(rev_recipe), 1) if rev_recipe else (dt, count)
            if rev_recipe:
                assert udt.info()["size"] == S
            cp, cu = ompi_amd.Convertor(), ompi_amd.Convertor()
            st = torch.cuda.current_stream(dev)
            cp.set_stream(st, True)
            cu.set_stream(st, True)
            evs = []
            for i in range(args.steps + 3):
                a, b, b2, c = (torch.cuda.Event(enable_timing=True) for _ in range(4))
                touch(2 * i)
                a.record()
                if args.mode != "unpack":
                    cp.prepare_for_send(dt, count, uptr)
                    cp.pack([(packed, S)])
                b.record()
                touch(2 * i + 1)
                b2.record()
                if args.mode != "pack":
                    cu.prepare_for_recv(udt, ucount, uptr)
                    cu.unpack([(packed, S)])
                c.record()
                if i >= 3:
                    evs.append((a, b, b2, c))
            torch.cuda.synchronize()
            r = res[json.dumps(v)]
            r["pack"].append(statistics.median(a.elapsed_time(b) for a, b, _, _ in evs) * 1e3)
            r["unpack"].append(statistics.median(b2.elapsed_time(c) for _, _, b2, c in evs) * 1e3)
    for k, r in res.items():
        p, u = statistics.median(r["pack"]), statistics.median(r["unpack"])
        print(json.dumps({"config": args.config, "flush": args.flush, "variant": json.loads(k), "pack_us": round(p, 1),
                          "unpack_us": round(u, 1), "step_us": round(p + u, 1),
                          "frac": round(4 * S / ((p + u) * 1e-6) / 8e12, 4),
                          "pack_rounds": [round(x, 1) for x in r["pack"]],
                          "unpack_rounds": [round(x, 1) for x in r["unpack"]]}), flush=True)


if __name__ == "__main__":
    main()
