#!/usr/bin/env python3
"""Kernel micro-benchmarks for tuning (not the driver's bench): per-type pack/unpack
device time, measured three ways: HIP-graph replay of the convertor calls, an eager
Python loop, and (under rocprofv3) per-dispatch kernel durations."""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import ompi_amd  # noqa: E402
from ompi_amd import recipe as ER  # noqa: E402
import bench  # noqa: E402

GiB = float(1 << 30)


def run_type(name, recipe, count, iters, dev, user=None):
    dt = ER.build_committed(recipe)
    info = dt.info()
    S = info["size"] * count
    span, origin = bench.layout(info, count)
    if user is None or user.numel() < span:
        user = torch.randint(1, 255, (span,), dtype=torch.uint8, device=dev)
    packed = torch.empty(S, dtype=torch.uint8, device=dev)
    uptr = user.data_ptr() + origin
    s = torch.cuda.Stream(dev)
    cp, cu = ompi_amd.Convertor(), ompi_amd.Convertor()

    def step():
        st = torch.cuda.current_stream(dev)
        cp.set_stream(st, True)
        cu.set_stream(st, True)
        cp.prepare_for_send(dt, count, uptr)
        cp.pack([(packed, S)])
        cu.prepare_for_recv(dt, count, uptr)
        cu.unpack([(packed, S)])

    with torch.cuda.stream(s):
        for _ in range(3):
            step()
    torch.cuda.synchronize()
    # eager
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(s):
        e0.record()
        for _ in range(iters):
            step()
        e1.record()
    torch.cuda.synchronize()
    eager = e0.elapsed_time(e1) / iters / 1e3
    # graph replay
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s, capture_error_mode="relaxed"):
        for _ in range(iters):
            step()
    with torch.cuda.stream(s):
        g.replay()
        torch.cuda.synchronize()
        e0.record(s)
        g.replay()
        e1.record(s)
    torch.cuda.synchronize()
    graph = e0.elapsed_time(e1) / iters / 1e3
    res = {"type": name, "S": S, "eager_us": round(eager * 1e6, 2), "graph_us": round(graph * 1e6, 2),
           "graph_GiBs": round(2 * S / graph / GiB, 1), "graph_frac": round(4 * S / graph / 8e12, 4),
           "plan": dt.plan_info()}
    return res, user


def copy_baseline(nbytes, iters, dev):
    a = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    b = torch.empty_like(a)
    b.copy_(a)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        b.copy_(a)
    e1.record()
    torch.cuda.synchronize()
    t = e0.elapsed_time(e1) / iters / 1e3
    return {"type": f"d2d_copy_{nbytes >> 20}MiB", "us": round(t * 1e6, 2),
            "GBs_rw": round(2 * nbytes / t / 1e9, 1)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--types", default="halo,x,y,z,cfg1,cfg5s,cfg4s,copy")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    todo = args.types.split(",")
    out = []
    user = None
    halo, _ = bench.halo_recipe()
    faces = bench.face_recipes()
    for t in todo:
        if t == "halo":
            r, user = run_type("halo", halo, 16, args.iters, dev, user)
        elif t in faces:
            r, user = run_type(t, faces[t], 16, args.iters, dev, user)
        elif t == "cfg1":
            r, _ = run_type("cfg1", ("vector", 1024, 1, 2, ("basic", 16)), 2048, args.iters, dev)
        elif t == "cfg5s":
            st = ("struct", [1, 3], [0, 8], [("basic", 16), ("basic", 6)])
            r, _ = run_type("cfg5_16Mi", ("hvector", 16 << 20, 1, 32, st), 1, args.iters, dev)
        elif t == "cfg4s":
            n = 8 << 20
            d = bench.lcg_disps(n)
            r, _ = run_type("cfg4_8Mi", ("indexed_block", 1, d, ("basic", 15)), 1, args.iters, dev)
        elif t == "copy":
            for nb in (48 << 20, 512 << 20):
                out.append(copy_baseline(nb, args.iters, dev))
            continue
        else:
            continue
        out.append(r)
        print(json.dumps(r), flush=True)
    for r in out:
        if r["type"].startswith("d2d"):
            print(json.dumps(r), flush=True)
    print(json.dumps({"task_kb": os.environ.get("DDT_TASK_KB", "32")}))


if __name__ == "__main__":
    main()
