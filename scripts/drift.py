"""Timeline of one config's pack / unpack event times in ONE process, to see whether a run
drifts (round 4: cfg4's pack ran ~615 us in an A/B's first rounds and ~570 us later, for every
variant alike).  Builds the type once (or every --rebuild seconds), then times pack + unpack
pairs back to back for --seconds, printing the median of each --window seconds as one JSON line.
Usage: python scripts/drift.py --config cfg4 --seconds 90 --window 5 [--rebuild 10]"""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import torch  # noqa: E402

import bench  # noqa: E402
import ompi_amd  # noqa: E402
from ompi_amd import recipe as ER  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg4")
    ap.add_argument("--seconds", type=float, default=90)
    ap.add_argument("--window", type=float, default=5)
    ap.add_argument("--rebuild", type=float, default=0, help="rebuild the type every N seconds (0: never)")
    ap.add_argument("--cycles", type=int, default=0,
                    help="instead: N cycles of (new type, new convertors, 13 timed pairs, destroy), as ab.py runs")
    ap.add_argument("--pad-gb", type=float, default=0, help="cycles: allocate this much HBM first (placement probe)")
    ap.add_argument("--pad-after", action="store_true", help="allocate the pad after the user buffer, before the type")
    ap.add_argument("--pad-chunks", type=int, default=1, help="the pad as this many separate allocations")
    ap.add_argument("--tune", default="", help="ddt_tune settings k=v;k=v before anything is built")
    args = ap.parse_args()
    for kv in filter(None, args.tune.split(";")):
        k, v = kv.split("=")
        ompi_amd.lib().ddt_tune(k.encode(), int(v))
    if args.cycles:
        return cycles(args)
    dev = torch.device("cuda:0")
    recipe, count, _ = bench.make_workload(args.config)
    dt = ER.build_committed(recipe)
    info = dt.info()
    S = info["size"] * count
    span, origin = bench.layout(info, count)
    user = torch.randint(1, 255, (span,), dtype=torch.uint8, device=dev)
    packed = torch.empty(S, dtype=torch.uint8, device=dev)
    uptr = user.data_ptr() + origin
    st = torch.cuda.current_stream(dev)
    cp, cu = ompi_amd.Convertor(), ompi_amd.Convertor()
    cp.set_stream(st, True)
    cu.set_stream(st, True)
    t0 = time.perf_counter()
    last_build = t0
    win0, pk, up = t0, [], []
    while time.perf_counter() - t0 < args.seconds:
        if args.rebuild and time.perf_counter() - last_build > args.rebuild:
            dt = ER.build_committed(recipe)
            last_build = time.perf_counter()
        evs = []
        for _ in range(8):
            a, b, c = (torch.cuda.Event(enable_timing=True) for _ in range(3))
            a.record()
            cp.prepare_for_send(dt, count, uptr)
            cp.pack([(packed, S)])
            b.record()
            cu.prepare_for_recv(dt, count, uptr)
            cu.unpack([(packed, S)])
            c.record()
            evs.append((a, b, c))
        torch.cuda.synchronize()
        pk += [a.elapsed_time(b) * 1e3 for a, b, _ in evs]
        up += [b.elapsed_time(c) * 1e3 for _, b, c in evs]
        now = time.perf_counter()
        if now - win0 >= args.window:
            print(json.dumps({"config": args.config, "t_s": round(now - t0, 1), "n": len(pk),
                              "pack_us": round(statistics.median(pk), 1),
                              "unpack_us": round(statistics.median(up), 1)}), flush=True)
            win0, pk, up = now, [], []


def cycles(args):
    import ctypes
    dev = torch.device("cuda:0")
    recipe, count, _ = bench.make_workload(args.config)
    probe = ER.build_committed(recipe)
    info = probe.info()
    S = info["size"] * count
    span, origin = bench.layout(info, count)
    del probe
    pad = None
    if args.pad_gb and not args.pad_after:
        pad = [torch.empty(int(args.pad_gb * (1 << 30)) // args.pad_chunks, dtype=torch.uint8, device=dev)
               for _ in range(args.pad_chunks)]
    user = torch.randint(1, 255, (span,), dtype=torch.uint8, device=dev)
    if args.pad_gb and args.pad_after:
        pad = torch.empty(int(args.pad_gb * (1 << 30)), dtype=torch.uint8, device=dev)
    packed = torch.empty(S, dtype=torch.uint8, device=dev)
    uptr = user.data_ptr() + origin
    st = torch.cuda.current_stream(dev)
    L = ompi_amd.lib()
    pool = (ctypes.c_int64 * 6)()
    for k in range(args.cycles):
        dt = ER.build_committed(recipe)
        cp, cu = ompi_amd.Convertor(), ompi_amd.Convertor()
        cp.set_stream(st, True)
        cu.set_stream(st, True)
        evs = []
        for i in range(13):
            a, b, c = (torch.cuda.Event(enable_timing=True) for _ in range(3))
            a.record()
            cp.prepare_for_send(dt, count, uptr)
            cp.pack([(packed, S)])
            b.record()
            cu.prepare_for_recv(dt, count, uptr)
            cu.unpack([(packed, S)])
            c.record()
            if i >= 3:
                evs.append((a, b, c))
        torch.cuda.synchronize()
        L.ddt_pool_info(pool)
        print(json.dumps({"config": args.config, "cycle": k, "tune": args.tune, "pad_gb": args.pad_gb, "pad_after": args.pad_after,
                          "pad_chunks": args.pad_chunks,
                          "pack_us": round(statistics.median(a.elapsed_time(b) for a, b, _ in evs) * 1e3, 1),
                          "unpack_us": round(statistics.median(b.elapsed_time(c) for _, b, c in evs) * 1e3, 1),
                          "pool": list(pool)}), flush=True)
        del cp, cu, dt


if __name__ == "__main__":
    main()
