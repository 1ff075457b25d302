#!/usr/bin/env python3
"""End-to-end rate with a HOST-resident packed stream (SURVEY.md §8d "End-to-end"):
pack e2e = pack kernel + D2H into pinned host memory; unpack e2e = H2D from pinned host
+ unpack kernel.  Two schedules:
  serialized -- whole-message kernel into an HBM buffer, then one hipMemcpy (and reverse);
  overlapped -- the convertor's own host-iovec path: 16 MiB chunks double-buffered through
                two HBM staging slots on a copy stream (ddt_convertor.cpp, ensure_staging).
Also prints the plain pinned copy rates, the PCIe ceiling both schedules sit under."""
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

import ompi_amd  # noqa: E402
from ompi_amd import recipe as ER  # noqa: E402
import bench  # noqa: E402

GiB = float(1 << 30)


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return statistics.median(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--stage-mb", type=int, default=0, help="ddt_tune('stage_mb'): staging slot MiB")
    ap.add_argument("--tune", default="", help="extra ddt_tune settings, k=v;k=v")
    ap.add_argument("--hostdirect", type=int, default=-1,
                    help="ddt_tune('hostdirect'): 1 = kernel moves pinned host bytes itself, 0 = HBM staging")
    ap.add_argument("--pageable", action="store_true",
                    help="host packed stream in pageable memory (staged through HBM slots)")
    ap.add_argument("--variants", default="",
                    help="several runs in one process, '|'-separated tune strings (k=v;k=v), each "
                         "with fresh convertors (the staging slot size is read when a slot is made)")
    args = ap.parse_args()
    if not args.variants:
        run(args, args.tune)
        return
    for v in args.variants.split("|"):
        run(args, v)


def run(args, tune):
    dev = torch.device("cuda:0")
    if args.hostdirect >= 0:
        ompi_amd.lib().ddt_tune(b"hostdirect", args.hostdirect)
    if args.stage_mb:
        ompi_amd.lib().ddt_tune(b"stage_mb", args.stage_mb)
    for kv in filter(None, tune.split(";")):
        k, v = kv.split("=")
        ompi_amd.lib().ddt_tune(k.encode(), int(v))
    recipe, count, desc = bench.make_workload(args.config)
    dt = ER.build_committed(recipe)
    info = dt.info()
    S = info["size"] * count
    span, origin = bench.layout(info, count)
    user = torch.randint(1, 255, (span,), dtype=torch.uint8, device=dev)
    uptr = user.data_ptr() + origin
    dpk = torch.empty(S, dtype=torch.uint8, device=dev)
    hpk = torch.empty(S, dtype=torch.uint8, pin_memory=not args.pageable)
    st = torch.cuda.current_stream(dev)
    cp, cu = ompi_amd.Convertor(), ompi_amd.Convertor()
    for c in (cp, cu):
        c.set_stream(st, True)

    def pack_dev():
        cp.prepare_for_send(dt, count, uptr)
        cp.pack([(dpk, S)])

    def unpack_dev():
        cu.prepare_for_recv(dt, count, uptr)
        cu.unpack([(dpk, S)])

    def pack_ser():
        pack_dev()
        hpk.copy_(dpk, non_blocking=True)

    def unpack_ser():
        dpk.copy_(hpk, non_blocking=True)
        unpack_dev()

    def pack_ovl():
        cp.prepare_for_send(dt, count, uptr)
        cp.pack([(hpk.data_ptr(), S)])

    def unpack_ovl():
        cu.prepare_for_recv(dt, count, uptr)
        cu.unpack([(hpk.data_ptr(), S)])

    def gpu_time(fn, reps):
        """stream time of fn alone: a sleep kernel holds the stream while the host enqueues,
        so host-side call overhead is not counted (the wall-clock rows count it)"""
        fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda._sleep(2_000_000)
            e0.record(st)
            fn()
            e1.record(st)
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) / 1e3)
        return statistics.median(ts)

    def host_time(fn, reps):
        """host time of one call (the stream is held by a sleep kernel: nothing waits)"""
        fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(reps):
            torch.cuda._sleep(2_000_000)
            a = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - a)
            torch.cuda.synchronize()
        return statistics.median(ts)

    r = args.reps
    h = {k: host_time(f, r) for k, f in (("pack_device", pack_dev), ("pack_overlapped", pack_ovl),
                                         ("unpack_overlapped", unpack_ovl),
                                         ("d2h_copy", lambda: hpk.copy_(dpk, non_blocking=True)))}
    g = {k: gpu_time(f, r) for k, f in (("pack_overlapped", pack_ovl), ("unpack_overlapped", unpack_ovl),
                                        ("d2h_copy", lambda: hpk.copy_(dpk, non_blocking=True)),
                                        ("h2d_copy", lambda: dpk.copy_(hpk, non_blocking=True)))}
    t = {k: timed(f, r) for k, f in (("pack_kernel", pack_dev), ("unpack_kernel", unpack_dev),
                                     ("pack_serialized", pack_ser), ("unpack_serialized", unpack_ser),
                                     ("pack_overlapped", pack_ovl), ("unpack_overlapped", unpack_ovl),
                                     ("d2h_copy", lambda: hpk.copy_(dpk, non_blocking=True)),
                                     ("h2d_copy", lambda: dpk.copy_(hpk, non_blocking=True)))}
    # the overlapped path must produce the same stream as the device path
    pack_dev()
    ref = dpk.clone()
    pack_ovl()
    torch.cuda.synchronize()
    same = bool(torch.equal(ref.cpu(), hpk))
    # and the overlapped unpack must restore what the device path restores
    keep = user.clone()
    user.fill_(0xA5)
    unpack_ovl()
    torch.cuda.synchronize()
    got_o = user.clone()
    user.fill_(0xA5)
    dpk.copy_(hpk)
    unpack_dev()
    torch.cuda.synchronize()
    same_u = bool(torch.equal(got_o, user))
    user.copy_(keep)
    out = {"config": args.config, "workload": desc["workload"], "packed_bytes": S,
           "host_memory": "pageable" if args.pageable else "pinned",
           "hostdirect": int(args.hostdirect), "stage_mb": args.stage_mb, "tune": tune,
           "overlapped_matches_device_path": same, "overlapped_unpack_matches": same_u,
           "GiBs": {k: round(S / v / GiB, 2) for k, v in t.items()},
           "overlapped_vs_bare_copy": {"pack": round(t["d2h_copy"] / t["pack_overlapped"], 3),
                                       "unpack": round(t["h2d_copy"] / t["unpack_overlapped"], 3)},
           "us": {k: round(v * 1e6, 1) for k, v in t.items()},
           "stream_us": {k: round(v * 1e6, 1) for k, v in g.items()},
           "host_call_us": {k: round(v * 1e6, 1) for k, v in h.items()},
           "stream_overlapped_vs_bare_copy": {"pack": round(g["d2h_copy"] / g["pack_overlapped"], 3),
                                              "unpack": round(g["h2d_copy"] / g["unpack_overlapped"], 3)},
           "pack+unpack_GiBs": {
               "device_resident": round(2 * S / (t["pack_kernel"] + t["unpack_kernel"]) / GiB, 2),
               "serialized": round(2 * S / (t["pack_serialized"] + t["unpack_serialized"]) / GiB, 2),
               "overlapped": round(2 * S / (t["pack_overlapped"] + t["unpack_overlapped"]) / GiB, 2)}}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
