#!/usr/bin/env python3
"""Benchmark: device-resident MPI derived-datatype pack+unpack on MI355X.

Metric (BASELINE.json): "pack+unpack GiB/s/GPU (device-resident), 256^3 double
3D-vector; %HBM peak".  Default workload = BASELINE config 2: the 6-face halo of a
256^3 double grid (x faces vector(65536,1,256), y faces vector(256,256,65536), z faces
contiguous(65536)), the six faces of one field expressed as ONE committed struct type
resized to the field extent, F = 16 fields per GPU (count = 16, a 2 GiB working set,
well past the 256 MiB Infinity Cache).  One step = one pack (ddt_convertor_pack, whole
message, device iovec) + one unpack of the same message.

  value      = whole-job 2*S*N_gpus / (t_pack + t_unpack)        [GiB/s]
  roofline   = algorithmic bytes (read S + write S per op) / kernel time vs 8 TB/s
  request_roofline = memory-side requests per step (committed PMC pass, profiles/
               requests_<config>.json) / this run's kernel time vs the highest request
               rate measured for any access pattern
  cpu_baseline = the CPU oracle (oracle/ddt_oracle.c, a restatement of the reference
               convertor) on the host cores of the same box, bounded sample.

Other BASELINE configs: --config cfg1|cfg3|cfg4|cfg5 (cfg2 is the default).
Launch: python bench.py --gpus N --steps K --warmup W.  For N > 1 the driver starts one rank
per GPU with torch.distributed.run; run by hand without WORLD_SIZE, bench.py starts that
launcher itself as a child process (before anything touches the GPU) and exits with its code.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK = 8.0e12          # MI355X HBM3E spec (MI355X_MICROARCH.md)
GiB = float(1 << 30)


# ------------------------------------------------------------------ workloads
def halo_recipe(n=256, esize=8, tid=16):
    """6 faces of an n^3 grid in C order [z][y][x] as one struct, resized to the field."""
    field = n * n * n * esize
    xface = ("vector", n * n, 1, n, ("basic", tid))
    yface = ("vector", n, n, n * n, ("basic", tid))
    zface = ("contig", n * n, ("basic", tid))
    disps = [0, (n - 1) * esize, 0, (n - 1) * n * esize, 0, (n - 1) * n * n * esize]
    st = ("struct", [1] * 6, disps, [xface, xface, yface, yface, zface, zface])
    return ("resized", st, 0, field), field


def face_recipes(n=256, esize=8, tid=16):
    field = n * n * n * esize
    return {
        "x": ("resized", ("vector", n * n, 1, n, ("basic", tid)), 0, field),
        "y": ("resized", ("vector", n, n, n * n, ("basic", tid)), 0, field),
        "z": ("resized", ("contig", n * n, ("basic", tid)), 0, field),
    }


def cfg3_face_recipes(n=512):
    """BASELINE config 3's three faces of the 512^3 float grid (C order, start 511), each alone
    and resized to the field (ompi_datatype_create_subarray.c:32-112): dim0 = the last plane
    (1 MiB contiguous), dim1 = 512 rows of 2 KiB at a plane stride, dim2 = 4-byte elements at a
    2 KiB row stride."""
    field = n * n * n * 4
    f4 = ("basic", 15)
    return {
        "dim0": ("resized", ("subarray", [n] * 3, [1, n, n], [n - 1, 0, 0], 0, f4), 0, field),
        "dim1": ("resized", ("subarray", [n] * 3, [n, 1, n], [0, n - 1, 0], 0, f4), 0, field),
        "dim2": ("resized", ("subarray", [n] * 3, [n, n, 1], [0, 0, n - 1], 0, f4), 0, field),
    }


def lcg_disps(n):
    """cfg4 displacements: x_{i+1} = (1664525 x_i + 1013904223) mod 2^28, x_0 = 0x5EED."""
    out = np.empty(n, dtype=np.int64)
    x = 0x5EED
    # vectorised by jumping: compute in chunks with the closed form of the affine map
    a, c, m = 1664525, 1013904223, 1 << 28
    chunk = 1 << 16
    # powers for the first chunk
    first = np.empty(chunk, dtype=np.int64)
    for i in range(chunk):
        first[i] = x
        x = (a * x + c) % m
    out[:chunk] = first
    # A = a^chunk, C = c*(a^chunk - 1)/(a - 1) mod m  (per-step affine composition)
    A, C = 1, 0
    for _ in range(chunk):
        A, C = (A * a) % m, (C * a + c) % m
    prev = first
    for s in range(chunk, n, chunk):
        nxt = (A * prev + C) % m
        k = min(chunk, n - s)
        out[s:s + k] = nxt[:k]
        prev = nxt
    return out


def make_workload(name):
    """-> (recipe, count, description dict)"""
    if name == "cfg2":
        rec, field = halo_recipe()
        return rec, 16, {"workload": "256^3 double 6-face halo, struct of vector faces resized "
                                     "to the 128 MiB field, count = 16 fields per GPU",
                         "grid": [256, 256, 256], "dtype_elem": "double", "fields_per_gpu": 16,
                         "faces": 6}
    if name == "cfg1":
        return ("vector", 1024, 1, 2, ("basic", 16)), 2048, {
            "workload": "MPI_Type_vector(1024,1,2) double x 2048 (16 MiB packed)"}
    if name == "cfg3":
        n, e = 512, 4
        field = n * n * n * e
        faces = [("subarray", [n, n, n], [1, n, n], [n - 1, 0, 0], 0, ("basic", 15)),
                 ("subarray", [n, n, n], [n, 1, n], [0, n - 1, 0], 0, ("basic", 15)),
                 ("subarray", [n, n, n], [n, n, 1], [0, 0, n - 1], 0, ("basic", 15))]
        st = ("struct", [1, 1, 1], [0, 0, 0], faces)
        return ("resized", st, 0, field), 8, {
            "workload": "512^3 float subarray faces (dim0/dim1/dim2, start 511) as one struct, "
                        "count = 8 fields per GPU (64 fields over 8 GPUs)"}
    if name == "cfg4":
        n = 64 << 20
        d = lcg_disps(n)
        return ("indexed_block", 1, d, ("basic", 15)), 1, {
            "workload": "MPI_Type_indexed 64Mi unique LCG displacements into 1 GiB float"}
    if name == "cfg5":
        st = ("struct", [1, 3], [0, 8], [("basic", 16), ("basic", 6)])
        return ("hvector", 128 << 20, 1, 32, st), 1, {
            "workload": "hvector(128Mi,1,32B) of struct{double,int[3]} (2.5 GiB packed)"}
    raise SystemExit(f"unknown config {name}")


def layout(info, count, align=256):
    """(span, origin): a buffer of `span` bytes whose byte `origin` is the type origin (the
    array's base address; negative when the type touches nothing before true_lb).  The buffer
    holds only the touched bytes, starting up to align - 1 bytes early so that the type origin
    sits on an `align`-byte boundary, as an allocator places an array: without it cfg3's grid
    (first touched byte at 2044) would start 4-byte aligned and its planes and rows with it."""
    ext = info["ub"] - info["lb"]
    lo = min(info["true_lb"], info["true_lb"] + (count - 1) * ext)
    hi = max(info["true_ub"], info["true_ub"] + (count - 1) * ext)
    pad = lo % align
    return hi - lo + pad, pad - lo


# ------------------------------------------------------------------ CPU baseline
def sample_recipe(name, recipe, count):
    """A bounded piece of the workload whose packed stream is a PREFIX of the full one
    (same base pointer): about 10 s of oracle work, so the default run stays short."""
    if name == "cfg2":
        return recipe, 2, "2 of 16 fields"
    if name == "cfg3":
        return recipe, 1, f"1 of {count} fields"
    if name == "cfg4":
        n = 1 << 20
        return ("indexed_block", 1, recipe[2][:n], recipe[3]), 1, \
            f"the first {n} of {len(recipe[2])} displacements (same 1 GiB base)"
    if name == "cfg5":
        n = 1 << 20
        return ("hvector", n, recipe[2], recipe[3], recipe[4]), 1, \
            f"the first {n} of {recipe[1]} records"
    return recipe, count, "the whole message"


def tukey_stats(times):
    """to_self.c:674-776: sort, keep the samples inside Tukey's fence [q1 - 1.5 IQR,
    q3 + 1.5 IQR] (the middle half when fewer than MIN_GOOD_TIMERS = 5 survive); returns
    (best, median, mean) of the retained samples and how many were retained."""
    o = sorted(times)
    n = len(o)
    q1, q3 = o[n // 4], o[(3 * n) // 4]
    lo, hi = q1 - 1.5 * (q3 - q1), q3 + 1.5 * (q3 - q1)
    kept = [t for t in o if lo <= t <= hi]
    if len(kept) < 5:
        kept = o[n - (3 * n) // 4: n - n // 4]
    return kept[0], float(np.median(kept)), float(np.mean(kept)), len(kept)


def cpu_cores():
    """Cores this process may run on (its affinity set, the GPU box's CPU share) and the
    physical cores among them (distinct (package, core) pairs)."""
    cpus = sorted(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else list(range(os.cpu_count() or 1))
    phys = set()
    for c in cpus:
        try:
            base = f"/sys/devices/system/cpu/cpu{c}/topology/"
            phys.add((open(base + "physical_package_id").read().strip(), open(base + "core_id").read().strip()))
        except OSError:
            phys.add(("?", str(c)))
    return len(cpus), len(phys)


def cpu_baseline(name, srec, scount, what, host_user, origin, gpu_prefix, budget_s=12.0):
    """The reference convertor's algorithm restated in C (oracle/ddt_oracle.c) timed on the
    host cores of the same box, per SURVEY.md §8d: 1 thread and every physical core this
    process may use (position-sharded: each thread packs its byte range of the stream
    through its own cursor, the set_position sharding of opal_convertor.h:357-394), each a
    series of pack+unpack trials summarised like to_self.c:674-776 (Tukey-IQR fence; best,
    median and mean of the retained trials).  A bounded prefix of the same workload, on the
    GPU's own input bytes.

    The oracle is the checker here, never the measured product: it also re-packs the
    prefix and reports whether the GPU's packed bytes match."""
    from tests import recipes as R
    b = R.Built(srec)
    info = b.o.info()
    S = info["size"] * scount
    packed = np.zeros(S, dtype=np.uint8)
    logical, physical = cpu_cores()
    threads_all = max(1, min(physical, int(os.environ.get("OMP_NUM_THREADS", physical))))
    ptr = host_user.ctypes.data + origin
    b.o.run_mt(scount, ptr, packed.ctypes.data, threads_all, False)   # warm + reference bytes
    match = bool(np.array_equal(packed, gpu_prefix[:S]))
    scratch = host_user.copy()
    sptr = scratch.ctypes.data + origin
    series = {}
    for th in sorted({1, threads_all}):
        times, t0 = [], time.perf_counter()
        while (time.perf_counter() - t0 < budget_s / 2 and len(times) < 400) or len(times) < 8:
            a = time.perf_counter()
            b.o.run_mt(scount, sptr, packed.ctypes.data, th, False)
            b.o.run_mt(scount, sptr, packed.ctypes.data, th, True)
            times.append(time.perf_counter() - a)
        best, med, mean, kept = tukey_stats(times)
        series[th] = {"threads": th, "trials": len(times), "retained": kept,
                      "best_GiBs": round(2 * S / best / GiB, 3), "median_GiBs": round(2 * S / med / GiB, 3),
                      "mean_GiBs": round(2 * S / mean / GiB, 3)}
    top = series[threads_all]
    return {"value": top["median_GiBs"], "unit": "GiB/s", "cores": threads_all, "kind": "port",
            "gpu_matches_oracle": match,
            "one_thread": series[1], "all_cores": top,
            "host": {"cpus_available": logical, "physical_cores_available": physical,
                     "machine_cpus": os.cpu_count()},
            "sample": f"{what} of config {name}: pack+unpack of {S} packed bytes per trial, "
                      f"oracle/ddt_oracle.c position-sharded over {threads_all} threads ("
                      + ("every physical core of this process's CPU set" if threads_all == physical else
                         f"the CPU share OMP_NUM_THREADS grants this one-GPU process, of {physical} "
                         f"physical cores visible")
                      + f") and over 1 thread; value = median of the Tukey-retained trials at "
                      f"{threads_all} threads"}


# ------------------------------------------------------------------ latency
def single_face_latency(dev, stream, user, origin, reps=200):
    """one 512 KiB face of one field is launch-bound.  Reports, for
    packing ONE x face and ONE z face of field 0: `call_to_done_us`, HIP events around the
    call on an idle stream (host enqueue + launch + kernel); `device_us`, the same events with
    the stream held by a sleep kernel while the host enqueues (launch + kernel + one event
    record, scripts/face_scaling.py); and the synchronous MPI_Pack call time (host wall clock,
    plan cached)."""
    import torch
    import ompi_amd
    from ompi_amd import recipe as ER
    out = {}
    for name, rec in (("x", face_recipes()["x"]), ("z", face_recipes()["z"])):
        ft = ER.build_committed(rec)
        fs = ft.info()["size"]
        buf = torch.empty(fs, dtype=torch.uint8, device=dev)
        c = ompi_amd.Convertor()
        c.set_stream(stream, True)
        for _ in range(5):
            c.prepare_for_send(ft, 1, user.data_ptr() + origin)
            c.pack([(buf, fs)])
        torch.cuda.synchronize()
        evs = []
        for _ in range(reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)
            c.prepare_for_send(ft, 1, user.data_ptr() + origin)
            c.pack([(buf, fs)])
            b.record(stream)
            evs.append((a, b))
            torch.cuda.synchronize()
        k_us = float(np.median([a.elapsed_time(b) for a, b in evs])) * 1e3
        held = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                for _ in range(min(reps, 50))]
        torch.cuda._sleep(int(5e7))   # hold the stream while the host enqueues
        for a, b in held:
            a.record(stream)
            c.prepare_for_send(ft, 1, user.data_ptr() + origin)
            c.pack([(buf, fs)])
            b.record(stream)
        torch.cuda.synchronize()
        d_us = float(np.median([a.elapsed_time(b) for a, b in held])) * 1e3
        L = ompi_amd.lib()
        mpi = {}
        # synchronous MPI_Pack (data in place on return, pack.c.in:129-150): completed on the
        # signal kernel's pinned host word (default, r6), and on hipStreamSynchronize beside it
        for key, sig in (("mpi_pack_call_us", 1), ("mpi_pack_call_us_stream_sync", 0)):
            L.ddt_tune(b"sigsync", sig)
            walls = []
            for _ in range(reps):
                t0 = time.perf_counter()
                ompi_amd.pack(user.data_ptr() + origin, 1, ft, buf, fs, 0)
                walls.append(time.perf_counter() - t0)
            mpi[key] = round(float(np.median(walls)) * 1e6, 2)
        L.ddt_tune(b"sigsync", 1)
        out[name] = dict({"bytes": fs, "call_to_done_us": round(k_us, 2), "device_us": round(d_us, 2)}, **mpi)
    return out


# ------------------------------------------------------------------ back-to-back small launches
HBM_MEASURED = 6.29e12     # float4 copy on MI355X (MI355X_MICROARCH.md, chip-level table)
BOUNDARY_US = (1.45, 1.9)  # dependent kernel boundary, same stream (MI355X_MICROARCH.md "boundary")


def back_to_back(dev, fields, K=200, faces=("x", "y", "z"), with_copy=True):
    """Small-message throughput where halos live: K operations of ONE face type
    over `fields` fields between ONE event pair -- no event pair per operation.

      eager:  the K launches are enqueued while a sleep kernel holds the stream, so the events
              time the device running them back to back (each launch's boundary + kernel), not
              the host's enqueue rate;
      host:   the same K launches from an idle stream (events around the whole loop): what a
              host that enqueues one operation at a time sustains;
      graph:  the K operations captured once into a HIP graph and replayed.
    For every path: K packs, K unpacks, and K pack+unpack pairs (per operation = /2K).  Paths:
    the engine (Convertor.prepare + pack/unpack), the face's bare kernel (ddt_floor.hip) and,
    for the dense faces, a contiguous copy of the same bytes; an empty kernel prices the
    boundary under the same protocol.  `hbm_us` = the operation's 2S bytes at the measured
    6.29 TB/s; `model_us` = that + the guide's 1.45-1.9 us boundary."""
    import ctypes
    import torch
    import ompi_amd
    from ompi_amd import recipe as ER
    recs = face_recipes()
    field = 256 ** 3 * 8
    user = torch.empty(fields * field, dtype=torch.uint8, device=dev)
    user.fill_(0x5A)
    stream = torch.cuda.current_stream(dev)
    L, Part = floor_lib()
    tiny = torch.zeros(1, device=dev)

    def timed(fn, mode):
        """per-operation us of K calls of fn(i) (i = call index) under `mode`"""
        for i in range(4):
            fn(i)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        if mode == "graph":
            gs = torch.cuda.Stream(dev)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=gs, capture_error_mode="relaxed"):
                for i in range(K):
                    fn(i, torch.cuda.current_stream(dev))
            with torch.cuda.stream(gs):
                g.replay()
                torch.cuda.synchronize()
                a.record(gs)
                g.replay()
                b.record(gs)
            torch.cuda.synchronize()
            del g
        else:
            if mode == "eager":
                torch.cuda._sleep(int(3e8))   # hold the stream while the host enqueues the K calls
            a.record(stream)
            for i in range(K):
                fn(i)
            b.record(stream)
            torch.cuda.synchronize()
        return a.elapsed_time(b) * 1e3 / K

    out = {"fields": fields, "K": K}
    op = [0]

    def empty(i, s=None):
        tiny.add_(1)
    out["empty_kernel_us"] = {m: round(timed(empty, m), 3) for m in ("eager", "host", "graph")}
    for k in faces:
        # "h": the whole 6-face halo type (the bench's workload) at this field count, engine only
        ft = ER.build_committed(halo_recipe()[0] if k == "h" else recs[k])
        S = ft.info()["size"] * fields
        pk = torch.empty(S, dtype=torch.uint8, device=dev)
        cv = ompi_amd.Convertor()
        if k != "h":
            kind, es, ls, ss, base, lw = face_floor_part(k, fields)
            part = Part(kind, es, ls[0], ls[1], ls[2], lw, ss[0], ss[1], ss[2], base, 0)

        def engine(d):
            def f(i, s=None):
                dd = d if d < 2 else i & 1
                cv.set_stream(s or stream, True)
                if dd == 0:
                    cv.prepare_for_send(ft, fields, user.data_ptr())
                    cv.pack([(pk, S)])
                else:
                    cv.prepare_for_recv(ft, fields, user.data_ptr())
                    cv.unpack([(pk, S)])
            return f

        def bare(d):
            def f(i, s=None):
                dd = d if d < 2 else i & 1
                L.ddt_floor_launch(ctypes.c_void_p(user.data_ptr()), ctypes.c_void_p(pk.data_ptr()),
                                   ctypes.byref(part), dd, ctypes.c_void_p((s or stream).cuda_stream))
            return f
        src = user[:S]

        def copy(d):
            def f(i, s=None):
                dd = d if d < 2 else i & 1
                (pk.copy_(src) if dd == 0 else src.copy_(pk))
            return f
        paths = [("engine", engine)] + ([("bare", bare)] if k != "h" else []) \
            + ([("copy", copy)] if with_copy and k not in ("x", "h") else [])
        res = {"bytes": S, "hbm_us": round(2 * S / HBM_MEASURED * 1e6, 3)}
        res["model_us"] = [round(res["hbm_us"] + x, 3) for x in BOUNDARY_US]
        for name, mk in paths:
            r = {}
            for mode in ("eager", "host", "graph"):
                r[mode] = {"pack": round(timed(mk(0), mode), 3), "unpack": round(timed(mk(1), mode), 3),
                           "pair_per_op": round(timed(mk(2), mode), 3)}
            res[name] = r
        e = res["engine"]
        # the bench line's keys: per-operation us of alternating pack/unpack pairs
        res["back_to_back_us"] = e["eager"]["pair_per_op"]
        res["graph_us"] = e["graph"]["pair_per_op"]
        res["frac_back_to_back"] = round(2 * S / (e["eager"]["pair_per_op"] * 1e-6) / HBM_PEAK, 4)
        res["frac_graph"] = round(2 * S / (e["graph"]["pair_per_op"] * 1e-6) / HBM_PEAK, 4)
        out[k] = res
        cv.set_stream(stream, True)
        del pk, cv
    del user
    torch.cuda.empty_cache()
    return out


# ------------------------------------------------------------------ per-face throughput
def face_throughput(dev, fields, steps, warmup=2, faces=("x", "y", "z"), flush="read", grid="cfg2"):
    """The north star's per-face figure: ONE face type of the 256^3
    double grid over `fields` fields in one launch (count = fields), pack then unpack, each
    timed with HIP events (median over `steps`).  With 512 fields a face's working set
    (user lines + packed stream, 2 x 256 MiB) is twice the 256 MiB Infinity Cache; at the
    bench's 16 fields a face is 8 MiB and launch-bound.

    flush ("exceed the 256 MB Infinity Cache, or flush it between reps"): before
    every pack and between the pack and the unpack, outside the events, the stream touches a
    1 GiB scribble buffer (4x the Infinity Cache, 32x the L2s).
      "read"  (default): a reduction reads it, so each operation starts cold AND clean: none
               of its inputs cached, and the other operation's dirty lines already written back
               (during the flush, outside the events);
      "write": a fill writes it, so each operation starts cold but with up to 256 MiB of dirty
               scribble lines whose write-back it pays inside its own events;
      None:    no flush (the face's own 512 MiB working set, partly cache-resident).

    grid "cfg3": config 3's faces of the 512^3 float grid instead (faces dim0 / dim1 / dim2).
    Faces of single elements (x, dim2) also report the rate in 128-byte lines: each element is
    one whole-line request (profiles/r5_counter_calibration.json)."""
    import torch
    import ompi_amd
    from ompi_amd import recipe as ER
    recs = face_recipes() if grid == "cfg2" else cfg3_face_recipes()
    field = 256 ** 3 * 8 if grid == "cfg2" else 512 ** 3 * 4
    elem = 8 if grid == "cfg2" else 4
    user = torch.empty(fields * field, dtype=torch.uint8, device=dev)
    user.fill_(0x5A)
    scribble = torch.full((1 << 27,), 3, dtype=torch.int64, device=dev) if flush else None
    stream = torch.cuda.current_stream(dev)
    out = {"fields": fields, "flush": flush}

    def touch(i):
        if flush == "write":
            scribble.fill_(i)
        elif flush == "read":
            scribble.sum()
    # the launch floor under the same protocol: the events around one 1-element kernel (at 16
    # fields a y / z face moves 8 MiB in well under a microsecond of HBM time, so this is most of
    # its event time; profiles/r4_small_launch_trace.txt separates the kernel durations)
    tiny = torch.zeros(1, device=dev)
    tev = []
    for i in range(warmup + steps):
        a, b_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        if flush:
            touch(2 * i)
        a.record(stream)
        tiny.add_(1)
        b_.record(stream)
        if i >= warmup:
            tev.append((a, b_))
    torch.cuda.synchronize()
    out["launch_floor_us"] = round(float(np.median([a.elapsed_time(b_) for a, b_ in tev])) * 1e3, 2)
    for k in faces:
        ft = ER.build_committed(recs[k])
        fS = ft.info()["size"] * fields
        fp = torch.empty(fS, dtype=torch.uint8, device=dev)
        c1 = ompi_amd.Convertor()
        c1.set_stream(stream, True)
        evs = []
        for i in range(warmup + steps):
            a, b_, c_, d_ = (torch.cuda.Event(enable_timing=True) for _ in range(4))
            if flush:
                touch(2 * i)
            a.record(stream)
            c1.prepare_for_send(ft, fields, user.data_ptr())
            c1.pack([(fp, fS)])
            b_.record(stream)
            if flush:
                touch(2 * i + 1)
            c_.record(stream)
            c1.prepare_for_recv(ft, fields, user.data_ptr())
            c1.unpack([(fp, fS)])
            d_.record(stream)
            if i >= warmup:
                evs.append((a, b_, c_, d_))
        torch.cuda.synchronize()
        tp = float(np.median([a.elapsed_time(b_) for a, b_, _, _ in evs])) / 1e3
        tu = float(np.median([c_.elapsed_time(d_) for _, _, c_, d_ in evs])) / 1e3
        out[k] = {"packed_bytes": fS, "pack_us": round(tp * 1e6, 2), "unpack_us": round(tu * 1e6, 2),
                  "GiBs": round(2 * fS / (tp + tu) / GiB, 1), "frac": round(4 * fS / (tp + tu) / HBM_PEAK, 4),
                  "pack_frac": round(2 * fS / tp / HBM_PEAK, 4), "unpack_frac": round(2 * fS / tu / HBM_PEAK, 4)}
        if k in ("x", "dim2"):
            # one element per 128-byte line: the memory moves whole lines (the pack reads them,
            # the unpack's partial writes complete as whole lines below the L2)
            lines = fS // elem
            out[k]["line_bytes"] = lines * 128
            out[k]["pack_line_GBs"] = round(lines * 128 / tp / 1e9, 1)
            out[k]["pack_line_frac"] = round(lines * 128 / tp / HBM_PEAK, 4)
            out[k]["unpack_line_GBs"] = round((lines * 128 + fS) / tu / 1e9, 1)
        # the same protocol around the face's bare kernel (ompi_amd/csrc/ddt_floor.hip): same
        # buffers, events, flushes; frac_of_floor = floor / engine (1.0 = the engine at the floor)
        try:
            import ctypes
            L, Part = floor_lib()
            kind, es, ls, ss, base, lw = face_floor_part(k, fields, grid=grid)
            part = Part(kind, es, ls[0], ls[1], ls[2], lw, ss[0], ss[1], ss[2], base, 0)
            fev = []
            for i in range(warmup + steps):
                a, b_, c_, d_ = (torch.cuda.Event(enable_timing=True) for _ in range(4))
                if flush:
                    touch(2 * i)
                a.record(stream)
                L.ddt_floor_launch(ctypes.c_void_p(user.data_ptr()), ctypes.c_void_p(fp.data_ptr()),
                                   ctypes.byref(part), 0, ctypes.c_void_p(stream.cuda_stream))
                b_.record(stream)
                if flush:
                    touch(2 * i + 1)
                c_.record(stream)
                L.ddt_floor_launch(ctypes.c_void_p(user.data_ptr()), ctypes.c_void_p(fp.data_ptr()),
                                   ctypes.byref(part), 1, ctypes.c_void_p(stream.cuda_stream))
                d_.record(stream)
                if i >= warmup:
                    fev.append((a, b_, c_, d_))
            torch.cuda.synchronize()
            fpk = float(np.median([a.elapsed_time(b_) for a, b_, _, _ in fev])) * 1e3
            fup = float(np.median([c_.elapsed_time(d_) for _, _, c_, d_ in fev])) * 1e3
            out[k].update({"floor_pack_us": round(fpk, 2), "floor_unpack_us": round(fup, 2),
                           "frac_of_floor": round((fpk + fup) / ((tp + tu) * 1e6), 4)})
        except (OSError, AssertionError) as ex:
            out[k]["floor_error"] = f"{type(ex).__name__}: {ex}"[:160]
        del fp
    del user, scribble
    torch.cuda.empty_cache()
    return out


# ------------------------------------------------------------------ floor (bare kernels)
def floor_parts(name):
    """The workload as the access primitives of ompi_amd/csrc/ddt_floor.hip -- element gathers
    (one 4/8-byte element per position), element scatters, block copies -- with the same user
    offsets the engine moves: [(label, kind, esize, (l0, l1, l2), (s0, s1, s2), base, lw)].
    Position counts are powers of two (decomposed by shifts).  None where the workload is not
    made of these primitives (cfg4: address-ordered index list; cfg5: line-dense records)."""
    if name == "cfg2":
        n, F, e = 256, 16, 8
        field, row, plane = n * n * n * e, n * e, n * n * e
        return [("x faces", 0, 8, (16, 1, 4), (row, row - e, field), 0, 0),
                ("y faces", 1, 0, (8, 1, 4), (plane, (n - 1) * row, field), 0, 7),
                ("z faces", 1, 0, (1, 4, 0), ((n - 1) * plane, field, 0), 0, 15)]
    if name == "cfg3":
        n, F, e = 512, 8, 4
        field, row, plane = n * n * n * e, n * e, n * n * e
        return [("dim0 planes", 1, 0, (3, 0, 0), (field, 0, 0), (n - 1) * plane, 16),
                ("dim1 rows", 1, 0, (9, 3, 0), (plane, field, 0), (n - 1) * row, 7),
                ("dim2 elements", 0, 4, (18, 3, 0), (row, field, 0), (n - 1) * e, 0)]
    if name == "cfg1":
        return [("elements", 0, 8, (10, 11, 0), (16, 16376, 0), 0, 0)]
    if name == "cfg5":
        # 128 Mi records of 20 bytes at a 32-byte pitch: the r3 bare LDS kernels (pack: whole-line
        # span loads; unpack: plain dwordx4 + dword record stores)
        return [("records", 2, 20, (27, 0, 0), (32, 0, 0), 0, 0)]
    if name == "cfg4":
        # the address-ordered design's passes: (1) every touched line read once in
        # address order into a compact stream / the masked scatter of every element in address
        # order, with a 4-byte index per element; (2) the permutation pass between that stream
        # and the packed order, priced as a contiguous copy of its bytes between two scratch
        # buffers (no user or packed bytes; the engine permutes through LDS)
        n = 64 << 20
        return [("address-ordered elements", 3, 4, (0, 0, 0), (0, 0, 0), 0, 0, {"count": n, "list": True}),
                ("permutation stream", 1, 0, (14, 0, 0), (16384, 0, 0), 0, 10, {"scratch": 4 * n})]
    return None


_FLOOR = None


def floor_lib():
    """ompi_amd/libddt_floor.so (bare kernels, measurement only) and its part structure."""
    global _FLOOR
    if _FLOOR is None:
        import ctypes

        class Part(ctypes.Structure):
            _fields_ = [("kind", ctypes.c_int32), ("esize", ctypes.c_int32), ("l0", ctypes.c_uint32),
                        ("l1", ctypes.c_uint32), ("l2", ctypes.c_uint32), ("lw", ctypes.c_uint32),
                        ("s0", ctypes.c_int64), ("s1", ctypes.c_int64), ("s2", ctypes.c_int64),
                        ("base", ctypes.c_int64), ("poff", ctypes.c_int64), ("list", ctypes.c_uint64),
                        ("count", ctypes.c_uint64), ("ubuf", ctypes.c_uint64), ("pbuf", ctypes.c_uint64)]
        L = ctypes.CDLL(os.path.join(ROOT, "ompi_amd", "libddt_floor.so"))
        L.ddt_floor_run.restype = ctypes.c_int
        L.ddt_floor_run.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                    ctypes.c_int, ctypes.c_void_p]
        L.ddt_floor_launch.restype = ctypes.c_int
        L.ddt_floor_launch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                       ctypes.c_void_p]
        _FLOOR = (L, Part)
    return _FLOOR


def face_floor_part(face, fields, n=256, e=8, grid="cfg2"):
    """One face type over `fields` fields (a power of two) as a floor part.  cfg2 (256^3
    double): x = element gather/scatter, y = 2 KiB rows, z = 512 KiB planes; cfg3 (512^3 float,
    start 511): dim0 = the 1 MiB last plane, dim1 = 2 KiB rows at a plane stride, dim2 = 4-byte
    elements at a 2 KiB row stride (floor_parts("cfg3") per face)."""
    lf = fields.bit_length() - 1
    assert 1 << lf == fields
    if grid == "cfg3":
        n, e = 512, 4
        field, row, plane = n * n * n * e, n * e, n * n * e
        return {"dim0": (1, 0, (lf, 0, 0), (field, 0, 0), (n - 1) * plane, 16),
                "dim1": (1, 0, (9, lf, 0), (plane, field, 0), (n - 1) * row, 7),
                "dim2": (0, 4, (18, lf, 0), (row, field, 0), (n - 1) * e, 0)}[face]
    field, row, plane = n * n * n * e, n * e, n * n * e
    return {"x": (0, 8, (16, lf, 0), (row, field, 0), 0, 0),
            "y": (1, 0, (8, lf, 0), (plane, field, 0), 0, 7),
            "z": (1, 0, (lf, 0, 0), (field, 0, 0), 0, 15)}[face]


def floor_run(name, user_ptr, packed_ptr, reps=10, recipe=None, dev=None):
    """Each part of the workload by its bare kernel, pack then unpack, in the same run and on
    the same buffers as the engine; returns per-part medians (us) or None.  Parts with extras:
    "list" = the workload's element indices in ascending order uploaded for the part (config 4:
    from `recipe`'s displacements), "scratch" = a pass between two scratch buffers of that many
    bytes (not counted in the packed bytes the parts cover)."""
    import ctypes
    parts = floor_parts(name)
    if parts is None:
        return None
    L, Part = floor_lib()
    arr = (Part * len(parts))()
    poff = 0
    keep = []
    for i, (_, kind, es, ls, ss, base, lw, *ex) in enumerate(parts):
        ex = ex[0] if ex else {}
        arr[i] = Part(kind, es, ls[0], ls[1], ls[2], lw, ss[0], ss[1], ss[2], base, poff)
        if ex.get("list"):
            import torch
            idx = np.sort(np.asarray(recipe[2], dtype=np.int64))
            assert len(idx) == ex["count"] and idx[0] >= 0 and idx[-1] < (1 << 32)
            t = torch.from_numpy(idx.astype(np.uint32).view(np.int32)).to(dev)
            keep.append(t)
            arr[i].list, arr[i].count = t.data_ptr(), ex["count"]
        if ex.get("scratch"):
            import torch
            bufs = [torch.empty(ex["scratch"], dtype=torch.uint8, device=dev) for _ in range(2)]
            keep += bufs
            arr[i].ubuf, arr[i].pbuf, arr[i].poff = bufs[0].data_ptr(), bufs[1].data_ptr(), 0
            continue
        npos = ex["count"] if "count" in ex else 1 << sum(ls)
        poff += npos * (es if kind in (0, 2, 3) else 16 << lw)
    out = (ctypes.c_float * (2 * len(parts)))()
    rc = L.ddt_floor_run(ctypes.c_void_p(user_ptr), ctypes.c_void_p(packed_ptr), arr, len(parts), reps, out)
    del keep
    if rc != 0:
        return {"error": f"hip error {rc}"}
    res = {label: {"pack_us": round(out[2 * i], 2), "unpack_us": round(out[2 * i + 1], 2)}
           for i, (label, *_r) in enumerate(parts)}
    return {"parts": res, "bytes": poff,
            "pack_us": round(sum(v["pack_us"] for v in res.values()), 2),
            "unpack_us": round(sum(v["unpack_us"] for v in res.values()), 2)}


def touched_lines(dt, count, max_iov=8 << 20):
    """128-byte lines of user memory the type map of `count` instances touches (the engine's raw
    iovec export, opal_convertor_raw semantics, on a NULL base: offsets only), or None beyond
    `max_iov` iovecs.  The memory side moves whole lines (r5 calibration: one 128-B read request
    per touched line for every access pattern the engine has)."""
    import ctypes
    import ompi_amd
    from ompi_amd._lib import IOVec, lib
    conv = ompi_amd.Convertor().prepare_for_raw(dt, count, 0)
    chunk = 1 << 20
    arr = (IOVec * chunk)()
    firsts, lasts, total = [], [], 0
    while True:
        n = ctypes.c_uint32(chunk)
        ln = ctypes.c_size_t(0)
        rc = lib().ddt_convertor_raw(conv.h, arr, ctypes.byref(n), ctypes.byref(ln))
        if rc < 0:
            return None
        v = np.frombuffer(arr, dtype=np.int64, count=2 * n.value).reshape(-1, 2)
        v = v[v[:, 1] > 0]
        firsts.append(v[:, 0] >> 7)
        lasts.append((v[:, 0] + v[:, 1] - 1) >> 7)
        total += n.value
        if rc == 1 or n.value == 0:
            break
        if total > max_iov:
            return None
    f, l_ = np.concatenate(firsts), np.concatenate(lasts)
    o = np.argsort(f, kind="stable")
    f, l_ = f[o], l_[o]
    # union of the [first, last] line ranges
    reach = np.maximum.accumulate(l_)
    new = np.ones(len(f), dtype=bool)
    new[1:] = f[1:] > reach[:-1]
    starts = f[new]
    ends = np.maximum.reduceat(l_, np.flatnonzero(new))
    return int((ends - starts + 1).sum())


def copy_ceiling(dev, nbytes=1 << 30, reps=10):
    """"also report against a measured contiguous D2D copy ceiling".  One
    contiguous GiB copied each way by the floor library's block-copy kernel (16 KiB per
    workgroup, non-temporal loads), 4x the Infinity Cache so HBM serves it; GB/s counts the
    read and the write (2 x nbytes per copy), as the roofline's algorithmic bytes do."""
    import ctypes
    import torch
    L, Part = floor_lib()
    a = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    b = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    a.fill_(1)
    b.fill_(2)
    blocks = nbytes >> 14
    l0 = blocks.bit_length() - 1
    assert 1 << l0 == blocks
    part = (Part * 1)(Part(1, 0, l0, 0, 0, 10, 16384, 0, 0, 0, 0))
    out = (ctypes.c_float * 2)()
    rc = L.ddt_floor_run(ctypes.c_void_p(a.data_ptr()), ctypes.c_void_p(b.data_ptr()), part, 1, reps, out)
    del a, b
    torch.cuda.empty_cache()
    if rc != 0:
        return {"error": f"hip error {rc}"}
    gbs = [2 * nbytes / (out[i] * 1e-6) / 1e9 for i in range(2)]
    return {"bytes": nbytes, "copy_us": [round(out[0], 2), round(out[1], 2)],
            "GB_per_s": round(sum(gbs) / 2, 1),
            "source": "ompi_amd/csrc/ddt_floor.hip copy_blocks, 1 GiB each way, median of 10"}


# ------------------------------------------------------------------ end to end (host packed stream)
def end_to_end(dev, config, pageable=False, reps=10, tune="", hostdirect=-1, stage_mb=0):
    """End-to-end rate with a HOST-resident packed stream (SURVEY.md §8d "End-to-end"; the north
    star's "copies to and from the GPU"): pack e2e = pack kernel + D2H into host memory, unpack
    e2e = H2D from host memory + unpack kernel, the user buffer device-resident.  Schedules:
      serialized -- whole-message kernel into an HBM buffer, then one copy (and reverse);
      overlapped -- the convertor's own host-iovec path (pinned: the kernel moves the host bytes
                    itself over PCIe; pageable: chunks double-buffered through HBM staging).
    Beside them the bare pinned copies (the PCIe ceiling).  Wall-clock medians of `reps` calls;
    `stream_us` = the stream time alone, `host_call_us` = the host time of one call.  Outside the
    bench's timed region; never `value`."""
    import statistics
    import torch
    import ompi_amd
    from ompi_amd import recipe as ER
    if hostdirect >= 0:
        ompi_amd.lib().ddt_tune(b"hostdirect", hostdirect)
    if stage_mb:
        ompi_amd.lib().ddt_tune(b"stage_mb", stage_mb)
    for kv in filter(None, tune.split(";")):
        k, v = kv.split("=")
        ompi_amd.lib().ddt_tune(k.encode(), int(v))
    recipe, count, desc = make_workload(config)
    dt = ER.build_committed(recipe)
    info = dt.info()
    S = info["size"] * count
    span, origin = layout(info, count)
    user = torch.randint(1, 255, (span,), dtype=torch.uint8, device=dev)
    uptr = user.data_ptr() + origin
    dpk = torch.empty(S, dtype=torch.uint8, device=dev)
    hpk = torch.empty(S, dtype=torch.uint8, pin_memory=not pageable)
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

    r = reps

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
    out = {"config": config, "workload": desc["workload"], "packed_bytes": S,
           "host_memory": "pageable" if pageable else "pinned",
           "hostdirect": int(hostdirect), "stage_mb": stage_mb, "tune": tune,
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
    del user, dpk, hpk
    torch.cuda.empty_cache()
    return out




# ------------------------------------------------------------------ multi-rank harness
def self_launch_argv(gpus, argv, port):
    """The launcher command for `--gpus N` run by hand: one rank per GPU on this node, the
    same command line, rendezvous on 127.0.0.1 (torch.distributed.run sets RANK, LOCAL_RANK,
    WORLD_SIZE and MASTER_*; every rank binds cuda:LOCAL_RANK)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def timed_region(step, steps, world, sync, reduce_max, barrier):
    """Time exactly `steps` calls of step(i) between a barrier + device synchronize on both
    sides; returns the wall time, max over ranks (the driver contract)."""
    if world > 1:
        barrier()
    sync()
    t0 = time.perf_counter()
    for i in range(steps):
        step(i)
    sync()
    wall = time.perf_counter() - t0
    if world > 1:
        wall = reduce_max(wall)
        barrier()
    return wall


def gather_check(packed, S, world, rank, dev, backend):
    """The RCCL leg of SURVEY.md §8e, outside the timed region: the packed shards are
    all-gathered (backend "nccl" = RCCL over xGMI) and every rank checks that its slice of the
    gathered stream is its own shard."""
    import torch
    import torch.distributed as dist
    from ompi_amd import shard
    side = dev if backend == "nccl" else "cpu"
    g0 = time.perf_counter()
    full = shard.gather_packed(packed if backend == "nccl" else packed.cpu())
    if backend == "nccl":
        torch.cuda.synchronize()
    g_s = time.perf_counter() - g0
    sizes = [torch.zeros(1, dtype=torch.int64, device=side) for _ in range(world)]
    dist.all_gather(sizes, torch.tensor([S], dtype=torch.int64, device=side))
    off = sum(int(x.item()) for x in sizes[:rank])
    ok = torch.tensor([1 if torch.equal(full[off:off + S].to(packed.device), packed) else 0],
                      dtype=torch.int64, device=side)
    dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    return {"backend": backend, "gathered_bytes": int(full.numel()), "ok": bool(ok.item()),
            "seconds": round(g_s, 4)}


def per_rank_times(tp, tu, world, dev, backend):
    """All ranks' pack / unpack event times (seconds in, ms out), all-gathered after the timed
    region: min / max over ranks and the per-rank list in rank order."""
    import torch
    import torch.distributed as dist
    mine = torch.tensor([tp * 1e3, tu * 1e3], dtype=torch.float64,
                        device=dev if backend == "nccl" else "cpu")
    allk = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(allk, mine)
    rk = [[round(float(x[0]), 4), round(float(x[1]), 4)] for x in allk]
    return {"pack": {"min": min(r[0] for r in rk), "max": max(r[0] for r in rk)},
            "unpack": {"min": min(r[1] for r in rk), "max": max(r[1] for r in rk)},
            "ranks": rk,
            "source": "each rank's HIP events on every Nth timed step, all-gathered after the timed "
                      "region; [pack_ms, unpack_ms] per rank in rank order"}


# ------------------------------------------------------------------ main
def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # ~35 ms timed at the default config: long enough that one rank's launch jitter does not
    # set the max-over-ranks time of a multi-GPU run
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-faces", action="store_true", help="skip the per-face measurement")
    ap.add_argument("--no-gather", action="store_true",
                    help="skip the post-run all-gather of the packed shards (N > 1)")
    ap.add_argument("--strong", action="store_true",
                    help="strong scaling: ONE message of the config's total size split over the ranks "
                         "(top-level count, outer loop or index prefix: ompi_amd.shard.split_recipe); "
                         "cfg3 = 64 fields in total")
    ap.add_argument("--face-fields", type=int, default=512,
                    help="fields per face launch for the per-face figure (512: beyond the Infinity Cache)")
    ap.add_argument("--no-graph", action="store_true", help="skip the HIP-graph replay measurement")
    ap.add_argument("--event-every", type=int, default=10,
                    help="bracket every Nth timed step with HIP events (kernel durations)")
    ap.add_argument("--no-floor", action="store_true", help="skip the bare-kernel floor of the workload")
    ap.add_argument("--no-latency", action="store_true",
                    help="skip the single-face latency probe (profiling runs: one workload per trace)")
    ap.add_argument("--e2e", action="store_true",
                    help="after the line's measurements: end-to-end rates with a host-resident packed "
                         "stream (cfg1, cfg2, cfg5; pinned and pageable), outside the timed region")
    ap.add_argument("--no-cold", action="store_true", help="skip the cold-unpack step (cold_step)")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # run by hand: start one rank per GPU as child processes, before any HIP call here
        import subprocess
        rc = subprocess.call(self_launch_argv(args.gpus, sys.argv[1:], free_port()))
        sys.exit(rc)

    # stdout carries exactly ONE line, the JSON result of rank 0: everything else the process (or
    # a library below it: gloo reports its peer connections on stdout) writes to fd 1 goes to
    # stderr, and the result is written to the saved descriptor at the end
    sys.stdout.flush()
    result_fd = os.dup(1)
    os.dup2(2, 1)

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # backend "nccl" is RCCL on ROCm; DDT_BENCH_BACKEND=gloo rehearses the multi-rank path
    # with several ranks sharing one GPU (code-path check only, not a scaling number)
    if args.gpus != world:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; launch N > 1 with "
              "python -m torch.distributed.run --nproc-per-node N (reporting n_gpus = WORLD_SIZE)",
              file=sys.stderr)
    backend = os.environ.get("DDT_BENCH_BACKEND", "nccl" if torch.cuda.is_available() else "gloo")
    local = local % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    # DDT_BENCH_PG=1 builds the process group (and runs the post-run RCCL gather) at world size 1
    # too: a single-rank RCCL communicator on the one GPU executes the code the driver's 8-GPU
    # run reaches (tests/test_gpu_rccl.py)
    use_pg = world > 1 or os.environ.get("DDT_BENCH_PG") == "1"
    if use_pg:
        # bind the RCCL communicator to this rank's GPU up front (no device guess in barrier())
        dist.init_process_group(backend=backend, **({"device_id": dev} if backend == "nccl" else {}))

    import ompi_amd
    from ompi_amd import recipe as ER

    recipe, count, desc = make_workload(args.config)
    split = None
    if args.strong:
        # one message of the configuration's total size; each rank commits and moves its
        # own part, resident in its own HBM, with no data-path collective
        from ompi_amd import shard
        if args.config == "cfg3":
            count = 64
            desc = dict(desc, workload="512^3 float subarray faces (dim0/dim1/dim2, start 511) as one "
                                       "struct, 64 fields in total split by top-level count")
        sp = shard.split_recipe(recipe, count, rank, world)
        if sp is None:
            raise SystemExit(f"no strong split for {args.config}")
        split = {"total_count": count, "method": ("top-level count" if count > 1 else
                                                  ("outer loop" if recipe[0] in ("vector", "hvector")
                                                   else "index prefix"))}
        recipe, count = sp[0], sp[1]
    dt = ER.build_committed(recipe)
    info = dt.info()
    S = info["size"] * count
    span, origin = layout(info, count)
    S_total = S * world
    if split and world > 1:
        t_s = torch.tensor([S], device=dev if backend == "nccl" else "cpu", dtype=torch.int64)
        dist.all_reduce(t_s)
        S_total = int(t_s.item())

    user = torch.empty(span, dtype=torch.uint8, device=dev)
    user.copy_(torch.randint(1, 255, (span,), dtype=torch.uint8, device=dev))
    packed = torch.empty(S, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)

    cp = ompi_amd.Convertor()
    cu = ompi_amd.Convertor()
    for c in (cp, cu):
        c.set_stream(stream, True)
    uptr = user.data_ptr() + origin

    def pack():
        cp.prepare_for_send(dt, count, uptr)
        rc, _, md = cp.pack([(packed, S)])
        assert rc == 1 and md == S

    def unpack():
        cu.prepare_for_recv(dt, count, uptr)
        rc, _, md = cu.unpack([(packed, S)])
        assert rc == 1 and md == S

    pack()
    unpack()
    torch.cuda.synchronize()
    base_sample = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from ompi_amd import recipe as _R
        srec, scount, what = sample_recipe(args.config, recipe, count)
        si = _R.build_committed(srec).info()
        sext = si["ub"] - si["lb"]
        hi = max(si["true_ub"], si["true_ub"] + (scount - 1) * sext) if si["size"] else 0
        host_user = user[:min(span, origin + hi)].cpu().numpy()
        base_sample = (srec, scount, what, host_user, packed[:si["size"] * scount].cpu().numpy())

    for _ in range(args.warmup):
        pack()
        unpack()

    every = max(1, args.event_every)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True),
           torch.cuda.Event(enable_timing=True)) if (args.steps - 1 - i) % every == 0 else None
          for i in range(args.steps)]   # counted from the last step: step 0 (host enqueue lag) is skipped

    def step(i):
        es = ev[i]
        if es is None:
            pack()
            unpack()
            return
        e0, e1, e2 = es
        e0.record(stream)
        pack()
        e1.record(stream)
        unpack()
        e2.record(stream)

    def reduce_max(x):
        t = torch.tensor([x], device=dev if backend == "nccl" else "cpu", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    wall = timed_region(step, args.steps, world, torch.cuda.synchronize, reduce_max, dist.barrier)
    ev = [es for es in ev if es is not None]
    tp = float(np.mean([a.elapsed_time(b) for a, b, _ in ev])) / 1e3
    tu = float(np.mean([b.elapsed_time(c) for _, b, c in ev])) / 1e3

    # Every rank's own pack / unpack event times, gathered outside the timed region, so an N > 1
    # line shows the imbalance or a slow rank behind the max-over-ranks wall time
    per_rank = per_rank_times(tp, tu, world, dev, backend) if world > 1 else None

    # The same K steps captured once into a HIP graph and replayed: the launch-bound
    # regime a persistent halo exchange runs in (reported beside the eager value).
    graph_step = None
    if not args.no_graph:
        gs = torch.cuda.Stream(dev)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=gs, capture_error_mode="relaxed"):
            cs = torch.cuda.current_stream(dev)
            cp.set_stream(cs, True)
            cu.set_stream(cs, True)
            for _ in range(args.steps):
                pack()
                unpack()
        cp.set_stream(stream, True)
        cu.set_stream(stream, True)
        with torch.cuda.stream(gs):
            g.replay()
            torch.cuda.synchronize()
            g0, g1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            g0.record(gs)
            g.replay()
            g1.record(gs)
        torch.cuda.synchronize()
        graph_step = g0.elapsed_time(g1) / 1e3 / args.steps

    # The cold-unpack step, outside the timed region: the same pack + unpack
    # with the 1 GiB read flush of face_throughput before the pack and again between pack and
    # unpack (outside the events), so the unpack finds none of the lines the pack just read in
    # the Infinity Cache -- what the headline owes to the stream policy's cache merge.
    cold = None
    if rank == 0 and world == 1 and not args.no_cold:
        scribble = torch.full((1 << 27,), 3, dtype=torch.int64, device=dev)
        cev = []
        for i in range(8):
            a, b_, c_, d_ = (torch.cuda.Event(enable_timing=True) for _ in range(4))
            scribble.sum()
            a.record(stream)
            pack()
            b_.record(stream)
            scribble.sum()
            c_.record(stream)
            unpack()
            d_.record(stream)
            if i >= 2:
                cev.append((a, b_, c_, d_))
        torch.cuda.synchronize()
        cp_ = float(np.median([a.elapsed_time(b_) for a, b_, _, _ in cev])) * 1e3
        cu_ = float(np.median([c_.elapsed_time(d_) for _, _, c_, d_ in cev])) * 1e3
        cold = {"pack_us": round(cp_, 2), "unpack_us": round(cu_, 2), "step_us": round(cp_ + cu_, 2),
                "frac": round(4.0 * S / ((cp_ + cu_) * 1e-6) / HBM_PEAK, 4),
                "GiBs": round(2.0 * S / ((cp_ + cu_) * 1e-6) / GiB, 2),
                "warm_step_us": round((tp + tu) * 1e6, 2),
                "flush": "1 GiB read (a reduction) before the pack and between pack and unpack, outside "
                         "the events: cold and clean caches for each operation"}
        del scribble
        torch.cuda.empty_cache()

    # The floor of this workload on this box, outside the timed region: each of its parts moved
    # by a bare kernel (ompi_amd/csrc/ddt_floor.hip) on the same buffers, in the same pack-then-
    # unpack order.  frac_of_floor = floor / the engine's own event time (1.0 = at the floor).
    floor = None
    if rank == 0 and world == 1 and not args.no_floor and not split:
        try:
            fl = floor_run(args.config, uptr, packed.data_ptr(), recipe=recipe, dev=dev)
        except OSError as ex:   # the measurement library is missing: report, never fail the line
            fl = {"error": f"{type(ex).__name__}: {ex}"[:200]}
        if fl and "error" not in fl:
            if fl["bytes"] != S:
                fl["error"] = f"floor parts cover {fl['bytes']} of {S} packed bytes"
            else:
                step_floor = fl["pack_us"] + fl["unpack_us"]
                fl["step_us"] = round(step_floor, 2)
                fl["frac_of_floor"] = {"pack": round(fl["pack_us"] / (tp * 1e6), 4),
                                       "unpack": round(fl["unpack_us"] / (tu * 1e6), 4),
                                       "step": round(step_floor / ((tp + tu) * 1e6), 4)}
                fl["source"] = ("ompi_amd/csrc/ddt_floor.hip: element gathers (plain loads), element "
                                "scatters (non-temporal stores), 16 KiB block copies (non-temporal loads), "
                                "records through LDS (cfg5), listed elements in address order (cfg4), "
                                "median of 10 rounds; floor = sum of the parts")
        floor = fl
        torch.cuda.synchronize()
    copy = None
    if rank == 0 and world == 1 and not args.no_floor:
        try:
            copy = copy_ceiling(dev)
        except (OSError, AssertionError) as ex:
            copy = {"error": f"{type(ex).__name__}: {ex}"[:200]}

    # The RCCL leg of SURVEY.md §8e, outside the timed region: a consumer that needs the
    # whole packed stream on one device all-gathers the shards (backend "nccl" = RCCL over
    # xGMI); every rank checks that its slice of the gathered stream is its own shard.
    rccl = None
    if use_pg and not args.no_gather:
        try:
            rccl = gather_check(packed, S, world, rank, dev, backend)
        except Exception as ex:   # the timed line stands on its own; report the failed check in it
            rccl = {"backend": backend, "ok": False, "error": f"{type(ex).__name__}: {ex}"[:300]}

    result = None
    if rank == 0:
        ms_per_step = wall / args.steps * 1e3
        value = 2.0 * S_total * args.steps / wall / GiB
        achieved = 4.0 * S / (tp + tu)
        result = {
            "metric": "pack+unpack GiB/s/GPU (device-resident), 256^3 double 3D-vector; %HBM peak",
            # value = the whole job's packed bytes in and out / wall time (the driver
            # contract: units all ranks processed / max-over-ranks time); per GPU beside it
            "value": round(value, 3), "unit": "GiB/s", "n_gpus": world, "steps": args.steps,
            "per_gpu_GiBs": round(value / world, 3), "aggregate_GiBs": round(value, 3),
            "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True, "scaling": "strong" if split else "weak", "vs_baseline": None,
            "dtype": "u8", "data": "synthetic",
            "config": dict(desc, config=args.config, packed_bytes_per_gpu=S,
                           parallelism=(f"strong split over {world} ranks by {split['method']} "
                                        f"({split['total_count']} instances in total, no collective)"
                                        if split else
                                        f"replicas x{world} (fields sharded by count, no collective)")),
            # rank 0's pack + unpack kernel time from HIP events on every 10th timed step (the
            # events add a few us of stream time to those steps, so this sits slightly below
            # a per-GPU share of `value`, which is wall clock over all K steps)
            "per_gpu_GiBs_from_events": round(2.0 * S / (tp + tu) / GiB, 3),
            "all_gather_check": rccl,
            "kernel_ms": {"pack": round(tp * 1e3, 4), "unpack": round(tu * 1e3, 4)},
            "per_rank_kernel_ms": per_rank,
            "graph_replay_GiBs_per_gpu": (round(2.0 * S / graph_step / GiB, 3) if graph_step else None),
            # achieved/frac: the step's pack + unpack launches together (traffic is per step too);
            # dominant_kernel: the longer of the two alone, 2S over its own event time
            "roofline": {"bound": "hbm", "achieved": round(achieved / 1e9, 2), "peak": 8000.0,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK, 4), "traffic": None,
                         "dominant_kernel": {
                             "kernel": "unpack" if tu >= tp else "pack",
                             "us": round(max(tp, tu) * 1e6, 2),
                             "achieved": round(2.0 * S / max(tp, tu) / 1e9, 2),
                             "frac": round(2.0 * S / max(tp, tu) / HBM_PEAK, 4)}},
            "floor_us": floor,
            "cold_step": cold,
        }
        # build provenance: the loaded library's baked-in source identity against the tree this
        # run is in (scripts/srcsha.py)
        try:
            sys.path.insert(0, os.path.join(ROOT, "scripts"))
            import srcsha
            lib_id = ompi_amd.lib().ddt_build_id().decode()
            tree_id = srcsha.source_sha(ROOT)
            result["build"] = {"library_source_sha256": lib_id, "tree_source_sha256": tree_id,
                               "library_built_from_this_tree": lib_id == tree_id,
                               "library": os.path.relpath(ompi_amd.LIB_PATH, ROOT)}
        except Exception as ex:   # reported, never fatal
            result["build"] = {"error": f"{type(ex).__name__}: {ex}"[:200]}
        if copy and "GB_per_s" in copy:
            copy["engine_frac_of_copy"] = round(achieved / 1e9 / copy["GB_per_s"], 4)
        result["copy_ceiling"] = copy
        # The step at the memory's own granularity (r5): the pack reads every touched 128-B user
        # line and writes S, the unpack reads S and writes every touched line back -- the least
        # the memory side can move, since a gather costs its whole line and a partial write
        # completes as one (r5_counter_calibration.json) -- priced at this run's copy ceiling.
        if world == 1 and not split and not args.no_floor:
            try:
                lines = touched_lines(dt, count)
            except (OSError, RuntimeError) as ex:
                lines, result["line_floor_error"] = None, f"{type(ex).__name__}: {ex}"[:200]
            if lines:
                lb = 2 * (lines * 128 + S)
                rate = copy["GB_per_s"] * 1e9 if copy and "GB_per_s" in copy else HBM_MEASURED
                result["line_floor"] = {
                    "touched_lines": lines, "bytes_per_step": lb, "rate_GBs": round(rate / 1e9, 1),
                    "step_us": round(lb / rate * 1e6, 2),
                    "frac": round(lb / rate / (tp + tu), 4),
                    "rule": "2 x (touched 128-B user lines x 128 + packed bytes) per pack + unpack, "
                            "at the copy ceiling measured in this run"}
        # the committed PMC passes were measured on the config's default (weak) message; a
        # --strong message of another size does not inherit them
        tfile = os.path.join(ROOT, "profiles", f"traffic_{args.config}.json")
        if os.path.exists(tfile) and not split:
            with open(tfile) as f:
                result["roofline"]["traffic"] = json.load(f).get("bytes_per_step")
        # Memory-side request roofline: the sparse faces are bound by requests,
        # not bytes.  Request counts per step come from the committed rocprofv3 PMC pass
        # (scripts/requests.py); the rate uses this run's own kernel time.
        rfile = os.path.join(ROOT, "profiles", f"requests_{args.config}.json")
        if os.path.exists(rfile) and not split:
            with open(rfile) as f:
                rq = json.load(f)
            ops = rq["ops_per_step"]
            result["request_roofline"] = {
                "ops_per_step": round(ops), "achieved_G_per_s": round(ops / (tp + tu) / 1e9, 2),
                "peak_G_per_s": rq["ceiling_requests_per_s"] / 1e9,
                "frac": round(ops / (tp + tu) / rq["ceiling_requests_per_s"], 4),
                "source": f"profiles/requests_{args.config}.json"}

    # the single-face and per-face probes run at N = 1 only: under the driver's N > 1 launch they
    # would keep rank 0 busy for tens of seconds after the others (the scaling run needs the line)
    if rank == 0 and world == 1 and args.config == "cfg2" and not args.no_latency:
        result["single_face_latency_us"] = single_face_latency(dev, stream, user, origin)

    if rank == 0 and world == 1 and args.config == "cfg2" and not args.no_faces:
        # per-face figure of the north star: each face type alone, batched over many fields
        # (beyond the Infinity Cache), and at the bench's own 16 fields (launch-bound)
        result["faces"] = face_throughput(dev, args.face_fields, max(5, min(args.steps, 20)))
        result["faces_unflushed"] = face_throughput(dev, args.face_fields, max(5, min(args.steps, 20)),
                                                    flush=None)
        result["faces_at_bench_fields"] = face_throughput(dev, count, max(5, min(args.steps, 20)))
        # back-to-back operations between one event pair, eager and as a replayed graph: the
        # per-operation cost without an event pair around every operation
        for fields, key in ((count, "faces_at_bench_fields"), (1, "single_face_latency_us")):
            if key not in result:
                continue
            bb = back_to_back(dev, fields)
            result[key]["back_to_back"] = bb
            for k in ("x", "y", "z"):
                result[key].setdefault(k, {})
                result[key][k]["back_to_back_us"] = bb[k]["back_to_back_us"]
                result[key][k]["graph_us"] = bb[k]["graph_us"]

    if rank == 0 and world == 1 and args.config == "cfg3" and not args.no_faces and not split:
        # config 3's faces alone: dim0 / dim1 / dim2 of the 512^3 float grid,
        # cold and clean over --face-fields fields (at most 256 here: 128 GiB of fields, 256 MiB
        # per plane face, so one launch is not dominated by the event and launch floor as it is
        # at 64 fields), with each face's bare kernel under the same protocol
        user = packed = None
        torch.cuda.empty_cache()
        ff = min(args.face_fields, 256)
        result["faces"] = face_throughput(dev, ff, max(5, min(args.steps, 20)),
                                          faces=("dim0", "dim1", "dim2"), grid="cfg3")

    if rank == 0 and world == 1 and args.e2e:
        # the path starts and ends in host memory (north star): the copies to and from the GPU
        # included, for the small, the default and the largest config, pinned and pageable
        user = packed = None
        torch.cuda.empty_cache()
        result["e2e"] = [end_to_end(dev, c, pageable=pg, reps=5)
                         for c in ("cfg1", "cfg2", "cfg5") for pg in (False, True)]

    if rank == 0 and base_sample is not None:
        srec, scount, what, host_user, gpu_prefix = base_sample
        result["cpu_baseline"] = cpu_baseline(args.config, srec, scount, what, host_user, origin,
                                              gpu_prefix)
    elif rank == 0:
        result["cpu_baseline"] = None   # timed on rank 0 at N = 1 only
    if rank == 0:
        sys.stdout.flush()
        os.write(result_fd, (json.dumps(result) + "\n").encode())
    if use_pg:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
