#!/usr/bin/env python3
"""HBM traffic per pack+unpack step from rocprofv3 --pmc passes (FETCH_SIZE and WRITE_SIZE
collected in separate runs, MI355X_MICROARCH.md "HBM [CDNA4]").

FETCH_SIZE and WRITE_SIZE are KiB.  gfx950 correction: FETCH_SIZE tallies each 128-B read
request at 64 B (exactly half of a 16-B/lane streaming read, guide + our own calibration
with scripts/kbench.py on a contiguous copy), so read bytes = 2 x FETCH_SIZE.  For the
8-B x-face gathers one request per element is issued, so the same factor prices each at a
128-B line -- verified in round 2 (scripts/ubench_gran.hip, profiles/r2_ubench_gran.log): an
8-byte gather per line costs the same request, FETCH_SIZE and time as a whole 128-byte line.  WRITE_SIZE is taken as is (exact for streaming stores; scattered 8-B stores
are tallied as 32-B sectors, which is what the memory side receives).

usage: python scripts/traffic.py FETCH.csv WRITE.csv CONFIG > profiles/traffic_CONFIG.json
"""
from __future__ import annotations

import collections
import csv
import json
import sys


def family(kernel_name):
    """ddt_move_kernel / ddt_move_inline_kernel (either launch form) = one family per step."""
    for f in ("k_pack1", "k_pack2", "k_unpack1", "k_unpack2"):
        if f in kernel_name:
            return f
    return "move"


def per_kernel(path, counter):
    """Per direction: the sum over its kernels of each kernel's mean per dispatch (the
    address-ordered list engine runs two kernels per pack and per unpack)."""
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"]
        if r["Counter_Name"] != counter:
            continue
        if "ddt_move" in k or "ddt_dense" in k:
            direction = "pack" if ("<0," in k or "<0>" in k) else "unpack"
        elif "k_pack" in k or "k_unpack" in k:
            direction = "pack" if "k_pack" in k else "unpack"
        else:
            continue
        acc[(direction, family(k))].append(float(r["Counter_Value"]) * 1024.0)
    out, n = collections.defaultdict(float), collections.defaultdict(int)
    for (d, _), v in acc.items():
        out[d] += sum(v) / len(v)
        n[d] += len(v)
    return dict(out), dict(n)


def main():
    fetch_csv, write_csv, cfg = sys.argv[1:4]
    fetch, nf = per_kernel(fetch_csv, "FETCH_SIZE")
    write, nw = per_kernel(write_csv, "WRITE_SIZE")
    out = {"config": cfg, "unit": "bytes", "read_correction": 2.0,
           "launches_averaged": {"fetch": nf, "write": nw}, "per_launch": {}}
    total = 0.0
    for d in ("pack", "unpack"):
        rd = 2.0 * fetch.get(d, 0.0)
        wr = write.get(d, 0.0)
        out["per_launch"][d] = {"FETCH_SIZE_bytes": fetch.get(d), "read_bytes": rd,
                                "WRITE_SIZE_bytes": wr, "hbm_bytes": rd + wr}
        total += rd + wr
    out["bytes_per_step"] = total
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
