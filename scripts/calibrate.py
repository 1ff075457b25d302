#!/usr/bin/env python3
"""Counter calibration on the engine's own access patterns: combines the
rocprofv3 --pmc passes over scripts/calib.hip with its own event timings into per-line figures.

usage: python scripts/calibrate.py TIMING.jsonl LINES PASS.csv [PASS.csv ...] > profiles/r5_counter_calibration.json

Per (pattern, cold|warm): each counter per line (KiB counters as bytes), the event time and the
line rate.  Derived:
  fetch_factor  = known line bytes (128 per touched line; the stream's own bytes) / FETCH_SIZE bytes:
                  the factor that turns FETCH_SIZE into whole 128-B lines for that pattern
  rdreq_per_line, wrreq_per_line (64-B and partial): memory-side requests per touched line
  write_factor  = useful bytes written / WRITE_SIZE bytes
The guide's one calibrated case (16-B/lane streaming read: FETCH_SIZE = half the bytes) is the
stream_read row; every other row is this program's own known byte count."""
from __future__ import annotations

import collections
import csv
import json
import re
import sys

NAMES = ["stream_read", "stream_write", "gather8", "gather4", "gather8_pair64", "gather8_pair8",
         "scatter8_nt", "scatter8", "scatter4_nt", "gather8_dense", "gather8_nt", "coop8", "coop8_nt",
         "gather16"]
# useful bytes read / written per line by each pattern (streams: one 128-B line = 8 lanes x 16 B)
USEFUL = {"stream_read": (128, 0), "stream_write": (0, 128), "gather8": (8, 8), "gather4": (4, 4),
          "gather8_pair64": (16, 16), "gather8_pair8": (16, 16), "scatter8_nt": (0, 8),
          "scatter8": (0, 8), "scatter4_nt": (0, 4), "gather8_dense": (8, 8), "gather8_nt": (8, 8),
          "coop8": (8, 8), "coop8_nt": (8, 8), "gather16": (8, 8)}
KIB = {"FETCH_SIZE", "WRITE_SIZE"}


def main():
    timing, lines = sys.argv[1], int(sys.argv[2])
    pmc = sys.argv[3:]
    t = {}
    for ln in open(timing):
        if ln.startswith("{"):
            r = json.loads(ln)
            t[(r["pattern"], r["run"])] = r["us"]
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    pat = re.compile(r"cal<(\d+), (\d+)>")
    for path in pmc:
        for r in csv.DictReader(open(path)):
            m = pat.search(r["Kernel_Name"])
            if not m:
                continue
            name, run = NAMES[int(m.group(1))], "warm" if m.group(2) == "1" else "cold"
            v = float(r["Counter_Value"]) * (1024.0 if r["Counter_Name"] in KIB else 1.0)
            acc[(name, run)][r["Counter_Name"]].append(v)
    out = {"lines": lines, "pitch_bytes": 2048, "source": "scripts/calib.hip under rocprofv3 --pmc "
           "(one pass per counter group) and its own HIP-event timings", "patterns": {}}
    for name in NAMES:
        for run in ("cold", "warm"):
            c = acc.get((name, run), {})
            per = {k: sum(v) / len(v) / lines for k, v in c.items()}
            row = {"us": t.get((name, run)), "per_line": {k: round(v, 3) for k, v in per.items()}}
            if row["us"]:
                row["G_lines_per_s"] = round(lines / (row["us"] * 1e-6) / 1e9, 2)
            rd, wr = USEFUL[name]
            f = per.get("FETCH_SIZE")
            if f:
                # bytes a touched line is worth: the stream's own 128, a gather's whole line
                row["fetch_factor_to_128B_lines"] = round(128.0 / f, 3) if rd else None
            w = per.get("WRITE_SIZE")
            if w and wr:
                row["write_factor"] = round(wr / w, 3)
            rq = per.get("TCC_EA0_RDREQ_sum")
            if rq is not None:
                row["rdreq_per_line"] = round(rq, 3)
            wq, w64 = per.get("TCC_EA0_WRREQ_sum"), per.get("TCC_EA0_WRREQ_64B_sum")
            if wq is not None:
                row["wrreq_per_line"] = round(wq, 3)
                if w64 is not None:
                    row["wrreq_partial_per_line"] = round(wq - w64, 3)
            out["patterns"][f"{name}/{run}"] = row
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
