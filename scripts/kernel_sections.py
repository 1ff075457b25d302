#!/usr/bin/env python3
"""Summarise a `rocprofv3 --kernel-trace` database of scripts/small_launch.py by section.

small_launch.py enqueues each (face, fields, path) measurement behind torch's spin kernel, so the
spin kernels split the trace into sections: the empty-kernel probe, then y/z/x faces at 1 and
16 fields through the engine, the bare kernel and a contiguous copy.  For each section: the mean
start-to-end span per kernel, the median gap between kernels, and per kernel name its count,
median duration and workgroup count.

usage: scripts/kernel_sections.py gpurun_out/r4_small_prof
"""
import glob
import sqlite3
import statistics as st
import sys


def main(path):
    db = glob.glob(path + "/*.db")[0]
    c = sqlite3.connect(db)
    rows = c.execute("select name,start,end,duration,grid_x,workgroup_x from kernels order by start").fetchall()
    secs, cur = [], None
    for r in rows:
        if "spin_kernel" in r[0]:
            cur = []
            secs.append(cur)
            continue
        if cur is not None:
            cur.append(r)
    labels = ["empty"] + [f"{f}{n} {p}" for f in "yzx" for n in (1, 16) for p in ("engine", "bare", "copy")]
    for lab, s in zip(labels, secs):
        if not s:
            continue
        by = {}
        for r in s:
            by.setdefault(r[0].split("(")[0].replace("void ", "")[-48:], []).append(r)
        gaps = [(s[i + 1][1] - s[i][2]) / 1e3 for i in range(len(s) - 1)]
        span = (s[-1][2] - s[0][1]) / 1e3 / len(s)
        parts = "; ".join(f"{nm} x{len(v)} {st.median([x[3] / 1e3 for x in v]):.2f}us wg{v[0][4] // v[0][5]}"
                          for nm, v in by.items())
        print(f"{lab:18s} per-kernel span {span:6.2f}us gap {st.median(gaps) if gaps else 0:5.2f}us | {parts}")


if __name__ == "__main__":
    main(sys.argv[1])
