#!/usr/bin/env python3
"""Per-kernel means of rocprofv3 --pmc counters over any number of passes (one CSV each):
one JSON object {kernel family: {counter: mean per dispatch, "dispatches": n}}.  Families:
the engine's move kernels by direction, the address-ordered passes by name, anything else by
its demangled name's first 60 characters.

usage: python scripts/pmc_summary.py PASS.csv [PASS.csv ...] > profiles/rN_pmc_CFG.json"""
from __future__ import annotations

import collections
import csv
import json
import sys


def family(k):
    for f in ("k_pack1", "k_pack2", "k_unpack1", "k_unpack2"):
        if f in k:
            return f
    if "ddt_move" in k or "ddt_dense" in k:
        return ("pack " if ("<0," in k or "<0>" in k) else "unpack ") + k.split("(")[0].split("::")[-1][:40]
    return k.split("(")[0][:60]


def main():
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for path in sys.argv[1:]:
        for r in csv.DictReader(open(path)):
            acc[family(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {}
    for fam, cs in sorted(acc.items()):
        out[fam] = {c: round(sum(v) / len(v), 1) for c, v in sorted(cs.items())}
        out[fam]["dispatches"] = max(len(v) for v in cs.values())
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
