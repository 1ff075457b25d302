#!/usr/bin/env python3
"""Per-kernel memory-side request counts from rocprofv3 --pmc CSVs (TCC_EA0_RDREQ /
TCC_EA0_WRREQ ... per dispatch): median per kernel name.
Usage: python scripts/reqs.py a.csv [b.csv ...]"""
import collections
import csv
import statistics
import sys


def main(paths):
    agg = collections.defaultdict(list)
    for p in paths:
        for r in csv.DictReader(open(p)):
            name = r["Kernel_Name"].split("(")[0][:60]
            agg[(name, r["Counter_Name"])].append(float(r["Counter_Value"]))
    for (name, ctr), v in sorted(agg.items()):
        print(f"{name:60s} {ctr:28s} median {statistics.median(v):14.0f}  (n={len(v)})")


if __name__ == "__main__":
    main(sys.argv[1:])
