#!/usr/bin/env python3
"""Short per-kernel table from a rocprofv3 --stats kernel_stats.csv."""
import csv
import re
import sys


def short(name):
    name = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return re.sub(r"\(.*", "", name)[:70]


for r in csv.DictReader(open(sys.argv[1])):
    print(f"{short(r['Name']):70s} calls {r['Calls']:>5} avg {float(r['AverageNs']) / 1e3:10.1f} us")
