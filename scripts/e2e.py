#!/usr/bin/env python3
"""bench.end_to_end from the command line (variants and tunings): the end-to-end rate with a
HOST-resident packed stream, one JSON line per run.  `bench.py --e2e` runs the
standard set (cfg1, cfg2, cfg5; pinned and pageable) into the bench line."""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402


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
    out = bench.end_to_end(dev, args.config, pageable=args.pageable, reps=args.reps, tune=tune,
                           hostdirect=args.hostdirect, stage_mb=args.stage_mb)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
