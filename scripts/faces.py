#!/usr/bin/env python3
"""Per-face pack/unpack of the 256^3 double grid, alone (bench.face_throughput): the run
profiled with rocprofv3 for the per-face kernel statistics in profiles/r2_faces_*."""
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
    ap.add_argument("--fields", type=int, default=512)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--faces", default="x,y,z")
    ap.add_argument("--flush", default="read", choices=["read", "write", "none"],
                    help="1 GiB scribble touched between operations (bench.face_throughput)")
    args = ap.parse_args()
    r = bench.face_throughput(torch.device("cuda:0"), args.fields, args.steps,
                              faces=tuple(args.faces.split(",")), flush=None if args.flush == "none" else args.flush)
    print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
