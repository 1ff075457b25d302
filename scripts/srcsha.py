#!/usr/bin/env python3
"""The source identity of libddt_hip.so: sha256 over (path, NUL, content, NUL) of every file the
library is compiled from, in sorted path order.  The Makefile bakes it into the library at link
time (ddt_build_id); bench.py recomputes it from the tree it runs in and reports whether the
loaded library was built from exactly these sources (build provenance)."""
from __future__ import annotations

import glob
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def source_files(root: str = ROOT) -> list[str]:
    pats = ["ompi_amd/csrc/*.cpp", "ompi_amd/csrc/*.hip", "ompi_amd/csrc/*.h", "include/*.h",
            "bridge/opal_datatype_hip_bridge.c", "ompi_amd/csrc/Makefile"]
    out = set()
    for p in pats:
        out.update(os.path.relpath(f, root) for f in glob.glob(os.path.join(root, p)))
    out.discard(os.path.join("ompi_amd", "csrc", "ddt_floor.hip"))   # measurement library only
    return sorted(out)


def source_sha(root: str = ROOT) -> str:
    h = hashlib.sha256()
    for rel in source_files(root):
        h.update(rel.encode() + b"\0")
        with open(os.path.join(root, rel), "rb") as f:
            h.update(f.read())
        h.update(b"\0")
    return h.hexdigest()


if __name__ == "__main__":
    print(source_sha(sys.argv[1] if len(sys.argv) > 1 else ROOT))
