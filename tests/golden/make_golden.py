#!/usr/bin/env python3
"""Regenerate tests/golden/corpus_sha256.json.

For every entry of the reference datatype corpus (tests/corpus.py, restating
ompi/test/datatype/datatype_corpus.c), pack COUNT=7 instances (opt_desc_equiv.c:314)
of a position-hash-filled buffer with the reference's own by-hand packer and record
the SHA-256 of the packed stream, its length and the type bounds.  The by-hand packers
are independent of both the oracle and the engine, so these digests pin both.
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from tests import corpus, recipes as R  # noqa: E402

COUNT = 7


def byhand_stream(regions, buf, origin):
    return b"".join(buf[origin + off: origin + off + n].tobytes() for off, n in regions)


def main():
    out = {}
    for name, mk in corpus.CORPUS.items():
        rec, byhand = mk()
        b = R.Built(rec)
        info = b.o.info()
        span, origin = R.layout(info, COUNT)
        buf = R.fill(span, 0x5A)
        s = byhand_stream(byhand(COUNT), buf, origin)
        out[name] = {"count": COUNT, "packed_bytes": len(s), "sha256": hashlib.sha256(s).hexdigest(),
                     "size": info["size"], "lb": info["lb"], "extent": info["ub"] - info["lb"],
                     "true_lb": info["true_lb"], "true_extent": info["true_ub"] - info["true_lb"]}
    with open(os.path.join(HERE, "corpus_sha256.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print(f"wrote {len(out)} entries")


if __name__ == "__main__":
    main()
