"""Oracle and engine plans pinned to the reference's own known answers.

tests/golden/corpus_sha256.json holds, for every datatype of the reference corpus
(ompi/test/datatype/datatype_corpus.c), the SHA-256 of the stream its independent
by-hand packer produces for 7 instances (regenerate: tests/golden/make_golden.py).
"""
from __future__ import annotations

import hashlib
import json
import os

import numpy as np
import pytest

from . import corpus
from . import plan_emu as E
from . import recipes as R

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "corpus_sha256.json")))
NAMES = sorted(corpus.CORPUS)


def _setup(name):
    rec, byhand = corpus.CORPUS[name]()
    b = R.Built(rec)
    g = GOLD[name]
    info = b.o.info()
    span, origin = R.layout(info, g["count"])
    buf = R.fill(span, 0x5A)
    return b, byhand, g, info, span, origin, buf


def test_golden_covers_corpus():
    assert set(GOLD) == set(corpus.CORPUS)


@pytest.mark.parametrize("name", NAMES)
def test_oracle_matches_reference_byhand(name):
    b, byhand, g, info, span, origin, buf = _setup(name)
    s = b.o.pack(g["count"], buf, origin, 0, g["count"] * info["size"], element_granular=False)
    assert len(s) == g["packed_bytes"]
    assert hashlib.sha256(s).hexdigest() == g["sha256"]
    # fragment matrix of opt_desc_equiv.c:63 through the element-granular pack
    total = g["count"] * info["size"]
    for frag in (12, 16, 40, 4096):
        pos, parts = 0, []
        while pos < total:
            piece = b.o.pack(g["count"], buf, origin, pos, frag)
            if not piece:   # element larger than the fragment
                piece = b.o.pack(g["count"], buf, origin, pos, total - pos)
            parts.append(piece)
            pos += len(piece)
        assert hashlib.sha256(b"".join(parts)).hexdigest() == g["sha256"]


@pytest.mark.parametrize("name", NAMES)
def test_engine_bounds_and_plan_match(name):
    b, byhand, g, info, span, origin, buf = _setup(name)
    ei = b.engine().info()
    for k in ("size", "lb", "ub", "true_lb", "true_ub", "align"):
        assert ei[k] == info[k], (name, k)
    np.testing.assert_array_equal(E.engine_blocks(b.engine()), E.oracle_blocks(b.o))
    # the exact launch descriptors, replayed: whole message
    UA, PA = (1 << 40) + 4096, 1 << 41
    total = g["count"] * info["size"]
    its = E.items(b.engine(), g["count"], UA + origin, PA, 0, total)
    packed = np.zeros(total, dtype=np.uint8)
    cov = E.emulate(its, buf, UA, packed, PA, 0, E.list_tables(b.engine()))
    assert np.all(cov == 1)
    assert hashlib.sha256(packed.tobytes()).hexdigest() == g["sha256"]
