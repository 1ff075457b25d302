"""pack_description_sweep.c restated (ompi/test/datatype/pack_description_sweep.c) -- test
infrastructure shared by the CPU and GPU sweep tests.

The reference's sweep builds a regular typemap -- `total_items` items, each `data_count` blocks
of `blocklen` elements (4- or 8-byte) at a stride of `blocklen + block_gap` elements, items
`item_gap` elements apart -- commits it, and then either keeps the optimizer's result
(--commit-description) or REPLACES opt_desc with an exact synthetic shape
(install_synthetic_description, :254-316): one LOOP over `loop_items` DATA entries of
`count = data_count, blocklen, extent = block stride` -- not CREATE_ELEM-collapsed, so a gapless
stride still reads as `count` blocks -- closed by its END_LOOP, then the `total_items % loop_items`
items that do not fill a loop iteration as straight-line DATA entries after it, and the END_LOOP
sentinel.  Its accelerator backend swaps fAdvance for opal_pack/unpack_accelerator_simple after
prepare (:877-960) and converts in `fragment_bytes` pieces (run_prepared_convertor, :962-996);
every packed stream is checked against pack_reference (:454-476), an independent loop over
(datatype, item, block).
"""
from __future__ import annotations

import random

import numpy as np

from . import opal_shapes as S
from . import oracle as O

FLOAT4, FLOAT8 = 15, 16
BASIC_DATA = 0x136 | 0x100   # OPAL_DATATYPE_FLAG_BASIC | OPAL_DATATYPE_FLAG_DATA (:244-246)


class Sweep:
    """One configuration of the sweep (benchmark_config_t, :67-86)."""

    def __init__(self, element_size=8, data_count=3, blocklen=4, block_gap=1, item_gap=1,
                 total_items=10, loop_items=4, datatype_count=1, commit_description=False):
        assert element_size in (4, 8) and total_items >= loop_items >= 1
        assert not commit_description or total_items % loop_items == 0
        self.es, self.dc, self.bl, self.bg, self.ig = element_size, data_count, blocklen, block_gap, item_gap
        self.total, self.loop, self.count = total_items, loop_items, datatype_count
        self.commit = commit_description
        self.tid = FLOAT8 if element_size == 8 else FLOAT4
        # create_synthetic_datatype (:318-358)
        self.block_stride = (blocklen + block_gap) * element_size
        self.item_extent = blocklen * element_size + (data_count - 1) * self.block_stride + item_gap * element_size
        if commit_description:
            self.item_extent += element_size   # the trailing gap that keeps items apart (:352-359)
        self.otype = self._datatype()
        info = self.otype.info()
        self.info = info
        self.size = info["size"]
        self.extent = info["ub"] - info["lb"]

    def __repr__(self):
        return (f"Sweep(es={self.es}, dc={self.dc}, bl={self.bl}, bg={self.bg}, ig={self.ig}, "
                f"total={self.total}, loop={self.loop}, count={self.count}, commit={self.commit})")

    def _datatype(self):
        """The MPI datatype the sweep commits (:360-416), built by the oracle."""
        vec = O.vector(self.dc, self.bl, self.bl + self.bg, O.basic(self.tid))
        if self.commit:
            rec = O.struct([1] * self.loop, [i * self.item_extent for i in range(self.loop)], [vec] * self.loop)
            rec = O.resized(rec, 0, self.loop * self.item_extent)
            return O.contiguous(self.total // self.loop, rec)
        return O.contiguous(self.total, O.resized(vec, 0, self.item_extent))

    @property
    def contiguous(self) -> bool:
        """The synthetic backend refuses a contiguous datatype (:429-438)."""
        return bool(self.info["flags"] & S.F_CONTIGUOUS)

    def recipe(self):
        """The same datatype as an engine recipe (tests/recipes.py form)."""
        vec = ("vector", self.dc, self.bl, self.bl + self.bg, ("basic", self.tid))
        if self.commit:
            st = ("struct", [1] * self.loop, [i * self.item_extent for i in range(self.loop)], [vec] * self.loop)
            return ("contig", self.total // self.loop, ("resized", st, 0, self.loop * self.item_extent))
        return ("contig", self.total, ("resized", vec, 0, self.item_extent))

    def synthetic_entries(self):
        """install_synthetic_description (:254-316): the 32-byte opt_desc entries (no sentinel)."""
        iters = self.total // self.loop
        tail = self.total % self.loop
        loop_size = self.loop * self.dc * self.bl * self.es
        loop_extent = self.item_extent * self.loop
        ents = [S.loop(iters, self.loop + 1, loop_extent, 0)]
        for item in range(self.loop):
            ents.append(S.data(self.tid, self.dc, self.bl, self.block_stride, self.item_extent * item,
                               flags=BASIC_DATA))
        ents.append(S.end_loop(self.loop + 1, loop_size, 0, 0))
        for item in range(tail):
            ents.append(S.data(self.tid, self.dc, self.bl, self.block_stride,
                               loop_extent * iters + self.item_extent * item, flags=BASIC_DATA))
        return ents

    def opal_type(self):
        """The committed opal_datatype_t the sweep's convertor sees: desc from the constructors,
        opt_desc = the synthetic shape (or, with commit_description, the optimizer's own)."""
        if self.commit:
            return S.from_oracle(self.otype)
        i = self.info
        desc = [S.pack_entry(e) for e in self.otype.desc()]
        return S.OpalType(desc, i["size"], i["lb"], i["ub"], i["true_lb"], i["true_ub"],
                          flags=i["flags"] & (S.F_CONTIGUOUS | S.F_NO_GAPS),
                          opt_entries=self.synthetic_entries(), first_disp=0)

    def blocks(self):
        """(source offset, packed offset, bytes) of every block of `count` datatypes in the order
        pack_reference (:454-476) copies them."""
        bb = self.bl * self.es
        out, p = [], 0
        item_extent = self.extent // self.total
        for d in range(self.count):
            for item in range(self.total):
                for blk in range(self.dc):
                    out.append((d * self.extent + item * item_extent + blk * self.block_stride, p, bb))
                    p += bb
        return out

    def span(self):
        """Bytes of user memory `count` instances touch (from the type origin, lb = 0)."""
        return (self.count - 1) * self.extent + self.info["true_ub"]

    def pack_reference(self, source: np.ndarray) -> np.ndarray:
        """pack_reference (:454-476) on a byte array holding `count` datatypes."""
        bb = self.bl * self.es
        out = np.empty(self.count * self.size, dtype=np.uint8)
        for s, p, n in self.blocks():
            out[p:p + bb] = source[s:s + bb]
        return out

    def unpack_reference(self, packed: np.ndarray, target: np.ndarray) -> np.ndarray:
        """The inverse of pack_reference into a copy of `target` (gaps keep their bytes)."""
        out = target.copy()
        for s, p, n in self.blocks():
            out[s:s + n] = packed[p:p + n]
        return out


def random_sweeps(rng: random.Random, n: int, commit: bool = False):
    """Configurations across the matrix: element_size 4/8, data_count 1-5, blocklen 1-64,
    block_gap 0-3, item_gap 0-2, total_items mostly not a multiple of loop_items (tail entries),
    datatype_count 1-3; contiguous datatypes (refused by the sweep) are skipped."""
    out = []
    while len(out) < n:
        loop = rng.randint(1, 6)
        total = loop * rng.randint(1, 5) + (0 if commit else rng.choice([0, 1, 2, 3, loop - 1]) % loop)
        total = max(total, loop)
        sw = Sweep(element_size=rng.choice([4, 8]), data_count=rng.randint(1, 5),
                   blocklen=rng.choice([1, 2, 3, 5, 8, 13, 32, 64]), block_gap=rng.randint(0, 3),
                   item_gap=rng.randint(0, 2), total_items=total, loop_items=loop,
                   datatype_count=rng.randint(1, 3), commit_description=commit)
        if not sw.contiguous:
            out.append(sw)
    return out
