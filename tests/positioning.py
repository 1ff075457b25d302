"""position.c restated (ompi/test/datatype/position.c:42-135): shared by the CPU and GPU tests.

The reference simulates multi-network scheduling: a send convertor prepared on the datatype
cuts the packed stream into segments by set_position(segment start + fragment size), which
snaps back to a predefined-element boundary (opal_convertor_position_generic,
opal_convertor.c:458-470); the segments are shuffled, then packed through set_position + pack
on a send convertor and unpacked through set_position + unpack on a receive convertor.
"""
from __future__ import annotations

from typing import Callable, List, Tuple


def create_segments(total: int, segment_length: int,
                    set_position: Callable[[int], int]) -> List[Tuple[int, int]]:
    """position.c:42-85.  `set_position(p)` is opal_convertor_set_position on ONE send
    convertor (prepared once, positions increasing) and returns where it landed.  Starts with
    ceil(total / segment_length) segments and adds one until they cover the stream."""
    seg_count = total // segment_length
    if seg_count * segment_length != total:
        seg_count += 1
    while True:
        segs, position, covered = [], 0, 0
        for _ in range(seg_count):
            start = position
            position = set_position(position + segment_length)
            segs.append((start, position - start))
            covered += position - start
        if covered == total:
            return segs
        seg_count += 1


def shuffle_segments(segs):
    """position.c:87-98: swap segment i with its mirror for every other i in the first half."""
    segs = list(segs)
    n = len(segs)
    for i in range(0, n // 2, 2):
        segs[i], segs[n - i - 1] = segs[n - i - 1], segs[i]
    return segs
