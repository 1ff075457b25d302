#!/usr/bin/env python3
"""Memory-side requests per pack+unpack step from one rocprofv3 --pmc pass with
TCC_EA0_RDREQ_sum, TCC_EA0_WRREQ_sum and TCC_EA0_WRREQ_64B_sum (the L2 -> fabric request
counters FETCH_SIZE/WRITE_SIZE are derived from; MI355X_MICROARCH.md "HBM [CDNA4]").

Calibration (scripts/ubench4.hip, profiles/r1_ubench4_requests.log): a 16 B/lane streaming
read issues one RDREQ per 128 B line, a streaming store one 64 B WRREQ per 64 B; an 8-byte
gather one RDREQ per element; an 8-byte scatter one WRREQ (not 64 B) per element, which the
memory side completes as a read-modify-write of its sector.  So a step costs
    rd + wr + partial   memory-side operations,  partial = wr - wr64,
and the highest request rate measured for any access pattern is a streaming copy's.  Round 2
re-measured that ceiling (scripts/ubench_copy.hip, profiles/r2_ubench_copy.log and
profiles/r2_copy_requests.log): every copy variant issues one RDREQ per 128 B read and one
64 B WRREQ per 64 B written (3B/128 requests for B bytes), and the fastest (16 KiB chunks,
non-temporal loads and stores) copies at 6.2 TB/s r+w: 72.7 G requests/s.  (Round 1 quoted
61.7 G/s from a slower 5.2 TB/s copy.)

usage: python scripts/requests.py PMC.csv CONFIG > profiles/requests_CONFIG.json
"""
from __future__ import annotations

import collections
import csv
import json
import sys


def family(kernel_name):
    """ddt_move_kernel / ddt_move_inline_kernel (either launch form) = one family per step."""
    for f in ("k_pack1", "k_pack2", "k_unpack1", "k_unpack2"):
        if f in kernel_name:
            return f
    return "move"

CEILING = 72.7e9   # requests/s of the 6.2 TB/s streaming copy (ubench_copy, r2)


def main():
    path, cfg = sys.argv[1:3]
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"]
        if "ddt_move" in k or "ddt_dense" in k:
            d = "pack" if ("<0," in k or "<0>" in k) else "unpack"
        elif "k_pack" in k or "k_unpack" in k:
            d = "pack" if "k_pack" in k else "unpack"
        else:
            continue
        acc[(d, family(k), r["Counter_Name"])].append(float(r["Counter_Value"]))
    # per kernel family: mean over its dispatches; per direction: sum over its families (the
    # address-ordered list engine runs two kernels per direction).  The move kernel's
    # kernel-argument and by-pointer launches are one family: one of them runs per step.
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for (d, _, ctr), v in acc.items():
        per[d][ctr] += sum(v) / len(v)
    out = {"config": cfg, "ceiling_requests_per_s": CEILING, "per_step": {}}
    total = 0.0
    for d in ("pack", "unpack"):
        c = per[d]
        rd, wr, w64 = c["TCC_EA0_RDREQ_sum"], c["TCC_EA0_WRREQ_sum"], c["TCC_EA0_WRREQ_64B_sum"]
        ops = rd + wr + (wr - w64)
        out["per_step"][d] = {"rd": rd, "wr": wr, "wr64": w64, "partial": wr - w64, "ops": ops}
        total += ops
    out["ops_per_step"] = total
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
