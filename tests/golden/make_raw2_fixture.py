#!/usr/bin/env python3
"""Regenerate tests/golden/ddt_raw2_desc.json (run in the build container only).

The reference's raw-export test (ompi/test/datatype/ddt_raw2.c) installs a hand-written
committed description (185 dt_elem_desc_t entries) and bounds directly into a datatype.
Then it checks that opal_convertor_raw yields the same iovec list when called with room
for 300, 10 or 1 iovecs per call.

This script extracts that description, as numbers only, from the test's initializer.
The fixture rows are:
  ["loop",  flags, type, items, loops, unused, extent]
  ["elem",  flags, type, count, blocklen, extent, disp]
  ["end",   flags, type, items, unused, size, first_elem_disp]
(field order of opal_datatype_internal.h:119-160).
"""
import json
import os
import re
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = "/root/reference/ompi/test/datatype/ddt_raw2.c"


def main():
    text = open(SRC).read()
    body = text[text.index("dt_elem_desc_t descs[185]"):]
    body = body[:body.index("};")]
    rows = []
    for kind, flags, typ, rest in re.findall(
            r"\{\.(loop|elem|end_loop)\s*=\s*\{\{(-?\d+),\s*(-?\d+)\},\s*([-\d,\s]+)\}\}", body):
        nums = [int(x) for x in rest.replace(" ", "").split(",") if x]
        rows.append([{"end_loop": "end"}.get(kind, kind), int(flags), int(typ)] + nums)
    fields = {}
    for key in ("flags", "id", "bdt_used", "size", "true_lb", "true_ub", "lb", "ub", "nbElems",
                "align", "stack_depth"):
        m = re.search(r"datatype->super\.%s = (-?\d+);" % key, text)
        fields[key] = int(m.group(1))
    used = int(re.search(r"datatype->super\.opt_desc\.used = (\d+);", text).group(1))
    out = {"source": "ompi/test/datatype/ddt_raw2.c (descs[] initializer and datatype->super fields)",
           "used": used, "bounds": fields, "desc": rows,
           "checks": "raw export with 300, 10 and 1 iovecs per call must give the same list "
                     "(ddt_raw2.c:196-211); the bytes described must equal size"}
    assert len(rows) >= used, (len(rows), used)
    rows_txt = ",\n".join("  " + json.dumps(r) for r in rows)
    head = json.dumps({k: v for k, v in out.items() if k != "desc"}, indent=1)[:-2]
    with open(os.path.join(HERE, "ddt_raw2_desc.json"), "w") as f:
        f.write(head + ',\n "desc": [\n' + rows_txt + "\n ]\n}\n")
    print(f"{len(rows)} entries, used {used}")


if __name__ == "__main__":
    sys.exit(main())
