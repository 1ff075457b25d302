#!/bin/bash
# Round-6: threads through the drop-in after the per-thread objects moved to cache lines of their
# own (slot records, bridge thread state, convertors, descriptor sets, plans), beside HIP alone.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
T=${TAG:-r6t2}
: > gpurun_out/${T}_threads.jsonl
run() { local name=$1; shift; timeout -k 10 150 "$@" > gpurun_out/${T}_$name.log 2>&1 || { echo "$name failed"; tail -5 gpurun_out/${T}_$name.log; exit 1; }; grep '^{' gpurun_out/${T}_$name.log >> gpurun_out/${T}_threads.jsonl; }
run hip ./scripts/hipthreads 1000 0 1
run face ./scripts/bridgethreads 1000 own async face
run tiny ./scripts/bridgethreads 1000 own async tiny
run face_shared ./scripts/bridgethreads 1000 shared async face
run sync ./scripts/bridgethreads 500 own sync face
python3 - <<PY
import json
for l in open("gpurun_out/${T}_threads.jsonl"):
    r = json.loads(l)
    h = r.get("host_us_per_call")
    h = h["mean"] if isinstance(h, dict) else h
    print(r["what"][:60], r["threads"], h, r.get("aggregate_calls_per_s"), r.get("speedup_vs_1"))
PY
