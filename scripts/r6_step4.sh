#!/bin/bash
# Round-6 GPU step 4: the whole GPU suite, thread scaling after the run_windows restructure, and
# the pipelined pack pass 1 A/B on config 4.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
T=${TAG:-r6n}
timeout -k 10 900 python -u -m pytest -q -x -m gpu --timeout 300 --timeout-method thread tests > gpurun_out/${T}_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/${T}_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/${T}_pytest_gpu.log
run() { local name=$1; shift; timeout -k 10 300 "$@" > gpurun_out/${T}_$name.log 2>&1 || { echo "$name failed"; tail -5 gpurun_out/${T}_$name.log; exit 1; }; }
run threads_face ./scripts/bridgethreads 1000 own async face
run threads_face_shared ./scripts/bridgethreads 1000 shared async face
run threads_tiny_shared_direct ./scripts/bridgethreads 1000 shared async tiny direct
timeout -k 10 900 python3 scripts/ab.py --config cfg4 --rounds 3 --steps 15 --variants "${CFG4_VARIANTS:-spipe=0,spipe=1,spipe=256,spipe=512}" > gpurun_out/${T}_cfg4_ab.jsonl 2> gpurun_out/${T}_cfg4_ab.err || { tail -3 gpurun_out/${T}_cfg4_ab.err; exit 1; }
cut -c1-170 gpurun_out/${T}_cfg4_ab.jsonl
for f in threads_face threads_face_shared threads_tiny_shared_direct; do python3 -c "
import json,sys
for l in open('gpurun_out/${T}_$f.log'):
    d=json.loads(l); print(d['what'][:70], d['threads'], round(d['host_us_per_call']['mean'],2), round(d['device_us_per_op']['mean'],2), round(d['speedup_vs_1'],2))
"; done
