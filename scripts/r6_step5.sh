#!/bin/bash
# Round-6 GPU step 5: the whole GPU suite, thread scaling, config 3's faces at 256 fields.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
T=${TAG:-r6o}
timeout -k 10 900 python -u -m pytest -q -x -m gpu --timeout 300 --timeout-method thread tests > gpurun_out/${T}_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/${T}_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/${T}_pytest_gpu.log
run() { local name=$1; shift; timeout -k 10 300 "$@" > gpurun_out/${T}_$name.log 2>&1 || { echo "$name failed"; tail -5 gpurun_out/${T}_$name.log; exit 1; }; }
run threads_face ./scripts/bridgethreads 1000 own async face
run threads_face_shared ./scripts/bridgethreads 1000 shared async face
run threads_tiny ./scripts/bridgethreads 1000 own async tiny
run threads_tiny_shared ./scripts/bridgethreads 1000 shared async tiny
run threads_sync ./scripts/bridgethreads 500 own sync face
run hipthreads ./scripts/hipthreads 1000 0 4
timeout -k 10 400 python3 bench.py --config cfg3 --steps 20 --warmup 3 --no-latency --no-cold --no-cpu-baseline > gpurun_out/${T}_bench_cfg3.json 2> gpurun_out/${T}_bench_cfg3.err || { tail -5 gpurun_out/${T}_bench_cfg3.err; exit 1; }
for f in threads_face threads_face_shared threads_tiny threads_tiny_shared threads_sync; do python3 -c "
import json
for l in open('gpurun_out/${T}_$f.log'):
    d=json.loads(l); print(d['what'][:70], d['threads'], round(d['host_us_per_call']['mean'],2), round(d['device_us_per_op']['mean'],2), round(d['speedup_vs_1'],2))
"; done
python3 -c "
import json
r=json.loads(open('gpurun_out/${T}_bench_cfg3.json').read().strip().splitlines()[-1])
for k,v in r['faces'].items(): print(k, v)
"
