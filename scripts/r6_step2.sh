#!/bin/bash
# Round-6 GPU step 2: thread scaling (face and tiny messages, own and shared types, sync), the
# default bench line, and config 3's per-face line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
T=${TAG:-r6f}
run() { local name=$1; shift; timeout -k 10 300 "$@" > gpurun_out/${T}_$name.log 2>&1 || { echo "$name failed"; tail -5 gpurun_out/${T}_$name.log; exit 1; }; }
timeout -k 10 300 python -u -m pytest -q -x --timeout 120 --timeout-method thread tests/test_gpu_sync.py tests/test_gpu_slots.py > gpurun_out/${T}_pytest.log 2>&1 || { tail -20 gpurun_out/${T}_pytest.log; exit 1; }
tail -1 gpurun_out/${T}_pytest.log
run threads_own ./scripts/bridgethreads 2000 own async face
run threads_shared ./scripts/bridgethreads 2000 shared async face
run threads_tiny ./scripts/bridgethreads 4000 own async tiny
run threads_tiny_shared ./scripts/bridgethreads 4000 shared async tiny
run threads_sync ./scripts/bridgethreads 500 own sync face
run hipthreads ./scripts/hipthreads 4000
run bench timeout -k 10 280 python3 bench.py
run bench_cfg3 timeout -k 10 280 python3 bench.py --config cfg3 --steps 20 --warmup 3 --no-latency --no-cold
python3 - <<'PY'
import json
for f in ("bench", "bench_cfg3"):
    r = json.loads(open(f"gpurun_out/${T}_{f}.log").read().strip().splitlines()[-1])
    print(f, r["value"], r["ms_per_step"], r["roofline"]["frac"], r.get("build"))
PY
