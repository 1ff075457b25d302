#!/bin/bash
# Round-6 GPU step 3: the default bench line, config 3's per-face line, the 8-rank rehearsal line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
T=${TAG:-r6l}
timeout -k 10 300 python3 bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
timeout -k 10 300 python3 bench.py --config cfg3 --steps 20 --warmup 3 --no-latency --no-cold > gpurun_out/${T}_bench_cfg3.json 2> gpurun_out/${T}_bench_cfg3.err || { tail -20 gpurun_out/${T}_bench_cfg3.err; exit 1; }
DDT_BENCH_BACKEND=gloo timeout -k 10 300 python3 bench.py --gpus 8 --steps 20 --warmup 3 --no-faces --no-latency --no-cpu-baseline --no-graph > gpurun_out/${T}_world8_gloo.json 2> gpurun_out/${T}_world8_gloo.err || { tail -20 gpurun_out/${T}_world8_gloo.err; exit 1; }
python3 - <<PY
import json
for f in ("bench", "bench_cfg3", "world8_gloo"):
    r = json.loads(open("gpurun_out/${T}_%s.json" % f).read().strip().splitlines()[-1])
    print(f, r["value"], r["ms_per_step"], r["roofline"]["frac"], r.get("build"), r.get("per_rank_kernel_ms"))
PY
run() { local name=$1; shift; timeout -k 10 300 "$@" > gpurun_out/${T}_$name.log 2>&1 || { echo "$name failed"; tail -5 gpurun_out/${T}_$name.log; exit 1; }; }
run threads_tiny ./scripts/bridgethreads 1000 own async tiny
run threads_tiny_shared ./scripts/bridgethreads 1000 shared async tiny
run threads_face ./scripts/bridgethreads 1000 own async face
run threads_face_shared ./scripts/bridgethreads 1000 shared async face
run threads_sync ./scripts/bridgethreads 500 own sync face
run threads_direct ./scripts/bridgethreads 1000 own async tiny direct
run threads_noslots ./scripts/bridgethreads 1000 own async tiny direct noslots
run hipthreads ./scripts/hipthreads 1000
[ -n "$PROF" ] || exit 0
CFG=cfg2 TAG=$T bash scripts/profile_round.sh > gpurun_out/${T}_prof_cfg2.log 2>&1 || { tail -5 gpurun_out/${T}_prof_cfg2.log; exit 1; }
CFG=cfg4 TAG=$T bash scripts/profile_round.sh > gpurun_out/${T}_prof_cfg4.log 2>&1 || { tail -5 gpurun_out/${T}_prof_cfg4.log; exit 1; }
CFG=cfg4 bash scripts/gpu_pmc.sh > gpurun_out/${T}_pmc_cfg4.log 2>&1 || { tail -5 gpurun_out/${T}_pmc_cfg4.log; exit 1; }
echo prof done
