#!/bin/bash
# Round-6 final GPU step on the final build.  PART=a: the whole -m gpu suite, smoke(), the
# driver's default bench line.  PART=b: every BASELINE config's line, rocprofv3 kernel stats and
# traffic of cfg2 / cfg4, cfg4's PMC groups.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r6f}
if [ "${PART:-a}" = a ]; then
    timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/${T}_pytest_gpu.log; exit 1; }
    tail -2 gpurun_out/${T}_pytest_gpu.log
    timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { tail -20 gpurun_out/${T}_smoke.log; exit 1; }
    tail -3 gpurun_out/${T}_smoke.log
    timeout -k 10 400 python3 bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
    cut -c1-600 gpurun_out/${T}_bench.json
    exit 0
fi
TAG=$T bash scripts/gpu.sh configs || exit 1
CFG=cfg2 TAG=$T bash scripts/profile_round.sh > gpurun_out/${T}_prof_cfg2.log 2>&1 || { tail -5 gpurun_out/${T}_prof_cfg2.log; exit 1; }
CFG=cfg4 TAG=$T bash scripts/profile_round.sh > gpurun_out/${T}_prof_cfg4.log 2>&1 || { tail -5 gpurun_out/${T}_prof_cfg4.log; exit 1; }
CFG=cfg4 bash scripts/gpu_pmc.sh > gpurun_out/${T}_pmc_cfg4.log 2>&1 || { tail -5 gpurun_out/${T}_pmc_cfg4.log; exit 1; }
echo prof done
