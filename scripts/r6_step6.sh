#!/bin/bash
# Round-6 GPU step 6: chunk-major U for the address-ordered engine (ddt_tune slayout): the sorted
# parity tests, then config 4's A/B of the layouts, then a kernel trace of the chosen variant.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
T=${TAG:-r6q}
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -x -q -k "sorted_list_engine" --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { tail -30 gpurun_out/${T}_pytest.log; exit 1; }
tail -2 gpurun_out/${T}_pytest.log
timeout -k 10 900 python3 scripts/ab.py --config cfg4 --rounds 3 --steps 15 --variants "${CFG4_VARIANTS:-slayout=0,slayout=1,slayout=1;spol=4096,slayout=2,slayout=2;spol=4096,slayout=3}" > gpurun_out/${T}_cfg4_ab.jsonl 2> gpurun_out/${T}_cfg4_ab.err || { tail -3 gpurun_out/${T}_cfg4_ab.err; exit 1; }
cat gpurun_out/${T}_cfg4_ab.jsonl | cut -c1-200
[ -n "$TRACE" ] || exit 0
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof -o k -- python3 scripts/ab.py --config cfg4 --rounds 1 --steps 10 --variants "$TRACE" > gpurun_out/${T}_trace.log 2>&1 || { tail -5 gpurun_out/${T}_trace.log; exit 1; }
find gpurun_out/${T}_prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/${T}_kernel_stats.csv
cut -d, -f1-6 gpurun_out/${T}_kernel_stats.csv | head -12
