# kernel trace + request counters of one bench config (CFG=cfg4 by default)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
CFG=${CFG:-cfg4}
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$CFG -o trace -- python3 bench.py --config $CFG --steps 10 --warmup 2 --no-cpu-baseline --no-graph > gpurun_out/trace_$CFG.log 2>&1 || exit $?
f=$(find gpurun_out/prof_$CFG -name '*kernel_stats.csv' | head -1); cut -d, -f1-8 "$f" | head -20
timeout -s KILL 200 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum --output-format csv -d gpurun_out/req_$CFG -o pmc -- python3 bench.py --config $CFG --steps 3 --warmup 1 --no-cpu-baseline --no-graph > gpurun_out/req_$CFG.log 2>&1 || exit $?
python3 scripts/reqs.py $(find gpurun_out/req_$CFG -name '*counter_collection.csv') | grep -v rocclr
