# address-ordered list engine: parity tests, cfg4 A/B against the per-block kernel, kernel trace
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -q -m gpu -x -k sorted --timeout 120 --timeout-method thread > gpurun_out/pytest_sorted.log 2>&1 || { tail -40 gpurun_out/pytest_sorted.log; exit 1; }
tail -1 gpurun_out/pytest_sorted.log
timeout -k 10 400 python scripts/ab.py --config cfg4 --mode pair --variants "sorted=0,sorted=-1" --rounds 3 2>&1 | grep variant | cut -c1-160
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_cfg4 -o trace -- python3 bench.py --config cfg4 --steps 10 --warmup 2 --no-cpu-baseline --no-graph > gpurun_out/trace_cfg4.log 2>&1 || exit $?
python3 scripts/kstats.py gpurun_out/prof_cfg4/trace_kernel_stats.csv
