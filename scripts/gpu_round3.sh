# final evidence refresh: parity suite, rocprof trace/traffic/requests for every config,
# every config's bench line, the default bench line
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
for c in cfg2 cfg4 cfg3 cfg5 cfg1; do
  CFG=$c timeout -k 10 900 bash scripts/profile_round.sh > gpurun_out/profile_$c.log 2>&1 || { tail -20 gpurun_out/profile_$c.log; exit 1; }
  echo "profiled $c"
done
: > gpurun_out/bench_configs.jsonl
for c in cfg1 cfg2 cfg3 cfg4 cfg5; do
  timeout -k 10 400 python bench.py --config $c --steps 20 --warmup 3 >> gpurun_out/bench_configs.jsonl 2> gpurun_out/bench_$c.err || exit $?
done
timeout -k 10 400 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || exit $?
cut -c1-200 gpurun_out/bench_default.json
