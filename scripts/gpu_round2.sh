# refresh: parity suite, every config's bench line, cfg2/cfg4 rocprof evidence (trace, traffic, requests)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
CFG=cfg2 timeout -k 10 900 bash scripts/profile_round.sh || exit $?
CFG=cfg4 timeout -k 10 900 bash scripts/profile_round.sh || exit $?
: > gpurun_out/bench_configs.jsonl
for c in cfg1 cfg2 cfg3 cfg4 cfg5; do
  timeout -k 10 400 python bench.py --config $c --steps 20 --warmup 3 >> gpurun_out/bench_configs.jsonl 2> gpurun_out/bench_$c.err || exit $?
done
cut -c1-300 gpurun_out/bench_configs.jsonl
