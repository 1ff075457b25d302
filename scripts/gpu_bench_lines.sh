# every config's bench line and the default line (reads profiles/requests_*.json, traffic_*.json)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
: > gpurun_out/bench_configs.jsonl
for c in cfg1 cfg2 cfg3 cfg4 cfg5; do
  timeout -k 10 400 python bench.py --config $c --steps 20 --warmup 3 >> gpurun_out/bench_configs.jsonl 2> gpurun_out/bench_$c.err || exit $?
done
timeout -k 10 400 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || exit $?
cut -c1-200 gpurun_out/bench_default.json
