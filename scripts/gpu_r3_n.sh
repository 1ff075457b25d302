# Round 3 batch n: parity suite on the final build (dense only for records of several units),
# then cfg1 / cfg5 bench lines, the default line and its rocprof kernel stats
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/r3n_pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/r3n_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
: > gpurun_out/r3n_bench_configs.jsonl
for c in cfg1 cfg5; do
  timeout -k 10 400 python3 bench.py --config $c --steps 20 --warmup 3 --no-faces --no-latency >> gpurun_out/r3n_bench_configs.jsonl 2>>gpurun_out/r3n.err || exit $?
done
timeout -k 10 300 python3 -u bench.py > gpurun_out/r3n_bench_default.json 2>>gpurun_out/r3n.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3n_prof -o run -- python3 bench.py --no-faces --no-latency --no-cpu-baseline > gpurun_out/r3n_prof.log 2>&1 || exit $?
python3 - <<'PY'
import json
for l in open("gpurun_out/r3n_bench_configs.jsonl"):
    d = json.loads(l)
    print(d["config"]["config"], d["value"], d["kernel_ms"], d["roofline"]["frac"], (d.get("cpu_baseline") or {}).get("value"))
d = json.load(open("gpurun_out/r3n_bench_default.json"))
print("default", d["value"], d["ms_per_step"], d["kernel_ms"], d["roofline"]["frac"], d["faces"]["y"]["frac"], d["faces"]["z"]["frac"])
PY
