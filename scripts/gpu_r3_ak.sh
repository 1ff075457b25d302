# Round 3 batch ak: plain sparse gathers by default (use_nt): parity suite, every config's line,
# the default line, rocprofv3 kernel stats / traffic / requests of cfg2, cfg3, cfg5
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/r3ak_pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/r3ak_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
: > gpurun_out/r3ak_bench_configs.jsonl
for c in cfg1 cfg3 cfg4 cfg5; do
  timeout -k 10 400 python3 bench.py --config $c --steps 20 --warmup 3 --no-faces --no-latency >> gpurun_out/r3ak_bench_configs.jsonl 2>>gpurun_out/r3ak.err || exit $?
done
timeout -k 10 300 python3 -u bench.py > gpurun_out/r3ak_bench_default.json 2>>gpurun_out/r3ak.err || exit $?
for c in cfg2 cfg3 cfg5; do
  TAG=r3 CFG=$c timeout -k 10 900 bash scripts/profile_round.sh > gpurun_out/r3ak_profile_$c.log 2>&1 || exit $?
done
python3 - <<'PY'
import json
for l in open("gpurun_out/r3ak_bench_configs.jsonl"):
    d = json.loads(l)
    print(d["config"]["config"], d["value"], d["kernel_ms"], d["roofline"]["frac"], (d.get("cpu_baseline") or {}).get("value"))
d = json.load(open("gpurun_out/r3ak_bench_default.json"))
print("default", d["value"], d["ms_per_step"], d["kernel_ms"], d["roofline"]["frac"], d["faces"]["y"]["frac"], d["faces"]["z"]["frac"], d["faces"]["x"]["frac"])
PY
