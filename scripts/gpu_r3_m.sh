# Round 3 batch m: parity suite on the final kernels, then the measurements DESIGN §6 quotes
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/r3m_pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/r3m_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 ./scripts/ubench_face write > gpurun_out/r3m_ubench_face_write.log 2>&1 || exit $?
: > gpurun_out/r3m_ab.jsonl
for c in cfg5 cfg1; do
  timeout -k 10 300 python3 scripts/ab.py --config $c --rounds 3 --steps 10 --mode pair --variants "dense=-1,dense=0" >> gpurun_out/r3m_ab.jsonl 2>gpurun_out/r3m.err || exit $?
done
: > gpurun_out/r3m_bench_configs.jsonl
for c in cfg1 cfg2 cfg3 cfg4 cfg5; do
  timeout -k 10 400 python3 bench.py --config $c --steps 20 --warmup 3 --no-faces --no-latency >> gpurun_out/r3m_bench_configs.jsonl 2>>gpurun_out/r3m.err || exit $?
done
timeout -k 10 400 python3 bench.py --config cfg3 --strong --steps 10 --warmup 2 --no-faces --no-latency --no-cpu-baseline >> gpurun_out/r3m_bench_configs.jsonl 2>>gpurun_out/r3m.err || exit $?
timeout -k 10 300 python3 -u bench.py > gpurun_out/r3m_bench_default.json 2>>gpurun_out/r3m.err || exit $?
cat gpurun_out/r3m_ubench_face_write.log; cut -c1-170 gpurun_out/r3m_ab.jsonl
python3 - <<'PY'
import json
for l in open("gpurun_out/r3m_bench_configs.jsonl"):
    d = json.loads(l)
    print(d["config"]["config"], d["scaling"], d["value"], d["kernel_ms"], d["roofline"]["frac"], (d.get("cpu_baseline") or {}).get("value"))
d = json.load(open("gpurun_out/r3m_bench_default.json"))
print("default", d["value"], d["ms_per_step"], d["kernel_ms"], d["roofline"]["frac"], d["faces"]["y"]["frac"], d["faces"]["z"]["frac"])
PY
