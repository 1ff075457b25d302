# quick GPU regression pass: host overhead, parity suite, default bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 ./scripts/hostbench > gpurun_out/hostbench.log 2>&1 || exit $?
cat gpurun_out/hostbench.log
timeout -k 10 700 python -m pytest tests -q -m gpu -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/bench_quick.log 2>&1 || exit $?
python - <<'PY'
import json
d = json.loads(open("gpurun_out/bench_quick.log").read().strip().splitlines()[-1])
print("value", d["value"], "kernel_ms", d["kernel_ms"], "frac", d["roofline"]["frac"], "lat", d.get("single_face_latency_us"))
PY
exit $rc
