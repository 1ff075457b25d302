# Round 3 batch t: parity suite on the rebuilt tree (device-pool retry), default bench line
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/r3t_pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/r3t_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py > gpurun_out/r3t_bench_default.json 2>>gpurun_out/r3t.err || exit $?
cut -c1-400 gpurun_out/r3t_bench_default.json
