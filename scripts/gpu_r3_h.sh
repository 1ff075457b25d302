# Round 3 batch h: capture probe, lifetime tests, then the whole GPU suite on the pool build
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 ./scripts/probe_capture > gpurun_out/r3_probe_capture.log 2>&1
cat gpurun_out/r3_probe_capture.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_lifetime.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r3h_lifetime.log 2>&1
rc=$?; tail -30 gpurun_out/r3h_lifetime.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/r3h_pytest_gpu.log 2>&1
rc=$?; tail -15 gpurun_out/r3h_pytest_gpu.log; exit $rc
