# Round 3: new position tests first, then the whole GPU suite (one process each, own limits)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_position.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3_pos.log 2>&1 &&
timeout -k 10 800 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/r3_pytest_gpu.log 2>&1
rc=$?; tail -30 gpurun_out/r3_pos.log; tail -15 gpurun_out/r3_pytest_gpu.log; exit $rc
