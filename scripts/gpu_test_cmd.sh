# GPU parity suite + smoke (one process each, each under its own time limit)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 700 python -m pytest tests -q -m gpu -x > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -5 gpurun_out/smoke.log; tail -25 gpurun_out/pytest_gpu.log; exit $rc
