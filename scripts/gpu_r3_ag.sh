# Round 3 batch ag: opal_ddt_api.c typed-copy known answer
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -k "copy_content" --timeout 120 --timeout-method thread > gpurun_out/r3ag_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r3ag_pytest.log; exit $rc
