# Round 3 batch af: opal_datatype_test.c restated (tests/test_gpu_opal_ddt_test.py), smoke, bench tests
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_opal_ddt_test.py -q --timeout 300 --timeout-method thread > gpurun_out/r3af_pytest.log 2>&1
rc=$?; tail -30 gpurun_out/r3af_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3af_smoke.log 2>&1 || exit $?
tail -1 gpurun_out/r3af_smoke.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench.py tests/test_gpu_shard.py -q -x --timeout 300 --timeout-method thread > gpurun_out/r3af_pytest_bench.log 2>&1
rc=$?; tail -3 gpurun_out/r3af_pytest_bench.log; exit $rc
