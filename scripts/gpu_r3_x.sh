# Round 3 batch x: by-value single-item line-dense kernel (ddt_dense1_kernel): microbenchmark,
# dense parity, cfg5 A/B (dfast), cfg4 pipelined pack 1 parity and A/B
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 ./scripts/ubench_dense4 10 scripts/cfg5_item.bin > gpurun_out/r3x_ubench_dense4.log 2>&1 || exit $?
tail -12 gpurun_out/r3x_ubench_dense4.log
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread -k "dense or cfg5 or cfg4 or sorted or fuzz" > gpurun_out/r3x_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r3x_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 scripts/ab.py --config cfg5 --rounds 3 --steps 6 --mode pair --variants "dfast=1,dfast=0,dfast=3" > gpurun_out/r3x_ab_cfg5.jsonl 2>gpurun_out/r3x.err || exit $?
timeout -k 10 400 python3 scripts/ab.py --config cfg4 --rounds 3 --steps 6 --mode pair --variants "spol=0,spol=64" > gpurun_out/r3x_ab_cfg4.jsonl 2>>gpurun_out/r3x.err || exit $?
cut -c1-250 gpurun_out/r3x_ab_cfg5.jsonl gpurun_out/r3x_ab_cfg4.jsonl
