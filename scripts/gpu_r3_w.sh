# Round 3 batch w: lean one-chunk line-dense tasks (run_dense1): dense parity, then cfg5 A/B
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread -k "dense or cfg5 or fuzz" > gpurun_out/r3w_pytest_dense.log 2>&1
rc=$?; tail -3 gpurun_out/r3w_pytest_dense.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 scripts/ab.py --config cfg5 --rounds 3 --steps 6 --mode pair --variants "dense=-1,dense=-1;xcd=0,dense=2;dsplit=1,dense=1;dsplit=0;xcd=1" > gpurun_out/r3w_ab_cfg5.jsonl 2>gpurun_out/r3w.err || exit $?
cut -c1-250 gpurun_out/r3w_ab_cfg5.jsonl
