# Round 3 batch k: the line-dense LDS path v2 -- A/B dense on/off first, then the parity suite
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/r3k_dense_ab.jsonl
for c in cfg5 cfg1; do
  timeout -k 10 300 python3 scripts/ab.py --config $c --rounds 3 --steps 10 --mode pair --variants "dense=-1,dense=0" >> gpurun_out/r3k_dense_ab.jsonl 2>gpurun_out/r3k.err || exit $?
done
cut -c1-200 gpurun_out/r3k_dense_ab.jsonl
timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/r3k_pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/r3k_pytest_gpu.log; exit $rc
