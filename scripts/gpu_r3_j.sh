# Round 3 batch j: the line-dense LDS path -- parity suite, then A/B dense on/off (cfg5, cfg1, cfg2)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/r3j_pytest_gpu.log 2>&1
rc=$?; tail -6 gpurun_out/r3j_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
: > gpurun_out/r3j_dense_ab.jsonl
for c in cfg5 cfg1 cfg2 cfg3; do
  timeout -k 10 300 python3 scripts/ab.py --config $c --rounds 3 --steps 10 --mode pair --variants "dense=-1,dense=0" >> gpurun_out/r3j_dense_ab.jsonl 2>gpurun_out/r3j.err || exit $?
done
cut -c1-200 gpurun_out/r3j_dense_ab.jsonl
