# Round 3 batch s: full parity suite on the dsplit build, then rocprofv3 kernel stats, HBM
# traffic and request counts of cfg4 and cfg5 (the review asked for r3_cfg4_kernel_stats.csv
# and traffic_cfg4.json), and their bench lines
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/r3s_pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/r3s_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for c in cfg4 cfg5; do
  TAG=r3 CFG=$c timeout -k 10 900 bash scripts/profile_round.sh || exit $?
done
: > gpurun_out/r3s_bench_configs.jsonl
for c in cfg4 cfg5; do
  timeout -k 10 400 python3 bench.py --config $c --steps 20 --warmup 3 --no-faces --no-latency >> gpurun_out/r3s_bench_configs.jsonl 2>>gpurun_out/r3s.err || exit $?
done
cut -c1-300 gpurun_out/r3s_bench_configs.jsonl
