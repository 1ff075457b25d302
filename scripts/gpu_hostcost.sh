# host cost per call + kernel-time regression check of the pointer-launch path
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 120 ./scripts/hostbench > gpurun_out/hostbench.log 2>&1 || exit $?
cat gpurun_out/hostbench.log
timeout -k 10 400 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
for c in cfg2 cfg1 cfg3; do
  timeout -k 10 300 python scripts/ab.py --config $c --mode pair --variants "nt=-1" --rounds 3 2>&1 | grep variant | cut -c1-120 || exit 1
done
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_quick.log 2>&1 || exit $?
cut -c1-400 gpurun_out/bench_quick.log | grep metric
