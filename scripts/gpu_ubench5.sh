# random gather/scatter vs region size (ubench5) + x-face unpack-only A/B with the auto wt rule
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 200 ./scripts/ubench5 5 > gpurun_out/ubench5.log 2>&1 || exit $?
cat gpurun_out/ubench5.log
timeout -k 10 300 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python scripts/ab.py --config xx --mode unpack --variants "wt=-1,wt=0" --rounds 3 2>&1 | cut -c1-140
