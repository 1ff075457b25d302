# GPU parity suite, then the headline rocprofv3 evidence (kernel stats, traffic, requests)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
CFG=cfg2 TAG=r2 bash scripts/profile_round.sh > gpurun_out/profile_cfg2_final.log 2>&1
rc=$?; tail -14 gpurun_out/profile_cfg2_final.log; exit $rc
