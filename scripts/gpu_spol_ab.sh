# address-ordered engine access policy A/B (ddt_tune spol) on cfg4, pair loop
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -q -m gpu -x -k sorted --timeout 120 --timeout-method thread > gpurun_out/pytest_sorted.log 2>&1 || { tail -30 gpurun_out/pytest_sorted.log; exit 1; }
tail -1 gpurun_out/pytest_sorted.log
timeout -k 10 600 python scripts/ab.py --config cfg4 --mode pair --variants "spol=0,spol=1,spol=2,spol=4,spol=8,spol=6,spol=14,spol=15" --rounds 3 > gpurun_out/spol_ab.log 2>&1 || exit $?
grep variant gpurun_out/spol_ab.log | cut -c1-130
