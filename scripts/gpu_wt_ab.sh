# write-through store policy A/B (ddt_tune wt) over every config, plus GPU parity
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
: > gpurun_out/wt_ab.log
for c in cfg2 xx yz cfg3 cfg1 cfg5 cfg4; do
  for m in pair; do
    timeout -k 10 300 python scripts/ab.py --config $c --mode $m --variants "wt=0,wt=1,wt=2" --rounds 3 >> gpurun_out/wt_ab.log 2>&1 || exit $?
  done
done
for c in cfg2 xx; do
  for m in pack unpack; do
    echo "mode=$m" >> gpurun_out/wt_ab.log
    timeout -k 10 300 python scripts/ab.py --config $c --mode $m --variants "wt=0,wt=1,wt=2" --rounds 3 >> gpurun_out/wt_ab.log 2>&1 || exit $?
  done
done
grep -h "mode\|variant" gpurun_out/wt_ab.log | cut -c1-140
