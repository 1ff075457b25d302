# A/B of the XCD-aware workgroup->task mapping (ddt_tune "xcd"), parity with it on
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/xcd_ab.log
for c in cfg2 xx yz cfg3 cfg1 cfg5; do
  timeout -k 10 300 python scripts/ab.py --config $c --variants xcd=0,xcd=1,xcd=-1 --rounds 5 --steps 20 >> gpurun_out/xcd_ab.log 2>&1 || { tail -20 gpurun_out/xcd_ab.log; exit 1; }
done
for m in pack unpack; do
  echo "mode=$m" >> gpurun_out/xcd_ab.log
  timeout -k 10 300 python scripts/ab.py --config xx --mode $m --variants xcd=0,xcd=1,xcd=-1 --rounds 5 >> gpurun_out/xcd_ab.log 2>&1 || exit 1
done
cut -c1-140 gpurun_out/xcd_ab.log
timeout -k 10 400 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
DDT_XCD=1 timeout -k 10 400 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_xcd1.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_xcd1.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_xcd1.log
