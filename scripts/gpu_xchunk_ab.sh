# A/B of the XCD run length for slab items (ddt_tune "xchunk"), then the parity suite
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/xchunk_ab.log
V="xcd=0,xcd=-1,xcd=-1;xchunk=64,xcd=-1;xchunk=16,xcd=-1;xchunk=4"
for c in cfg5 yz cfg2; do
  timeout -k 10 300 python scripts/ab.py --config $c --variants "$V" --rounds 5 --steps 20 >> gpurun_out/xchunk_ab.log 2>&1 || { tail -20 gpurun_out/xchunk_ab.log; exit 1; }
done
echo "mode=pack" >> gpurun_out/xchunk_ab.log
timeout -k 10 300 python scripts/ab.py --config xx --mode pack --variants "xcd=0,xcd=1;xchunk=2,xcd=1;xchunk=4,xcd=1;xchunk=16" --rounds 5 >> gpurun_out/xchunk_ab.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/xchunk_ab.log | cut -c1-130
DDT_XCD=1 timeout -k 10 400 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_xcd1.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_xcd1.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_xcd1.log
