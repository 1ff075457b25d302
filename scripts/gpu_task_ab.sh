# task size A/B for line-dense leaves under the XCD slab mapping
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/task_ab.log
V="xcd=-1,xcd=-1;task_kb=16,xcd=-1;task_kb=32,xcd=-1;task_kb=64,xcd=0;task_kb=32"
for c in cfg5 yz cfg1; do
  timeout -k 10 300 python scripts/ab.py --config $c --variants "$V" --rounds 5 --steps 20 >> gpurun_out/task_ab.log 2>&1 || { tail -20 gpurun_out/task_ab.log; exit 1; }
done
grep -v amdgpu.ids gpurun_out/task_ab.log | cut -c1-130
