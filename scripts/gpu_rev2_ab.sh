# Infinity Cache reuse test: unpack in reverse order (timing only) x load policy
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
: > gpurun_out/rev2_ab.log
for c in xx cfg2; do
  for r in "" "--unpack-rev"; do
    echo "config=$c $r" >> gpurun_out/rev2_ab.log
    timeout -k 10 300 python scripts/ab.py --config $c $r --variants "nt=-1,nt=0,nt=-1;wt=0,nt=0;wt=0" --rounds 3 >> gpurun_out/rev2_ab.log 2>&1 || { tail -20 gpurun_out/rev2_ab.log; exit 1; }
  done
done
grep -v amdgpu.ids gpurun_out/rev2_ab.log | cut -c1-125
