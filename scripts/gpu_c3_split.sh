# cfg3 face subsets, each direction alone and the pair
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
: > gpurun_out/c3_split.log
for c in c3d2 c3d1 c3d0 cfg3 xx; do
  for m in pair pack unpack; do
    echo "mode=$m" >> gpurun_out/c3_split.log
    timeout -k 10 300 python scripts/ab.py --config $c --mode $m --variants xcd=-1 --rounds 3 >> gpurun_out/c3_split.log 2>&1 || exit 1
  done
done
grep -h "mode\|variant" gpurun_out/c3_split.log | cut -c1-120
