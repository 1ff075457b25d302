# where does the halo pack time go: direction-only loops and face subsets, one box
set -o pipefail
mkdir -p gpurun_out
A="timeout -k 10 300 python scripts/ab.py --variants policy=1 --rounds 3"
: > gpurun_out/ab_split.log
for c in cfg2 xx yz cfg3; do
  for m in pair pack unpack; do
    echo "mode=$m" >> gpurun_out/ab_split.log
    $A --config $c --mode $m >> gpurun_out/ab_split.log 2>&1 || exit $?
  done
done
grep -h "mode\|variant" gpurun_out/ab_split.log | cut -c1-150
