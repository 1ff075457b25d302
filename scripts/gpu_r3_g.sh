# Round 3 batch g: non-temporal unpack stores for isolated narrow blocks (wt=3) against
# write-through (wt=-1 auto = sc1) and plain (wt=0): pair loop and cold-clean protocol
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/r3g_wt.jsonl
for c in cfg2 xx cfg3 c3d2 cfg1; do
  for fl in none read; do
    timeout -k 10 300 python3 scripts/ab.py --config $c --rounds 3 --steps 20 --mode pair --flush $fl --variants "wt=-1,wt=3,wt=0" >> gpurun_out/r3g_wt.jsonl 2>gpurun_out/r3g.err || exit $?
  done
done
cut -c1-175 gpurun_out/r3g_wt.jsonl
