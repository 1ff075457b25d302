# Round 3 batch ah: x-face gather loads plain vs non-temporal under round 3's non-temporal unpack
# stores (does a MALL-allocating gather turn the next unpack's partial writes into cache hits?)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/r3ah_ab_nt.jsonl
for c in cfg2 xx; do
  timeout -k 10 300 python3 scripts/ab.py --config $c --rounds 3 --steps 20 --mode pair --variants "nt=-1,nt=0" >> gpurun_out/r3ah_ab_nt.jsonl 2>>gpurun_out/r3ah.err || exit $?
done
cut -c1-230 gpurun_out/r3ah_ab_nt.jsonl
