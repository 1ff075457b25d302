# Round 3 batch aj: x-face load policy x unpack store policy (nt x wt) in the pair loop
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/r3aj_ab_nt_wt.jsonl
for c in cfg2 cfg3 xx; do
  timeout -k 10 400 python3 scripts/ab.py --config $c --rounds 3 --steps 10 --mode pair --variants "nt=-1,nt=0,nt=0;wt=1,nt=0;wt=0,nt=-1;wt=1" >> gpurun_out/r3aj_ab_nt_wt.jsonl 2>>gpurun_out/r3aj.err || exit $?
done
cut -c1-200 gpurun_out/r3aj_ab_nt_wt.jsonl
