# Round 3 batch ai: x-face gather loads plain vs non-temporal: cfg3 and cfg1 in the pair loop, and
# cfg2 / both x faces under the cold-clean protocol (1 GiB read before every operation)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/r3ai_ab_nt.jsonl
for c in cfg3 cfg1 cfg5; do
  timeout -k 10 300 python3 scripts/ab.py --config $c --rounds 3 --steps 10 --mode pair --variants "nt=-1,nt=0" >> gpurun_out/r3ai_ab_nt.jsonl 2>>gpurun_out/r3ai.err || exit $?
done
for c in cfg2 xx; do
  timeout -k 10 300 python3 scripts/ab.py --config $c --rounds 3 --steps 10 --mode pair --flush read --variants "nt=-1,nt=0" >> gpurun_out/r3ai_ab_nt.jsonl 2>>gpurun_out/r3ai.err || exit $?
done
cut -c1-230 gpurun_out/r3ai_ab_nt.jsonl
