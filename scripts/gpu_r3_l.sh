# Round 3 batch l: dense chunks per task, XCD mapping; halo interleave
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/r3l_ab.jsonl
timeout -k 10 300 python3 scripts/ab.py --config cfg5 --rounds 3 --steps 10 --mode pair --variants "dense=0,dense=1,dense=2,dense=4,dense=1;xcd=0,dense=4;xcd=0" >> gpurun_out/r3l_ab.jsonl 2>gpurun_out/r3l.err || exit $?
timeout -k 10 300 python3 scripts/ab.py --config cfg2 --rounds 3 --steps 20 --mode pair --variants "interleave=0,interleave=1,interleave=4,interleave=16,interleave=64" >> gpurun_out/r3l_ab.jsonl 2>>gpurun_out/r3l.err || exit $?
cut -c1-170 gpurun_out/r3l_ab.jsonl
