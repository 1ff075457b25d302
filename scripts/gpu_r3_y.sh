# Round 3 batch y: cfg4 pack phases, pipelined (spol 0) and one-workgroup-per-chunk (spol 64) pack 1:
# 16 skips the address-ordered gather, 32 the run emission (timing only, wrong bytes)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 scripts/ab.py --config cfg4 --rounds 3 --steps 6 --mode pack --variants "spol=0,spol=16,spol=32,spol=48,spol=64,spol=80,spol=96,spol=112" > gpurun_out/r3y_ab_cfg4_phases.jsonl 2>gpurun_out/r3y.err || exit $?
cut -c1-200 gpurun_out/r3y_ab_cfg4_phases.jsonl
