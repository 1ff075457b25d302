# Round 3 batch q: cfg5 -- non-temporal user stores in the line-dense unpack, and where the
# pack's time goes (pack-only / unpack-only / pair loops)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 scripts/ab.py --config cfg5 --rounds 3 --steps 6 --mode pair --variants "wt=-1,wt=3" > gpurun_out/r3q_ab_cfg5.jsonl 2>gpurun_out/r3q.err || exit $?
timeout -k 10 400 python3 scripts/ab.py --config cfg5 --rounds 2 --steps 6 --mode pack --variants "wt=-1" >> gpurun_out/r3q_ab_cfg5.jsonl 2>>gpurun_out/r3q.err || exit $?
timeout -k 10 400 python3 scripts/ab.py --config cfg5 --rounds 2 --steps 6 --mode unpack --variants "wt=-1,wt=3" >> gpurun_out/r3q_ab_cfg5.jsonl 2>>gpurun_out/r3q.err || exit $?
timeout -k 10 400 python3 scripts/ab.py --config cfg5 --rounds 2 --steps 6 --mode pair --flush read --variants "wt=-1,wt=3" >> gpurun_out/r3q_ab_cfg5.jsonl 2>>gpurun_out/r3q.err || exit $?
timeout -k 10 100 ./scripts/ubench_dense2 10 > gpurun_out/r3q_ubench_dense2.log 2>&1 || exit $?
cut -c1-200 gpurun_out/r3q_ab_cfg5.jsonl; cat gpurun_out/r3q_ubench_dense2.log
