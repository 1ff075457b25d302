# Round 3 batch p: address-ordered pack 1 with 32 elements per thread in flight (cfg4)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread -k "sorted" > gpurun_out/r3p_pytest_sorted.log 2>&1
rc=$?; tail -3 gpurun_out/r3p_pytest_sorted.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 scripts/ab.py --config cfg4 --rounds 3 --steps 10 --mode pair --variants "sunroll=16,sunroll=32,sunroll=32;spol=16,sunroll=16;spol=16" > gpurun_out/r3p_ab_sunroll.jsonl 2>gpurun_out/r3p.err || exit $?
cut -c1-250 gpurun_out/r3p_ab_sunroll.jsonl
timeout -k 10 400 python3 scripts/ab.py --config cfg5 --rounds 3 --steps 6 --mode pair --variants "wt=-1,wt=0,wt=1,wt=3" > gpurun_out/r3p_ab_cfg5_wt.jsonl 2>>gpurun_out/r3p.err || exit $?
cut -c1-250 gpurun_out/r3p_ab_cfg5_wt.jsonl
