# Round 3 batch o: chunk-major U for the address-ordered engine (cfg4): parity, then A/B
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread -k "sorted or cfg4" > gpurun_out/r3o_pytest_sorted.log 2>&1
rc=$?; tail -3 gpurun_out/r3o_pytest_sorted.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 scripts/ab.py --config cfg4 --rounds 3 --steps 10 --mode pair --variants "scm=0,scm=1,scm=2,scm=3" > gpurun_out/r3o_ab_scm.jsonl 2>gpurun_out/r3o.err || exit $?
timeout -k 10 400 python3 scripts/ab.py --config cfg4 --rounds 2 --steps 10 --mode pair --variants "scm=0;spol=16,scm=3;spol=16,scm=0;spol=32,scm=3;spol=32,scm=0;spol=48,scm=3;spol=48" > gpurun_out/r3o_ab_scm_phases.jsonl 2>>gpurun_out/r3o.err || exit $?
cut -c1-250 gpurun_out/r3o_ab_scm.jsonl gpurun_out/r3o_ab_scm_phases.jsonl
