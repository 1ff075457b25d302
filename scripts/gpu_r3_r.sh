# Round 3 batch r: line-dense unpack as two workgroups per task (dsplit); dense parity tests
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread -k "dense or cfg5 or fuzz_full or pinned" > gpurun_out/r3r_pytest_dense.log 2>&1
rc=$?; tail -3 gpurun_out/r3r_pytest_dense.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 scripts/ab.py --config cfg5 --rounds 3 --steps 6 --mode pair --variants "dsplit=1,dsplit=0" > gpurun_out/r3r_ab_dsplit.jsonl 2>gpurun_out/r3r.err || exit $?
timeout -k 10 400 python3 scripts/ab.py --config cfg5 --rounds 2 --steps 6 --mode pair --flush read --variants "dsplit=1,dsplit=0" >> gpurun_out/r3r_ab_dsplit.jsonl 2>>gpurun_out/r3r.err || exit $?
cut -c1-220 gpurun_out/r3r_ab_dsplit.jsonl
