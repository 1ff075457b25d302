#!/bin/bash
# Counter calibration on the GPU box: scripts/calib (built here) timed alone,
# then one rocprofv3 --pmc pass per counter group, then scripts/calibrate.py.  Every pass under
# its own KILL timeout; a failed pass ends the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
L=${L:-4194304}
O=gpurun_out/calib_$L
rm -rf $O; mkdir -p $O
timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1
grep -o 'TCC_EA0_[A-Z0-9_]*' $O/counters.txt | sort -u > $O/tcc_ea0.txt
timeout -k 5 120 ./scripts/calib $L > $O/timing.jsonl || exit $?
pass() { local n=$1; shift; timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d $O/p_$n -o pmc -- ./scripts/calib $L > $O/p_$n.log 2>&1 || { echo "pass $n failed"; tail -3 $O/p_$n.log; exit 1; }; }
pass fetch FETCH_SIZE
pass write WRITE_SIZE
pass req TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum
if grep -q TCC_EA0_RDREQ_32B $O/tcc_ea0.txt; then pass req32 TCC_EA0_RDREQ_32B_sum; fi
pass hit TCC_HIT_sum TCC_MISS_sum
python3 scripts/calibrate.py $O/timing.jsonl $L $(find $O -name '*counter_collection.csv') > $O/calibration.json || exit 1
cat $O/timing.jsonl | cut -c1-120
