#!/bin/bash
# One GPU session: smoke, GPU parity tests, bench, rocprof kernel stats.
# Stops at the first step that dies abnormally (timeout, abort, segfault); an ordinary
# test failure (exit 1) still lets the measurement steps run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {   # step <name> <timeout> <cmd...>
    local name=$1 t=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"
    tail -n 5 "gpurun_out/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
        echo "abnormal exit ($rc): stopping"; exit $rc
    fi
    return 0
}
STEPS=${STEPS:-smoke,pytest,bench,prof}
[[ $STEPS == *smoke* ]] && step smoke 400 python -c "import __graft_entry__ as g; g.smoke()"
[[ $STEPS == *pytest* ]] && step pytest_gpu 700 python -m pytest tests -q -m gpu -x
[[ $STEPS == *bench* ]] && step bench 400 python bench.py --steps 30 --warmup 5 --faces
[[ $STEPS == *prof* ]] && step prof 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline
echo "== done"
