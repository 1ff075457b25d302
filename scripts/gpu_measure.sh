#!/bin/bash
# A/B of tuning variants, bench of every config, profile of cfg2.  Stops on abnormal exit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
    local name=$1 t=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"
    tail -n 6 "gpurun_out/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "abnormal exit ($rc): stopping"; exit $rc; fi
    return 0
}
STEPS=${STEPS:-ab,bench,prof}
if [[ $STEPS == *ab* ]]; then
  step ab_nt 300 python scripts/ab.py --config cfg2 --variants "nt=-1,nt=0,nt=1" --rounds 3
  step ab_task 300 python scripts/ab.py --config cfg2 --variants "task_kb=0,task_kb=8,task_kb=16,task_kb=32,task_kb=64" --rounds 3
fi
if [[ $STEPS == *bench* ]]; then
  for c in ${CFGS:-cfg1 cfg2 cfg3 cfg4 cfg5}; do step bench_$c 400 python bench.py --config $c --steps 20 --warmup 3; done
fi
if [[ $STEPS == *prof* ]]; then
  step profile 1100 bash scripts/profile_round.sh
fi
echo "== done"
