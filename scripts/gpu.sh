#!/bin/bash
# The one runner for GPU steps (run on the MI355X box through gpurun, from the repo root):
#
#   scripts/gpu.sh tests [pytest args]     GPU suite (default: all of tests/ -m gpu)
#   scripts/gpu.sh bench [bench.py args]   one bench line -> gpurun_out/$TAG_bench.json
#   scripts/gpu.sh configs                 bench line of every BASELINE config -> $TAG_configs.jsonl
#   scripts/gpu.sh prof [CFG]              rocprofv3 kernel stats + FETCH/WRITE passes (profile_round.sh)
#   scripts/gpu.sh ab [ab.py args]         A/B of engine tunables (scripts/ab.py) -> $TAG_ab.jsonl
#   scripts/gpu.sh ubench NAME [args]      a microbenchmark built here (scripts/NAME) -> $TAG_NAME.log
#
# Steps chain with &&: every step has its own time limit and a failing step ends the call.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r4}
step=$1
shift
case "$step" in
tests)
    [ $# -eq 0 ] && set -- tests
    timeout -k 10 1000 python -u -m pytest -q -m gpu -x --timeout 300 --timeout-method thread "$@" \
        > gpurun_out/${TAG}_pytest_gpu.log 2>&1
    rc=$?
    tail -25 gpurun_out/${TAG}_pytest_gpu.log
    exit $rc ;;
bench)
    timeout -k 10 600 python3 bench.py "$@" > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
    rc=$?
    tail -c 3000 gpurun_out/${TAG}_bench.json
    tail -5 gpurun_out/${TAG}_bench.err
    exit $rc ;;
configs)
    : > gpurun_out/${TAG}_configs.jsonl
    for c in cfg1 cfg2 cfg3 cfg4 cfg5; do
        timeout -k 10 400 python3 bench.py --config $c --steps 20 --warmup 3 --no-latency --no-faces "$@" \
            >> gpurun_out/${TAG}_configs.jsonl 2>> gpurun_out/${TAG}_configs.err || exit $?
    done
    cut -c1-400 gpurun_out/${TAG}_configs.jsonl ;;
prof)
    CFG=${1:-cfg2} TAG=$TAG bash scripts/profile_round.sh ;;
ab)
    timeout -k 10 900 python3 scripts/ab.py "$@" >> gpurun_out/${TAG}_ab.jsonl 2>> gpurun_out/${TAG}_ab.err
    rc=$?
    cut -c1-300 gpurun_out/${TAG}_ab.jsonl
    tail -3 gpurun_out/${TAG}_ab.err
    exit $rc ;;
ubench)
    name=$1
    shift
    timeout -k 10 300 ./scripts/$name "$@" > gpurun_out/${TAG}_$name.log 2>&1
    rc=$?
    cat gpurun_out/${TAG}_$name.log
    exit $rc ;;
*)
    echo "usage: scripts/gpu.sh tests|bench|configs|prof|ab|ubench ..." >&2
    exit 2 ;;
esac
