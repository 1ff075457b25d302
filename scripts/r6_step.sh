#!/bin/bash
# Round-6 GPU step: the suites touched this round, thread scaling, the 26-neighbour halo on this
# build and on the round-5 library (scratch_ab/r5, 8 inlined slots per direction), cfg4 A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
T=${TAG:-r6e}
timeout -k 10 600 python -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_gpu_sync.py tests/test_gpu_slots.py tests/test_gpu_parity.py -k "sync or slot or sorted" > gpurun_out/${T}_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/${T}_pytest.log; [ $rc -eq 0 ] || exit $rc
run() { local name=$1; shift; timeout -k 10 240 "$@" > gpurun_out/${T}_$name.log 2>&1 || { echo "$name failed"; tail -5 gpurun_out/${T}_$name.log; exit 1; }; }
run threads_own ./scripts/bridgethreads 2000 own
run threads_shared ./scripts/bridgethreads 2000 shared
run threads_sync ./scripts/bridgethreads 500 own sync
run hipthreads ./scripts/hipthreads 4000
run halo26 ./scripts/halo26 500 1 slots32
run halo26_off ./scripts/halo26 500 0 noslots
run halo26_r5 env LD_LIBRARY_PATH=$PWD/scratch_ab/r5 ./scripts/halo26 500 1 r5_slots8
run ldsprobe ./scripts/ldsprobe
run bridgecost ./scripts/bridgecost 2000
run bridgecost_r5 env LD_LIBRARY_PATH=$PWD/scratch_ab/r5 ./scripts/bridgecost 2000
timeout -k 10 900 python3 scripts/ab.py --config cfg4 --rounds 3 --steps 15 --variants "${CFG4_VARIANTS:-sskew=0;s2vec=0,sskew=4160,sskew=4160;spol=2,sskew=4160;sunroll=8,sskew=4160;spol=512}" > gpurun_out/${T}_cfg4_ab.jsonl 2> gpurun_out/${T}_cfg4_ab.err || { tail -3 gpurun_out/${T}_cfg4_ab.err; exit 1; }
cut -c1-160 gpurun_out/${T}_cfg4_ab.jsonl
