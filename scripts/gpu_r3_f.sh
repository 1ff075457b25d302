# Round 3 batch f: the x-face floor without the engine; face scaling in the pair loop and
# the cold-clean protocol
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 ./scripts/ubench_xpair > gpurun_out/r3f_ubench_xpair.log 2>&1 &&
timeout -k 10 300 python3 scripts/ab.py --config xx --rounds 3 --steps 20 --mode pair --flush none --variants "wt=-1,wt=0,nt=0" > gpurun_out/r3f_xx.jsonl 2>&1
rc=$?; cat gpurun_out/r3f_ubench_xpair.log; cut -c1-200 gpurun_out/r3f_xx.jsonl; exit $rc
