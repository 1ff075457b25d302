# Round 3 batch i: the evidence for the bench line on the round-3 build -- default bench line,
# rocprofv3 kernel stats + FETCH/WRITE traffic + requests of cfg2, x-face scaling in both protocols
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u bench.py > gpurun_out/r3i_bench_default.json 2> gpurun_out/r3i_bench.err || exit $?
head -c 1500 gpurun_out/r3i_bench_default.json; echo
TAG=r3 CFG=cfg2 timeout -k 10 900 bash scripts/profile_round.sh || exit $?
timeout -k 10 300 python3 scripts/face_scaling.py 1,2,4,8,16,32,64,256 x none > gpurun_out/r3i_face_scaling_pair.log 2>&1 || exit $?
timeout -k 10 300 python3 scripts/face_scaling.py 1,2,4,8,16,32,64,256 x read > gpurun_out/r3i_face_scaling_cold.log 2>&1 || exit $?
grep -h '"fields": 16\|fit' gpurun_out/r3i_face_scaling_pair.log gpurun_out/r3i_face_scaling_cold.log
