# Round 3 batch u: persistent line-dense pack shapes (scripts/ubench_dense3.hip)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 ./scripts/ubench_dense3 10 > gpurun_out/r3u_ubench_dense3.log 2>&1 || exit $?
cat gpurun_out/r3u_ubench_dense3.log
