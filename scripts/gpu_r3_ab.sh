# Round 3 batch ab: x-face access order (scripts/ubench_xorder.hip)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 ./scripts/ubench_xorder > gpurun_out/r3ab_ubench_xorder.log 2>&1 || exit $?
cat gpurun_out/r3ab_ubench_xorder.log
