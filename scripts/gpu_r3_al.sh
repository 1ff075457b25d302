# Round 3 batch al: config 5 unpack with the destination lines loaded first (scripts/ubench_dense5.hip)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 ./scripts/ubench_dense5 10 > gpurun_out/r3al_ubench_dense5.log 2>&1 || exit $?
cat gpurun_out/r3al_ubench_dense5.log
