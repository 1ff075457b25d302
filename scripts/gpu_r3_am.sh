# Round 3 batch am: x-face gather cache policies before a non-temporal scatter (scripts/ubench_xpol.hip)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 ./scripts/ubench_xpol > gpurun_out/r3am_ubench_xpol.log 2>&1 || exit $?
cat gpurun_out/r3am_ubench_xpol.log
