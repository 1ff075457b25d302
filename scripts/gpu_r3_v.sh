# Round 3 batch v: the engine's line-dense pack kernel vs lean kernels on config 5's descriptor
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 ./scripts/ubench_dense4 10 scripts/cfg5_item.bin > gpurun_out/r3v_ubench_dense4.log 2>&1 || exit $?
cat gpurun_out/r3v_ubench_dense4.log
