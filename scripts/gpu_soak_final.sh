# Final-build fuzz soak: every GPU fuzz test widened through its environment knob, one pytest process
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
DDT_FUZZ_SEEDS=1000 DDT_FUZZ_BIG_SEEDS=200 DDT_FUZZ_FRAG_TYPES=5000 DDT_FUZZ_OOO_SEEDS=300 \
DDT_FUZZ_EXT_TYPES=4000 DDT_FUZZ_PINNED_SEEDS=100 DDT_BRIDGE_FUZZ_SEEDS=200 \
  timeout -k 10 1000 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bridge.py -x -q -m gpu \
  -k "fuzz" --timeout 900 --timeout-method thread > gpurun_out/soak_final.log 2>&1
rc=$?; tail -3 gpurun_out/soak_final.log; exit $rc
