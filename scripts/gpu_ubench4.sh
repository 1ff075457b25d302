# memory-request accounting for the x-face pattern (ubench4), one PMC pass per TCC group
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 ./scripts/ubench4 20 > gpurun_out/ubench4.log 2>&1 || exit $?
cat gpurun_out/ubench4.log
timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_BUBBLE_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_DRAM_sum --output-format csv -d gpurun_out/u4_rd -o pmc -- ./scripts/ubench4 2 > gpurun_out/u4_rd.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_WRREQ_DRAM_sum --output-format csv -d gpurun_out/u4_wr -o pmc -- ./scripts/ubench4 2 > gpurun_out/u4_wr.log 2>&1 || exit $?
find gpurun_out/u4_rd gpurun_out/u4_wr -name '*.csv' | head
