# x-face gather under every load cache policy: timing + memory-side request counters
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 ./scripts/ubench6 20 > gpurun_out/ubench6.log 2>&1 || exit $?
cat gpurun_out/ubench6.log
timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_BUBBLE_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_DRAM_sum --output-format csv -d gpurun_out/u6_rd -o pmc -- ./scripts/ubench6 2 > gpurun_out/u6_rd.log 2>&1 || exit $?
python3 scripts/reqs.py $(find gpurun_out/u6_rd -name '*counter_collection.csv') | grep -v rocclr
