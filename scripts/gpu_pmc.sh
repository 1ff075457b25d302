#!/bin/bash
# PMC passes over one bench config (CFG, default cfg4): traffic, requests, wave-state and LDS
# counters, one rocprofv3 --pmc pass per group (slot limits: 8 SQ, 4 TCC), each under its own
# KILL timeout; then scripts/pmc_summary.py.  Output: gpurun_out/pmc_$CFG/summary.json.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
CFG=${CFG:-cfg4}
O=gpurun_out/pmc_$CFG
rm -rf $O; mkdir -p $O
B="python3 bench.py --config $CFG --steps 4 --warmup 1 --no-cpu-baseline --no-graph --no-latency --no-faces --no-floor --no-cold"
pass() { local n=$1; shift; timeout -s KILL 240 rocprofv3 --pmc "$@" --output-format csv -d $O/p_$n -o pmc -- $B > $O/p_$n.log 2>&1 || { echo "pass $n failed"; tail -3 $O/p_$n.log; exit 1; }; echo "pass $n ok"; }
pass fetch FETCH_SIZE
pass write WRITE_SIZE
pass req TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_128B_sum
pass hit TCC_HIT_sum TCC_MISS_sum
pass wave SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS
pass inst SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM
pass fifo SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_INST_LEVEL_VMEM SQ_LEVEL_WAVES SQ_WAVES SQ_BUSY_CU_CYCLES SQ_INST_CYCLES_VMEM_RD
python3 scripts/pmc_summary.py $(find $O -name '*counter_collection.csv') > $O/summary.json || exit 1
head -c 3000 $O/summary.json
