#!/bin/bash
# rocprofv3 evidence for the bench line: kernel trace + stats, then HBM traffic counters
# in separate --pmc passes (FETCH_SIZE and WRITE_SIZE do not fit one pass on gfx950).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
CFG=${CFG:-cfg2}
TAG=${TAG:-r1}
run() { local name=$1; shift; echo "== $name"; timeout -k 10 400 "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -n 2 gpurun_out/$name.log; [ $rc -eq 0 ] || exit $rc; }
run trace_$CFG rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$CFG -o trace -- python3 bench.py --config $CFG --steps 20 --warmup 3 --no-cpu-baseline --no-graph --no-latency --no-faces --no-floor --no-cold
run fetch_$CFG rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcf_$CFG -o pmc -- python3 bench.py --config $CFG --steps 5 --warmup 1 --no-cpu-baseline --no-graph --no-latency --no-faces --no-floor --no-cold
run write_$CFG rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcw_$CFG -o pmc -- python3 bench.py --config $CFG --steps 5 --warmup 1 --no-cpu-baseline --no-graph --no-latency --no-faces --no-floor --no-cold
run req_$CFG rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum --output-format csv -d gpurun_out/pmcr_$CFG -o pmc -- python3 bench.py --config $CFG --steps 5 --warmup 1 --no-cpu-baseline --no-graph --no-latency --no-faces --no-floor --no-cold
python3 scripts/traffic.py $(find gpurun_out/pmcf_$CFG -name '*counter_collection.csv') $(find gpurun_out/pmcw_$CFG -name '*counter_collection.csv') $CFG > gpurun_out/traffic_$CFG.json
python3 scripts/requests.py $(find gpurun_out/pmcr_$CFG -name '*counter_collection.csv') $CFG > gpurun_out/requests_$CFG.json
python3 scripts/kstats.py $(find gpurun_out/prof_$CFG -name "*kernel_stats.csv") > gpurun_out/kstats_$CFG.txt; head -8 gpurun_out/kstats_$CFG.txt
if [ -n "$CALIB" ]; then
run calib_fetch rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcf_calib -o pmc -- python3 scripts/kbench.py --iters 3 --types z,x,cfg1
run calib_write rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcw_calib -o pmc -- python3 scripts/kbench.py --iters 3 --types z,x,cfg1
fi
echo done
