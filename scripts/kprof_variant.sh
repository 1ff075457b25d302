#!/bin/bash
# Per-kernel times of one engine variant: rocprofv3 kernel trace of scripts/ab.py with that
# variant alone.  Usage: scripts/kprof_variant.sh NAME CONFIG "k=v;k=v"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
name=$1; cfg=$2; var=$3
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kp_$name -o kp -- \
    python3 scripts/ab.py --config $cfg --variants "$var" --rounds 1 --steps 10 > gpurun_out/kp_$name.log 2>&1 || exit $?
python3 scripts/kstats.py $(find gpurun_out/kp_$name -name "*kernel_stats.csv") > gpurun_out/kp_$name.txt
cat gpurun_out/kp_$name.txt
