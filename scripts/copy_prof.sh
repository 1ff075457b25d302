#!/bin/bash
# Kernel time of the typed copy (scripts/copy_bench.py --only copy) per config, under
# rocprofv3 kernel trace + stats; then the wall-clock comparison with pack + unpack.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in cfg1 cfg2 cfg3 cfg5; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_copy_$c -o copy \
    -- python3 scripts/copy_bench.py --only copy --configs $c > gpurun_out/copy_only_$c.log 2>&1 || exit 1
  python3 scripts/kstats.py $(find gpurun_out/prof_copy_$c -name '*kernel_stats.csv') | grep ddt_move | head -2
done
timeout -k 10 300 python3 scripts/copy_bench.py > gpurun_out/copy_bench.jsonl || exit 1
