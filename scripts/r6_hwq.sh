#!/bin/bash
# Round-6: thread scaling against HIP's hardware-queue count (GPU_MAX_HW_QUEUES, 4 by default on the
# box): HIP's own argument-free launch and the drop-in's asynchronous face calls, 1-8 threads.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
: > gpurun_out/r6_hwq.jsonl
for q in 4 8 16; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 120 ./scripts/hipthreads 1000 0 1 > gpurun_out/hwq_hip_$q.log 2>&1 || { tail -5 gpurun_out/hwq_hip_$q.log; exit 1; }
    sed "s/^{/{\"hw_queues\": $q, /" gpurun_out/hwq_hip_$q.log | grep '^{' >> gpurun_out/r6_hwq.jsonl
    GPU_MAX_HW_QUEUES=$q timeout -k 10 120 ./scripts/bridgethreads 1000 own async face > gpurun_out/hwq_bridge_$q.log 2>&1 || { tail -5 gpurun_out/hwq_bridge_$q.log; exit 1; }
    sed "s/^{/{\"hw_queues\": $q, /" gpurun_out/hwq_bridge_$q.log | grep '^{' >> gpurun_out/r6_hwq.jsonl
done
cut -c1-260 gpurun_out/r6_hwq.jsonl
