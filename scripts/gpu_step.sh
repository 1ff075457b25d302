#!/bin/bash
# Run GPU steps in order, each under its own time limit; stop at the first abnormal exit.
# usage: scripts/gpu_step.sh "name:seconds:command" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for spec in "$@"; do
    name=${spec%%:*}; rest=${spec#*:}; t=${rest%%:*}; cmd=${rest#*:}
    echo "== $name ($(date +%T)) $cmd"
    timeout -k 10 "$t" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
    rc=$?
    echo "== $name rc=$rc"
    grep -v amdgpu.ids "gpurun_out/$name.log" | tail -n 12
    if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
done
echo "== all steps ok"
