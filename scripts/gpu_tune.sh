#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
rc_ok() { [ $1 -eq 0 ] || [ $1 -eq 1 ]; }
if [ -z "$NOTEST" ]; then
timeout -k 10 600 python -m pytest tests -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -n 5 gpurun_out/pytest_gpu.log
rc_ok $rc || exit $rc
fi
for v in ${VARIANTS:-default}; do
  case $v in
    default) envs="";;
    nt) envs="DDT_NT=1";;
    t*) envs="DDT_TASK_KB=${v#t}";;
  esac
  env $envs timeout -k 10 300 python scripts/kbench.py ${KARGS} > gpurun_out/kbench_$v.log 2>&1; rc=$?
  echo "kbench $v rc=$rc"; grep -v amdgpu.ids gpurun_out/kbench_$v.log
  rc_ok $rc || exit $rc
done
if [ -n "$PROF" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kprof -o k -- python3 scripts/kbench.py --iters 5 ${KARGS} > gpurun_out/kprof.log 2>&1; rc=$?
  echo "prof rc=$rc"
fi
echo done
