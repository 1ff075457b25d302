# kernel durations of single-face launches (rocprofv3 kernel trace) beside their event times
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fprof -o fprof -- python3 scripts/face_scaling.py 1,16 y,x > gpurun_out/face_prof.log 2>&1 || { tail -20 gpurun_out/face_prof.log; exit 1; }
grep -v amdgpu.ids gpurun_out/face_prof.log | grep '^{'
f=$(find gpurun_out/fprof -name '*kernel_stats.csv' | head -1); cat "$f" | cut -c1-200
