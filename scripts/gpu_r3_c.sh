# Round 3 batch c: face ceilings with a cold clean cache, engine faces with read/write flush
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 ./scripts/ubench_face > gpurun_out/r3c_ubench_face.log 2>&1 &&
timeout -k 10 200 python3 scripts/faces.py --flush read > gpurun_out/r3c_faces_read.json 2>&1 &&
timeout -k 10 200 python3 scripts/faces.py --flush write --faces y,z > gpurun_out/r3c_faces_write.json 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3c_prof -o f -- python3 scripts/faces.py --faces y,z > gpurun_out/r3c_faces_prof.json 2>&1
rc=$?; cat gpurun_out/r3c_ubench_face.log gpurun_out/r3c_faces_read.json gpurun_out/r3c_faces_write.json; exit $rc
