#!/bin/bash
# rocprofv3 evidence for the per-face figure: one face type alone over 512 fields (beyond the
# Infinity Cache), kernel trace + stats per face, then FETCH_SIZE and WRITE_SIZE passes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1; shift; echo "== $name"; timeout -k 10 300 "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -n 1 gpurun_out/$name.log; [ $rc -eq 0 ] || exit $rc; }
for f in ${FACES:-x y z}; do
  run face_$f rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_face_$f -o face -- python3 scripts/faces.py --fields 512 --steps 10 --faces $f
  run face_fetch_$f rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcf_face_$f -o pmc -- python3 scripts/faces.py --fields 512 --steps 3 --faces $f
  run face_write_$f rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcw_face_$f -o pmc -- python3 scripts/faces.py --fields 512 --steps 3 --faces $f
  python3 scripts/traffic.py $(find gpurun_out/pmcf_face_$f -name '*counter_collection.csv') $(find gpurun_out/pmcw_face_$f -name '*counter_collection.csv') face_$f > gpurun_out/traffic_face_$f.json
done
echo done
