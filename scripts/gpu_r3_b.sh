# Round 3 batch b: new GPU tests, default bench line (flushed faces), face profiles
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_bench.py tests/test_gpu_baseline.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r3b_pytest.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r3b_bench.json 2> gpurun_out/r3b_bench.err &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r3b_prof_y -o y -- python3 scripts/faces.py --faces y > gpurun_out/r3b_faces_y.json 2>gpurun_out/r3b_faces_y.err &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r3b_prof_z -o z -- python3 scripts/faces.py --faces z > gpurun_out/r3b_faces_z.json 2>gpurun_out/r3b_faces_z.err
rc=$?; tail -12 gpurun_out/r3b_pytest.log; cat gpurun_out/r3b_bench.json | head -c 3000; echo; cat gpurun_out/r3b_faces_y.json gpurun_out/r3b_faces_z.json; exit $rc
