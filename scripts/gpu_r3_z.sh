# Round 3 batch z: by-value single-item streaming kernel (ddt_affine1_kernel) on the y / z faces
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/r3z_ab_faces.jsonl
for f in y z; do
  timeout -k 10 400 python3 scripts/ab.py --config $f --count 512 --rounds 3 --steps 6 --mode pair --flush read --variants "afast=0,afast=3,afast=1" >> gpurun_out/r3z_ab_faces.jsonl 2>>gpurun_out/r3z.err || exit $?
done
cut -c1-220 gpurun_out/r3z_ab_faces.jsonl
timeout -k 10 600 python -u -m pytest tests/test_gpu_byvalue.py tests/test_gpu_dense.py -q -x --timeout 300 --timeout-method thread > gpurun_out/r3z_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r3z_pytest.log; exit $rc
