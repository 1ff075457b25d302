set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -m pytest tests -q -m gpu -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
for c in cfg2 cfg4 cfg5; do
  timeout -k 10 400 python bench.py --config $c --steps 20 --warmup 3 > gpurun_out/bench_$c.log 2>&1 || exit $?
  grep -h metric gpurun_out/bench_$c.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['config']['config'], d['value'], d['roofline']['frac'], d['roofline']['traffic'], json.dumps(d['cpu_baseline']))"
done
DDT_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 10 --warmup 2 > gpurun_out/bench_n2_rehearsal.log 2>&1
rc=$?; grep -h metric gpurun_out/bench_n2_rehearsal.log | cut -c1-400; exit $rc
