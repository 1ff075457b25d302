# full-size BASELINE parity, RCCL init with device_id, 2-rank gloo rehearsal of bench.py
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_baseline.py -v -m gpu -x --timeout 300 --timeout-method thread --durations=0 > gpurun_out/pytest_baseline.log 2>&1 || { tail -40 gpurun_out/pytest_baseline.log; exit 1; }
tail -12 gpurun_out/pytest_baseline.log
MASTER_ADDR=127.0.0.1 MASTER_PORT=29531 RANK=0 WORLD_SIZE=1 timeout -k 10 120 python -c "
import torch, torch.distributed as dist
dev = torch.device('cuda', 0); torch.cuda.set_device(dev)
dist.init_process_group(backend='nccl', device_id=dev)
t = torch.tensor([3.0], device=dev, dtype=torch.float64); dist.all_reduce(t, op=dist.ReduceOp.MAX); dist.barrier()
print('rccl device_id init ok', t.item()); dist.destroy_process_group()
" > gpurun_out/rccl_init.log 2>&1 || { cat gpurun_out/rccl_init.log; exit 1; }
tail -1 gpurun_out/rccl_init.log
DDT_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --no-graph > gpurun_out/bench_n2_gloo.json 2> gpurun_out/bench_n2_gloo.err || { tail -20 gpurun_out/bench_n2_gloo.err; exit 1; }
cut -c1-300 gpurun_out/bench_n2_gloo.json
