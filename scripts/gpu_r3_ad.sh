# Round 3 batch ad: multi-rank rehearsal of bench.py's self-launched N = 4 and N = 8 path on the
# one-GPU box (gloo, ranks sharing the GPU: a code-path check of the driver's scaling command,
# not a scaling number)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/r3ad_rehearsal.jsonl
for n in 4 8; do
  DDT_BENCH_BACKEND=gloo timeout -k 10 300 python3 bench.py --gpus $n --steps 20 --warmup 3 --no-faces --no-latency >> gpurun_out/r3ad_rehearsal.jsonl 2>>gpurun_out/r3ad.err || exit $?
done
DDT_BENCH_BACKEND=gloo timeout -k 10 300 python3 bench.py --gpus 8 --config cfg3 --strong --steps 10 --warmup 2 --no-faces --no-latency >> gpurun_out/r3ad_rehearsal.jsonl 2>>gpurun_out/r3ad.err || exit $?
python3 - <<'PY'
import json
for l in open("gpurun_out/r3ad_rehearsal.jsonl"):
    assert l.startswith("{"), l[:200]
    d = json.loads(l)
    print(d["n_gpus"], d["config"]["config"], d["scaling"], d["value"], d["per_gpu_GiBs"], d["all_gather_check"])
PY
