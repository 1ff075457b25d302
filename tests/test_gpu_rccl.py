"""The RCCL leg of SURVEY.md §8e executed on the one GPU the builder has.

The driver's 8-GPU run initialises torch.distributed with backend "nccl" (RCCL on ROCm), times
the packs, then all-gathers the packed shards over xGMI and checks them (bench.gather_check ->
ompi_amd.shard.gather_packed).  Here that exact code runs as a single-rank RCCL communicator on
cuda:0: bench.py with DDT_BENCH_PG=1 at world size 1, and gather_packed / gather_check on an
engine-packed cfg2 shard.  Both in child processes (a communicator per process, torn down with
it), under a timeout."""
from __future__ import annotations

import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import os, sys, json
sys.path.insert(0, os.environ["ROOT"])
import torch, torch.distributed as dist
import bench, ompi_amd
from ompi_amd import recipe as ER, shard
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", device_id=dev)
rec, _ = bench.halo_recipe()
t = ER.build_committed(rec)
info = t.info()
count = 2
span, origin = bench.layout(info, count)
user = torch.randint(1, 255, (span,), dtype=torch.uint8, device=dev)
S = info["size"] * count
packed = torch.empty(S, dtype=torch.uint8, device=dev)
assert ompi_amd.pack(user.data_ptr() + origin, count, t, packed, S, 0) == S
full = shard.gather_packed(packed)
torch.cuda.synchronize()
ok_full = bool(torch.equal(full, packed))
chk = bench.gather_check(packed, S, 1, 0, dev, "nccl")
print(json.dumps({"gathered": int(full.numel()), "ok_full": ok_full, "check": chk,
                  "backend": dist.get_backend()}))
dist.destroy_process_group()
"""


def _env(port):
    env = {k: v for k, v in os.environ.items() if k not in ("LOCAL_RANK", "DDT_BENCH_BACKEND")}
    env.update(ROOT=ROOT, RANK="0", WORLD_SIZE="1", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    return env


def test_rccl_gather_packed_single_rank(device):
    import bench
    p = subprocess.run([sys.executable, "-c", CHILD], env=_env(bench.free_port()), cwd=ROOT,
                       capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    r = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    assert r["backend"] == "nccl" and r["ok_full"]
    assert r["check"]["ok"] and r["check"]["backend"] == "nccl"
    assert r["gathered"] == r["check"]["gathered_bytes"] == 2 * 6 * 512 * 1024   # 2 fields x 6 faces


def test_bench_line_with_rccl_process_group(device):
    """bench.py itself with the RCCL process group at world size 1: init with device_id, the
    barrier-free timed region, the post-run all-gather check in the line."""
    import bench
    env = _env(bench.free_port())
    env["DDT_BENCH_PG"] = "1"
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--steps", "6", "--warmup", "2",
           "--no-faces", "--no-latency", "--no-cpu-baseline", "--no-graph", "--no-floor"]
    p = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    r = json.loads(lines[0])
    g = r["all_gather_check"]
    assert g["ok"] and g["backend"] == "nccl"
    assert g["gathered_bytes"] == r["config"]["packed_bytes_per_gpu"]
