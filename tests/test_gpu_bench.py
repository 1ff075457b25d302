"""bench.py's multi-rank path on the one-GPU box: `--gpus 2` run by hand starts its own two
ranks (torch.distributed.run as a child process), both on cuda:0 with the gloo backend
(RCCL needs one GPU per rank; the driver's 8-GPU node runs the nccl leg).  The JSON line must
report both ranks and the post-run all-gather check of the packed shards."""
from __future__ import annotations

import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_self_launches_two_ranks(device):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env["DDT_BENCH_BACKEND"] = "gloo"
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "6", "--warmup", "2",
           "--no-faces", "--no-latency", "--no-cpu-baseline", "--no-graph"]
    p = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    r = json.loads(lines[0])
    assert r["n_gpus"] == 2 and r["steps"] == 6
    assert r["all_gather_check"]["ok"] and r["all_gather_check"]["backend"] == "gloo"
    assert r["all_gather_check"]["gathered_bytes"] == 2 * r["config"]["packed_bytes_per_gpu"]
    assert abs(r["per_gpu_GiBs"] * 2 - r["value"]) < 1e-2 and r["aggregate_GiBs"] == r["value"]
