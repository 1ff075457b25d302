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


def _run_bench(args, timeout=300):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env["DDT_BENCH_BACKEND"] = "gloo"
    cmd = [sys.executable, os.path.join(ROOT, "bench.py")] + args + [
        "--no-faces", "--no-latency", "--no-cpu-baseline", "--no-graph"]
    p = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    return json.loads(lines[0])


def _check_per_rank(r, world):
    pr = r["per_rank_kernel_ms"]
    assert len(pr["ranks"]) == world
    for d, i in (("pack", 0), ("unpack", 1)):
        vals = [x[i] for x in pr["ranks"]]
        assert all(v > 0 for v in vals)
        assert pr[d]["min"] == min(vals) and pr[d]["max"] == max(vals)


def test_bench_world8_weak_cfg2(device):
    """The driver's `--gpus 8` command (weak cfg2, 16 fields per rank) rehearsed with eight ranks
    on the one GPU over gloo: eight shards gathered and checked, per-rank kernel times present."""
    r = _run_bench(["--gpus", "8", "--steps", "6", "--warmup", "2"])
    assert r["n_gpus"] == 8 and r["scaling"] == "weak"
    g = r["all_gather_check"]
    assert g["ok"] and g["backend"] == "gloo"
    assert g["gathered_bytes"] == 8 * r["config"]["packed_bytes_per_gpu"]
    assert abs(r["per_gpu_GiBs"] * 8 - r["value"]) < 1e-2
    _check_per_rank(r, 8)


def test_bench_world8_strong_cfg3(device):
    """`--gpus 8 --strong --config cfg3`: 64 fields of the 512^3 float subarray faces split by
    top-level count over eight ranks (8 each), the packed shards gathered = the whole message."""
    r = _run_bench(["--gpus", "8", "--strong", "--config", "cfg3", "--steps", "4", "--warmup", "1"])
    assert r["n_gpus"] == 8 and r["scaling"] == "strong"
    g = r["all_gather_check"]
    assert g["ok"] and g["backend"] == "gloo"
    # 64 fields x the face struct's packed size, in eight equal shards
    assert g["gathered_bytes"] == 8 * r["config"]["packed_bytes_per_gpu"]
    assert "64 instances" in r["config"]["parallelism"]
    _check_per_rank(r, 8)


def test_bench_world4_weak_cfg1(device):
    r = _run_bench(["--gpus", "4", "--config", "cfg1", "--steps", "6", "--warmup", "2"])
    assert r["n_gpus"] == 4
    assert r["all_gather_check"]["ok"]
    assert r["all_gather_check"]["gathered_bytes"] == 4 * r["config"]["packed_bytes_per_gpu"]
    _check_per_rank(r, 4)
