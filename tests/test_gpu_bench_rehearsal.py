"""GPU: the N-rank bench path (bench.py under torch.distributed.run, 2 ranks) rehearsed on one GPU with gloo
(FDR_BENCH_REHEARSE=1): the lane sharding, the one-collective learner, the collective clock-settle decision
and the max-over-ranks timing must run to one JSON line.  The driver's 8-GPU scaling run uses the same code
with RCCL."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_bench_two_ranks_rehearsal():
    env = dict(os.environ, FDR_BENCH_REHEARSE="1", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29533", "bench.py", "--gpus", "2", "--steps", "2",
           "--warmup", "1", "--settle-ms", "10", "--timing-steps", "1", "--no-cpu-baseline", "--no-variant",
           "--perturbations", "512", "--episode-len", "50"]
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 2 and d["value"] > 0
    assert d["config"]["global_perturbations"] == 1024


@pytest.mark.gpu
def test_bench_self_launch_two_ranks():
    """`bench.py --gpus 2` with no external launcher starts the 2 ranks itself: one JSON
    line reporting n_gpus 2 / dp2 (gloo rehearsal: both ranks on cuda:0)."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["FDR_BENCH_REHEARSE"] = "1"
    cmd = [sys.executable, "bench.py", "--gpus", "2", "--steps", "2", "--warmup", "1", "--settle-ms", "10",
           "--timing-steps", "1", "--no-cpu-baseline", "--no-variant", "--perturbations", "512", "--episode-len", "50"]
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "dp2"
    assert d["config"]["global_perturbations"] == 1024 and d["value"] > 0
