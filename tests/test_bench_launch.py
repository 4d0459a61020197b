"""CPU: bench.py's rank-count checks run before any GPU work.  Under an external launcher
--gpus must equal WORLD_SIZE; without one, --gpus N > 1 self-launches N ranks and must not ask for more GPUs
than are visible.  Every case here exits non-zero in the parent, before the HIP runtime starts."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, **env_extra):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "FDR_BENCH_REHEARSE")}
    env.update(env_extra)
    return subprocess.run([sys.executable, "bench.py", "--no-cpu-baseline"] + args, cwd=ROOT, env=env,
                          capture_output=True, text=True, timeout=180)


def test_gpus_disagrees_with_launcher_world_size():
    p = _run(["--gpus", "3"], WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    assert p.returncode != 0
    assert "disagrees with WORLD_SIZE=2" in p.stderr


def test_more_gpus_than_visible_exits_nonzero():
    p = _run(["--gpus", "512"])
    assert p.returncode != 0
    assert "512 GPU(s) requested" in p.stderr
    assert not [l for l in p.stdout.splitlines() if l.startswith("{")]


def test_launcher_world_larger_than_visible_exits_nonzero():
    p = _run([], WORLD_SIZE="512", RANK="0", LOCAL_RANK="0")
    assert p.returncode != 0
    assert "512 GPU(s) requested" in p.stderr


def test_invalid_gpu_counts():
    assert _run(["--gpus", "0"]).returncode != 0
    p = _run(["--gpus", "2", "--config", "trap"])
    assert p.returncode != 0 and "single-process" in p.stderr
