"""GPU: the N-rank product path equals the 1-rank path.

tools/dist_check.py runs Worker.evaluate(lane_range="auto") + FiniteDifferences.step for 3 FD steps of a
HalfCheetah-shaped MujocoPolicy (96 antithetic directions, T = 200) once in one process and once as 2 ranks
(torch.distributed.run, gloo, both on cuda:0).  The z-score case exercises the one-collective moments form
(ONE all-reduce of [A | B | n | r' slots] per step), centred rank the all-gather + all-reduce form
(learner/finite_differences.py:24-64 in the reference).  Both ranks' theta must be bitwise equal (replicated
DSGD), and within 1e-6 of the single-process theta (the collective only changes the summation order)."""
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCRIPT = os.path.join(ROOT, "tools", "dist_check.py")

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("weighting,port,preset", [("zscore", 29541, "small"), ("centred_rank", 29542, "small"),
                                                   ("zscore", 29543, "bench"), ("zscore", 29544, "stale"),
                                                   ("centred_rank", 29545, "stale"), ("zscore", 29546, "uneven"),
                                                   ("centred_rank", 29547, "uneven")])
def test_two_rank_fd_steps_equal_one_rank(tmp_path, weighting, port, preset):
    """preset "bench" (VERDICT r3 item 6): bench.py's step at config 3 size -- 2 ranks x 2048 directions per rank
    x T = 1000, 2 FD steps, z-score through the one-collective [A | B | n | r' slots] all-reduce at its real size
    (2P + 1 + 8192 doubles), prefetched indices and step_async as in bench.py.  preset "stale" (VERDICT r3 missing
    3): lists of FDReturn with one-epoch-old returns (the drift-corrected lambda of finite_differences.py:66-92) on
    2 ranks equal the single-process delayed-return step.  preset "uneven" (ADVICE r4): lists split unevenly, one rank
    empty in two of the steps."""
    out = str(tmp_path)
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    p = subprocess.run([sys.executable, SCRIPT, "single", weighting, out, preset], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=180)
    assert p.returncode == 0, p.stderr[-2000:]
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), SCRIPT, "multi", weighting, out,
                        preset], cwd=ROOT, env=env, capture_output=True, text=True, timeout=180)
    assert p.returncode == 0, p.stderr[-2000:]
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    try:
        import dist_check
    finally:
        sys.path.pop(0)
    err = dist_check.compare(out)
    assert err <= 1e-6, err
    u1 = np.load(os.path.join(out, "upd_single.npy"))
    u0 = np.load(os.path.join(out, "upd_rank0.npy"))
    np.testing.assert_array_equal(u0, np.load(os.path.join(out, "upd_rank1.npy")))
    np.testing.assert_allclose(u0, u1, rtol=1e-6)
    assert np.all(u0 > 0)


@pytest.mark.parametrize("weighting,port", [("zscore", 29551), ("centred_rank", 29552)])
def test_rccl_one_rank_exchange_equals_single_process(tmp_path, weighting, port):
    """The exchange on RCCL (backend "nccl"): a one-rank process group with FDR_FORCE_COLLECTIVES=1 runs the
    sharded path -- count exchange and reward all-gathers, the one-collective moments all-reduce (z-score) or the
    gradient all-reduce (centred rank) -- through RCCL on the box's GPU, and must land where the single-process
    learner does (the moments form vs the direct z-score: rounding only)."""
    out = str(tmp_path)
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    p = subprocess.run([sys.executable, SCRIPT, "single", weighting, out], cwd=ROOT, env=env, capture_output=True,
                       text=True, timeout=180)
    assert p.returncode == 0, p.stderr[-2000:]
    env["FDR_FORCE_COLLECTIVES"] = "1"
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), SCRIPT, "nccl1", weighting, out],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=180)
    assert p.returncode == 0, p.stderr[-2000:]
    single = np.load(os.path.join(out, "theta_single.npy"))
    r0 = np.load(os.path.join(out, "theta_rank0.npy"))
    assert float(np.abs(r0 - single).max()) <= 1e-6
    np.testing.assert_allclose(np.load(os.path.join(out, "upd_rank0.npy")), np.load(os.path.join(out, "upd_single.npy")),
                               rtol=1e-6)
