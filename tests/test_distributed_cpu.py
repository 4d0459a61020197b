"""N>1 path on CPU: world_size-2 gloo ranks run the engine's exchange protocol (fdr.dist) with the
oracle's arithmetic and must reproduce the single-process FD gradient."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from conftest import PKG, REPO


def test_lane_range_partitions_whole_directions():
    from fdr import dist as fdist
    for n_dirs in (1, 7, 64, 2048, 2049):
        for world in (1, 2, 3, 8):
            for lpd in (1, 2):
                covered = []
                for r in range(world):
                    lo, hi = fdist.lane_range(n_dirs, lpd, world, r)
                    assert lo % lpd == 0 and hi % lpd == 0
                    covered.extend(range(lo, hi))
                assert covered == list(range(n_dirs * lpd))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


# (P, directions): the small case, and BASELINE config 3 at N = 8 (8 ranks x 4096 lanes = 16384 directions,
# 32768 r' slots in the moments payload)
SIZES = {"small": (1000, 37), "bench8": (6092, 16384)}


def _rank_main(rank, world, port, out_dir, size="small"):
    sys.path[:0] = [REPO, PKG]
    import torch.distributed as dist
    from fdr import dist as fdist
    from oracle import learner as olearn
    from oracle import noise as onoise
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    (P, D), sigma = SIZES[size], 0.02
    t = onoise.NoiseTable(1 << 16, P, 5)
    idx = t.sample_indices(D)                        # every rank draws the full stream
    lidx = np.repeat(idx, 2)
    sign = np.tile(np.array([1, -1], np.int8), D)
    rewards = np.random.RandomState(3).randn(2 * D)  # "rollout" results, globally consistent
    lo, hi = fdist.lane_range(D, 2, world, rank)
    local = torch.as_tensor(rewards[lo:hi])
    r_all, lane_lo = fdist.gather_rewards(local)
    assert lane_lo == lo and np.array_equal(r_all.numpy(), rewards)
    # known split (Worker.evaluate's FDBatch.rank_lanes): one all-gather, no count exchange
    sizes = [b - a for a, b in (fdist.lane_range(D, 2, world, k) for k in range(world))]
    r_all2, lane_lo2 = fdist.gather_rewards(local, sizes=sizes)
    assert lane_lo2 == lo and np.array_equal(r_all2.numpy(), rewards)
    even = torch.as_tensor(rewards[:2 * world][2 * rank:2 * rank + 2])   # equal counts: no re-packing
    r_even, lo_even = fdist.gather_rewards(even, sizes=[2] * world)
    assert lo_even == 2 * rank and np.array_equal(r_even.numpy(), rewards[:2 * world])
    # coefficient of every local lane with the GLOBAL z-score, then the local partial gradient
    x = r_all.numpy() - 0.1
    m, s = x.mean(), x.std()
    z = (x - m) / s
    V, _ = olearn.perturbation_vectors(t.table, P, lidx[lo:hi], sign[lo:hi], sigma)
    g = torch.as_tensor(np.dot(z[lo:hi], V))
    fdist.allreduce_grad(g)
    np.save(os.path.join(out_dir, "g%d.npy" % rank), g.numpy())
    dist.destroy_process_group()


@pytest.mark.parametrize("world,size", [(2, "small"), (8, "small"), (8, "bench8")])
def test_two_rank_gradient_matches_single_process(tmp_path, world, size):
    port = _free_port()
    mp.spawn(_rank_main, args=(world, port, str(tmp_path), size), nprocs=world, join=True)
    from oracle import learner as olearn
    from oracle import noise as onoise
    P, D = SIZES[size]
    t = onoise.NoiseTable(1 << 16, P, 5)
    idx = t.sample_indices(D)
    lidx = np.repeat(idx, 2)
    sign = np.tile(np.array([1, -1], np.int8), D)
    rewards = np.random.RandomState(3).randn(2 * D)
    g_ref, _ = olearn.fd_gradient(t.table, P, lidx, sign, rewards, 0.1, 0.02)
    for r in range(world):
        g = np.load(os.path.join(str(tmp_path), "g%d.npy" % r))
        assert np.linalg.norm(g - g_ref) / np.linalg.norm(g_ref) < 1e-12
    # every rank holds the identical reduced gradient -> replicated DSGD stays in lock-step (theta bitwise)
    g0 = np.load(os.path.join(str(tmp_path), "g0.npy"))
    theta0 = olearn.dsgd_step(np.zeros(P, np.float32), g0, 0.01)[0]
    for r in range(1, world):
        gr = np.load(os.path.join(str(tmp_path), "g%d.npy" % r))
        assert np.array_equal(g0, gr)
        assert np.array_equal(olearn.dsgd_step(np.zeros(P, np.float32), gr, 0.01)[0], theta0)


def _moment_rewards(kind, n):
    rs = np.random.RandomState(3)
    if kind == "spread":
        return rs.randn(n) * 7 + 40                 # a mean far from 0
    # near-constant (CartPole at its cap + the +-1e-12 jiggle, worker/agent.py:69): |m| / sd ~ 4e13, where a
    # one-pass sum r'^2 / n - m^2 variance is rounding noise and r'_+ v - r'_- v products cancel
    return 500.0 + rs.choice([-1e-12, 1e-12], n)


def _rank_main_moments(rank, world, port, out_dir, kind, size="small"):
    """The one-collective z-score protocol (FiniteDifferences._step_batch, sharded): every rank reduces its lanes
    to [A | B | n_local | r' slots], ONE all-reduce sums them, g = (A - m B) / sd with m, sd over all r'."""
    sys.path[:0] = [REPO, PKG]
    import torch.distributed as dist
    from fdr import dist as fdist
    from oracle import learner as olearn
    from oracle import noise as onoise
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    (P, D), sigma = SIZES[size], 0.02
    t = onoise.NoiseTable(1 << 16, P, 5)
    idx = t.sample_indices(D)
    lidx = np.repeat(idx, 2)
    sign = np.tile(np.array([1, -1], np.int8), D)
    rewards = _moment_rewards(kind, 2 * D)
    lo, hi = fdist.lane_range(D, 2, world, rank)
    mom = torch.as_tensor(olearn.fd_moments(t.table, P, lidx[lo:hi], sign[lo:hi], rewards[lo:hi], 0.5, sigma,
                                            lane_lo=lo, n_all=2 * D, lanes_per_dir=2))
    fdist.allreduce_grad(mom)                                      # the step's only collective
    np.save(os.path.join(out_dir, "g%d.npy" % rank), olearn.grad_from_moments(mom.numpy(), P))
    dist.destroy_process_group()


@pytest.mark.parametrize("world,kind,size", [(2, "spread", "small"), (3, "spread", "small"),
                                            (2, "near_constant", "small"), (8, "spread", "bench8"),
                                            (8, "near_constant", "bench8")])
def test_one_collective_moments_gradient_matches_two_collective(tmp_path, world, kind, size):
    port = _free_port()
    mp.spawn(_rank_main_moments, args=(world, port, str(tmp_path), kind, size), nprocs=world, join=True)
    from oracle import learner as olearn
    from oracle import noise as onoise
    P, D = SIZES[size]
    t = onoise.NoiseTable(1 << 16, P, 5)
    idx = t.sample_indices(D)
    lidx = np.repeat(idx, 2)
    sign = np.tile(np.array([1, -1], np.int8), D)
    rewards = _moment_rewards(kind, 2 * D)
    g_ref, _ = olearn.fd_gradient(t.table, P, lidx, sign, rewards, 0.5, 0.02)   # all-gather + z-score form
    tol = 1e-12 if kind == "spread" else 1e-9
    gs = [np.load(os.path.join(str(tmp_path), "g%d.npy" % r)) for r in range(world)]
    for g in gs:
        assert np.linalg.norm(g - g_ref) / np.linalg.norm(g_ref) <= tol
        assert np.array_equal(g, gs[0])                            # replicated DSGD stays in lock-step
