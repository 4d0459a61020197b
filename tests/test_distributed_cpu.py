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


def _rank_main(rank, world, port, out_dir):
    sys.path[:0] = [REPO, PKG]
    import torch.distributed as dist
    from fdr import dist as fdist
    from oracle import learner as olearn
    from oracle import noise as onoise
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    P, D, sigma = 1000, 37, 0.02
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


@pytest.mark.parametrize("world", [2])
def test_two_rank_gradient_matches_single_process(tmp_path, world):
    port = _free_port()
    mp.spawn(_rank_main, args=(world, port, str(tmp_path)), nprocs=world, join=True)
    from oracle import learner as olearn
    from oracle import noise as onoise
    P, D = 1000, 37
    t = onoise.NoiseTable(1 << 16, P, 5)
    idx = t.sample_indices(D)
    lidx = np.repeat(idx, 2)
    sign = np.tile(np.array([1, -1], np.int8), D)
    rewards = np.random.RandomState(3).randn(2 * D)
    g_ref, _ = olearn.fd_gradient(t.table, P, lidx, sign, rewards, 0.1, 0.02)
    for r in range(world):
        g = np.load(os.path.join(str(tmp_path), "g%d.npy" % r))
        assert np.linalg.norm(g - g_ref) / np.linalg.norm(g_ref) < 1e-12
    # every rank holds the identical reduced gradient -> replicated DSGD stays in lock-step
    assert np.array_equal(np.load(os.path.join(str(tmp_path), "g0.npy")),
                          np.load(os.path.join(str(tmp_path), "g1.npy")))


def _rank_main_moments(rank, world, port, out_dir):
    """The one-collective z-score protocol (FiniteDifferences._step_batch, sharded): every rank reduces its lanes
    to [A | B | sum r' | sum r'^2 | n], ONE all-reduce sums them, g = (A - m B) / sd."""
    sys.path[:0] = [REPO, PKG]
    import torch.distributed as dist
    from fdr import dist as fdist
    from oracle import learner as olearn
    from oracle import noise as onoise
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    P, D, sigma = 1000, 37, 0.02
    t = onoise.NoiseTable(1 << 16, P, 5)
    idx = t.sample_indices(D)
    lidx = np.repeat(idx, 2)
    sign = np.tile(np.array([1, -1], np.int8), D)
    rewards = np.random.RandomState(3).randn(2 * D) * 7 + 40      # a mean far from 0: cancellation check
    lo, hi = fdist.lane_range(D, 2, world, rank)
    mom = torch.as_tensor(olearn.fd_moments(t.table, P, lidx[lo:hi], sign[lo:hi], rewards[lo:hi], 0.5, sigma))
    fdist.allreduce_grad(mom)                                      # the step's only collective
    np.save(os.path.join(out_dir, "g%d.npy" % rank), olearn.grad_from_moments(mom.numpy(), P))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_one_collective_moments_gradient_matches_two_collective(tmp_path, world):
    port = _free_port()
    mp.spawn(_rank_main_moments, args=(world, port, str(tmp_path)), nprocs=world, join=True)
    from oracle import learner as olearn
    from oracle import noise as onoise
    P, D = 1000, 37
    t = onoise.NoiseTable(1 << 16, P, 5)
    idx = t.sample_indices(D)
    lidx = np.repeat(idx, 2)
    sign = np.tile(np.array([1, -1], np.int8), D)
    rewards = np.random.RandomState(3).randn(2 * D) * 7 + 40
    g_ref, _ = olearn.fd_gradient(t.table, P, lidx, sign, rewards, 0.5, 0.02)   # all-gather + z-score form
    for r in range(world):
        g = np.load(os.path.join(str(tmp_path), "g%d.npy" % r))
        assert np.linalg.norm(g - g_ref) / np.linalg.norm(g_ref) <= 1e-12
