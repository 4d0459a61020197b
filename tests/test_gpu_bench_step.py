"""GPU: the exact FD step bench.py times, at its own shape, against the oracle.

bench.py's fd_step (config 3): Worker.evaluate(2048 directions, antithetic, prefetch=True) -> ONE rollout launch of
4096 lanes x T = 1000 -> FiniteDifferences.step_async (fdr_fd_step: fused weights + gradient, then DSGD), with the
25 M-entry table, P = 6092, sigma = 0.02, lr = 0.01.  For 2 consecutive steps:
  * the lane indices are the reference's SharedNoiseTable stream (utils/noise_sources.py:44-47) drawn by the
    oracle's own table, and step 2's are the ones prefetched during step 1 (peek_batch);
  * sampled lanes' returns equal the oracle's episodes (worker/agent.py:20-71) with their global lane ids;
  * g equals the oracle's fd_gradient (learner/finite_differences.py:24-64) on the kernel's own returns
    (rel-L2 <= 1e-5), and theta the oracle's DSGD step (dsgd/dynamic_sgd.py:19-39) from the same theta:
    |d theta| <= 1e-6, ||d theta|| <= 1e-6 relative."""
import numpy as np
import pytest
import torch

from oracle import agent as oagent
from oracle import envs as oenvs
from oracle import learner as olearn
from oracle import noise as onoise

pytestmark = pytest.mark.gpu


def test_bench_fd_step_two_steps_match_oracle():
    from dsgd import DSGD
    from envs import SyntheticEnv
    from fdr import dist as fdist
    from learner import FiniteDifferences
    from policies import MujocoPolicy
    from utils import AdaptiveOmega, SharedNoiseTable
    from worker import Agent, Worker
    dev = torch.device("cuda", 0)
    torch.manual_seed(124)
    policy = MujocoPolicy(17, 6, seed=124, device=dev)
    P = policy.num_params
    T, n_dirs, sigma = 1000, 2048, 0.02
    env = SyntheticEnv.named("halfcheetah", device=dev, episode_len=T)
    table = SharedNoiseTable(25_000_000, P, random_seed=124)
    table.device_table(dev)
    agent = Agent(policy, env, random_seed=124)
    worker = Worker(policy, agent, table, None, sigma=sigma, random_seed=124)
    omega = AdaptiveOmega()
    dsgd = DSGD(policy.parameters(), lr=0.01)
    learner = FiniteDifferences(policy, dsgd, omega, table, noise_std=sigma)
    otab = onoise.NoiseTable(25_000_000, P, 124)
    lane_range = fdist.lane_range(n_dirs, 2, 1, 0)
    sign = np.tile(np.array([1, -1], np.int8), n_dirs)
    pick = np.array([0, 1, 2047, 4094, 4095])
    prefetched = None
    for step in range(2):
        theta0 = policy.get_trainable_flat().copy()
        seed = 1000 + step
        b = worker.evaluate(n_dirs, antithetic=True, lane_range=lane_range, seed=seed, prefetch=True)
        out = learner.step_async(b, 0.0, 0.0, 0.0)
        torch.cuda.synchronize()
        want = np.repeat(otab.sample_indices(n_dirs), 2)
        np.testing.assert_array_equal(b.idx_host, want)
        np.testing.assert_array_equal(b.sign_host, sign)
        if prefetched is not None:
            np.testing.assert_array_equal(b.idx_host, prefetched)
        prefetched = worker._next[1].copy()
        r = b.reward.cpu().numpy()
        # the returns that fed this step: sampled lanes against whole oracle episodes
        oenv = oenvs.BatchedSyntheticEnv(17, 6, False, T, len(pick))
        ref = oagent.evaluate_lanes("mujoco", 17, 6, theta0, otab.table, want[pick], sign[pick], sigma, oenv, seed,
                                    lane_ids=pick)[0]
        np.testing.assert_allclose(r[pick], ref, rtol=1e-4, atol=1e-4)
        # the learner on the kernel's own returns
        g_ref, _ = olearn.fd_gradient(otab.table, P, want, sign, r, 0.0, sigma)
        g = learner.gradient_memory.cpu().numpy()
        rel = np.linalg.norm(g - g_ref) / np.linalg.norm(g_ref)
        assert rel <= 1e-5, (step, rel)
        theta_ref, upd_ref = olearn.dsgd_step(theta0, g_ref, 0.01, omega.omega, omega.min_omega, omega.max_omega)
        theta1 = policy.get_trainable_flat()
        err = float(np.abs(theta1 - theta_ref).max())
        assert err <= 1e-6, (step, err)
        upd, gnorm = out.tolist()
        assert gnorm > 0 and abs(upd - upd_ref) <= 1e-6 * upd_ref, (step, upd, upd_ref)
        dn = np.linalg.norm((theta1 - theta0).astype(np.float64))
        assert abs(dn - upd_ref) <= 1e-6 * upd_ref, (step, dn, upd_ref)
