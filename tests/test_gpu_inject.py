"""GPU: fdr_rollout with host-injected draws (fdr_rollout_extras.u_inject)
replays the REFERENCE's own episodes of G7 directly -- no oracle in between.

G7 (tests/golden/make_golden.py g7_worker_synthetic) ran the reference's Worker.collect_returns(8)
(worker/worker.py:20-57 -> worker/agent.py:20-71) on the synthetic envs with the policies' action draws replaced by
a RandomState(31) stream: one f32 uniform per step for DiscretePolicy (inverse CDF), n_act f32 normals per step for
MujocoPolicy (mean + std z); eval episodes (worker rng RandomState(3), eval_prob 0.25) run deterministically and
draw nothing; the +-1e-12 jiggle comes from Agent.rng = RandomState(11), once per episode (agent.py:69).
Here the same streams feed ONE launch of 8 lanes (lane i = episode i, its training draws at u_inject[i]),
jiggle off in the kernel and added from the Agent stream: rewards and entropies must match G7 within 1e-4 rel."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

SHAPES = {"cartpole": ("discrete", 4, 2), "cheetah": ("mujoco", 17, 6)}


@pytest.mark.parametrize("name", ["cheetah", "cartpole"])
def test_injected_draws_replay_reference_episodes(golden, name):
    from envs import SyntheticEnv
    from fdr import engine
    from utils import SharedNoiseTable
    g = golden("g7_worker_synthetic.npz")
    kind, n_in, n_act = SHAPES[name]
    T = int(g[name + "_T"])
    theta = g[name + "_theta"]
    P = theta.size
    n = len(g[name + "_reward"])
    dev = torch.device("cuda", 0)
    tab = SharedNoiseTable(2 ** 22, P, random_seed=124)
    worker_rng, agent_rng, inj = np.random.RandomState(3), np.random.RandomState(11), np.random.RandomState(31)
    k = 1 if kind == "discrete" else n_act
    u = np.zeros((n, T, k), np.float32)
    idx = np.zeros(n, np.int64)
    sign = np.zeros(n, np.int8)
    jig = np.zeros(n)
    for i in range(n):
        is_eval = worker_rng.uniform(0, 1) < 0.25                       # worker.py:23
        assert is_eval == bool(g[name + "_is_eval"][i])
        if not is_eval:
            idx[i] = int(tab.sample_batch(1)[0])                          # worker.py:27
            assert idx[i] == g[name + "_idx"][i]
            sign[i] = 1
            for t in range(T):                                            # agent.py:43, one draw per step
                u[i, t] = np.float32(inj.uniform()) if kind == "discrete" else inj.randn(n_act).astype(np.float32)
        jig[i] = agent_rng.choice((-1e-12, 1e-12))                        # agent.py:69
    env = SyntheticEnv(n_in, n_act, kind == "discrete", T, env_seed=0, device=dev)
    spec = engine.PolicySpec(kind, n_in, n_act, P)
    lanes = engine.lanes_desc(torch.as_tensor(theta, device=dev), 0, tab.device_table(dev),
                              torch.as_tensor(idx, device=dev), torch.as_tensor(sign, device=dev), 0.02,
                              torch.as_tensor((sign == 0).astype(np.int8), device=dev))
    res = engine.rollout(spec, env, lanes, n, 99, jiggle=False, u_inject=torch.as_tensor(u, device=dev))
    torch.cuda.synchronize()
    ret = res.reward.cpu().numpy() + jig
    np.testing.assert_array_equal(res.timesteps.cpu().numpy(), g[name + "_timesteps"])
    np.testing.assert_allclose(ret, g[name + "_reward"], rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(res.entropy.cpu().numpy(), g[name + "_entropy"], rtol=1e-4, atol=1e-6)
    # the injected draws are what drove the training episodes: another stream changes their returns
    res2 = engine.rollout(spec, env, lanes, n, 99, jiggle=False, u_inject=torch.as_tensor(u[::-1].copy(), device=dev))
    r2 = res2.reward.cpu().numpy()
    assert not np.allclose(r2[sign == 1], res.reward.cpu().numpy()[sign == 1])
    np.testing.assert_array_equal(r2[sign == 0], res.reward.cpu().numpy()[sign == 0])


def test_injected_draws_shape_is_checked():
    from envs import SyntheticEnv
    from fdr import engine
    dev = torch.device("cuda", 0)
    theta = torch.zeros(6092, device=dev)
    env = SyntheticEnv(17, 6, False, 10, device=dev)
    spec = engine.PolicySpec("mujoco", 17, 6, 6092)
    lanes = engine.lanes_desc(theta, 0)
    with pytest.raises(ValueError):
        engine.rollout(spec, env, lanes, 2, 1, u_inject=torch.zeros(2, 10, 1, device=dev))
