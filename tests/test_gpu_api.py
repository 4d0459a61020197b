"""The reference-shaped host API (policies / worker / learner / DSGD / runner) on the HIP path."""
import numpy as np
import pytest
import torch

from oracle import agent as oagent
from oracle import envs as oenvs
from oracle import learner as olearn
from oracle import noise as onoise

pytestmark = pytest.mark.gpu

SHAPES = {"trap": ("discrete", 2, 9), "cartpole": ("discrete", 4, 2), "cheetah": ("mujoco", 17, 6)}


def make_policy(kind, n_in, n_act, seed):
    from policies import DiscretePolicy, MujocoPolicy
    torch.manual_seed(seed)
    cls = DiscretePolicy if kind == "discrete" else MujocoPolicy
    return cls(n_in, n_act, seed=seed)


@pytest.mark.parametrize("name", list(SHAPES))
def test_policy_init_bit_exact_and_flat_api(golden, name):
    g = golden("g2_perturb.npz")
    kind, n_in, n_act = SHAPES[name]
    for seed in (124, 123):
        pol = make_policy(kind, n_in, n_act, seed)
        assert np.array_equal(pol.get_trainable_flat(), g["%s_s%d_theta" % (name, seed)])
    # parameters are views of the flat buffer
    first = next(pol.parameters())
    assert first.data_ptr() == pol.flat.data_ptr()
    x = pol.get_trainable_flat() * 2
    pol.set_trainable_flat(x)
    assert np.array_equal(pol.get_trainable_flat(), x)
    s = pol.serialize()
    pol.set_trainable_flat(np.zeros_like(x))
    pol.deserialize(s)
    assert np.array_equal(pol.get_trainable_flat(), x)


@pytest.mark.parametrize("name", list(SHAPES))
def test_policy_forward_api(golden, name):
    g = golden("g3_forward.npz")
    kind, n_in, n_act = SHAPES[name]
    pol = make_policy(kind, n_in, n_act, 124)
    t = onoise.NoiseTable(2 ** 22, pol.num_params, 124)
    pol.set_trainable_flat((t.decode(int(g[name + "_idx"])) * 0.1).astype(np.float32))
    x = g[name + "_x"]
    if kind == "discrete":
        np.testing.assert_allclose(pol.get_strategy(x), g[name + "_probs"], atol=1e-5)
        assert abs(pol.get_entropy(x) - float(g[name + "_entropy"])) < 1e-5
        assert [pol.get_action(x[i], deterministic=True) for i in range(8)] == list(g[name + "_argmax"])
        pol.compute_vbn(g[name + "_vbn_buf"])
        bm, bv = pol.bn_stats()
        ref_m = np.concatenate([g["%s_vbn_rm%d" % (name, i)] for i in range(3)])
        ref_v = np.concatenate([g["%s_vbn_rv%d" % (name, i)] for i in range(3)])
        np.testing.assert_allclose(bm.cpu().numpy(), ref_m, rtol=1e-5, atol=1e-5)
        np.testing.assert_allclose(bv.cpu().numpy(), ref_v, rtol=1e-5, atol=1e-5)
        np.testing.assert_allclose(pol.get_strategy(x), g[name + "_vbn_probs"], atol=1e-5)
    else:
        np.testing.assert_allclose(pol.get_strategy(x), np.concatenate([g[name + "_mean"], g[name + "_std"]], 1),
                                   atol=1e-5)
        assert abs(pol.get_entropy(x) - float(g[name + "_entropy"])) < 1e-5
        np.testing.assert_allclose(np.array([pol.get_action(x[i], True) for i in range(8)]),
                                   g[name + "_det_action"], atol=1e-5)


def test_noise_source_api(golden):
    from utils import SharedNoiseTable
    g = golden("g1_noise.npz")
    t = SharedNoiseTable(2 ** 22, 5197, random_seed=124)
    a = [int(t.sample()[0]) for _ in range(10)]
    b = list(t.sample_batch(54))
    assert a + b == list(g["s124_p5197_idx"])
    assert np.array_equal(t.decode(a[0]), t._table[a[0]:a[0] + 5197])
    dt = t.device_table()
    assert dt.is_cuda and dt.numel() == 2 ** 22


def _worker(kind, n_in, n_act, T, sigma=0.02, eval_prob=0.0, seed=3):
    from envs import SyntheticEnv
    from utils import SharedNoiseTable
    from worker import Agent, Worker
    pol = make_policy(kind, n_in, n_act, 124)
    env = SyntheticEnv(n_in, n_act, kind == "discrete", T)
    table = SharedNoiseTable(2 ** 22, pol.num_params, random_seed=124)
    agent = Agent(pol, env, random_seed=11)
    return pol, table, Worker(pol, agent, table, None, sigma=sigma, eval_prob=eval_prob, random_seed=seed)


def test_worker_evaluate_matches_oracle():
    pol, table, worker = _worker("mujoco", 17, 6, 120)
    theta = pol.get_trainable_flat()
    batch = worker.evaluate(24, antithetic=True, seed=77)
    assert len(batch) == 48 and batch.lanes_per_dir == 2
    idx = np.repeat(onoise.NoiseTable(2 ** 22, theta.size, 124).sample_indices(24), 2)
    assert np.array_equal(batch.idx_host, idx)
    ret, ent, steps, n2 = oagent.evaluate_lanes("mujoco", 17, 6, theta, table._table, idx, batch.sign_host, 0.02,
                                                oenvs.BatchedSyntheticEnv(17, 6, False, 120, 48), 77)
    np.testing.assert_allclose(batch.reward.cpu().numpy(), ret, rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(batch.norm2.cpu().numpy(), n2, rtol=1e-9)


def test_collect_returns_api():
    pol, table, worker = _worker("discrete", 4, 2, 50, eval_prob=0.3, seed=5)
    rets = worker.collect_returns(16)
    rng = np.random.RandomState(5)
    is_eval = [rng.uniform(0, 1) < 0.3 for _ in range(16)]
    assert [r.is_eval for r in rets] == is_eval
    assert all(r.timesteps == 50 for r in rets)
    ref_idx = onoise.NoiseTable(2 ** 22, pol.num_params, 124).sample_indices(16 - sum(is_eval))
    assert [int(r.encoded_noise) for r in rets if not r.is_eval] == list(ref_idx)
    assert all(r.norm2 == 0 for r in rets if r.is_eval)


@pytest.mark.parametrize("case", ["cheetah_n16", "trap_n16"])
def test_learner_step_list_api_vs_reference(golden, case):
    """FiniteDifferences.step(list[FDReturn]) + DSGD through the product API vs the reference."""
    from dsgd import DSGD
    from learner import FDReturn, FiniteDifferences
    from utils import AdaptiveOmega, SharedNoiseTable
    g = golden("g4_fd_step.npz")
    name = case.split("_")[0]
    kind, n_in, n_act = SHAPES[name]
    pol = make_policy(kind, n_in, n_act, 124)
    assert np.array_equal(pol.get_trainable_flat(), g[case + "_theta0"])
    table = SharedNoiseTable(2 ** 22, pol.num_params, random_seed=124)
    omega = AdaptiveOmega()
    omega.omega = float(g[case + "_omega"])
    L = FiniteDifferences(pol, DSGD(pol.parameters(), lr=0.01), omega, table, noise_std=0.02)
    rets = []
    for i, r in enumerate(g[case + "_rewards"]):
        x = FDReturn()
        x.epoch = 0
        x.encoded_noise = table.sample()[0]
        x.reward = float(r)
        rets.append(x)
    upd = L.step(rets, 0.25, 0, 0)
    gref = g[case + "_g"]
    assert np.linalg.norm(L.gradient_memory.cpu().numpy() - gref) / np.linalg.norm(gref) < 1e-5
    np.testing.assert_allclose(pol.get_trainable_flat(), g[case + "_theta1"], rtol=0, atol=1e-6)
    assert abs(upd - float(g[case + "_update"])) < 1e-5
    # second step: half the returns one epoch stale (lambda drift path)
    rets = []
    for i, r in enumerate(g[case + "_rewards2"]):
        x = FDReturn()
        x.epoch = int(g[case + "_ep2"][i])
        x.encoded_noise = table.sample()[0]
        x.reward = float(r)
        rets.append(x)
    upd2 = L.step(rets, -0.5, 0, 0)
    gref = g[case + "_g2"]
    assert np.linalg.norm(L.gradient_memory.cpu().numpy() - gref) / np.linalg.norm(gref) < 1e-4
    np.testing.assert_allclose(pol.get_trainable_flat(), g[case + "_theta2"], rtol=0, atol=1e-6)
    assert abs(upd2 - float(g[case + "_update2"])) < 1e-5


def test_dsgd_optimizer_api():
    from dsgd import DSGD
    pol = make_policy("mujoco", 17, 6, 124)
    theta = pol.get_trainable_flat()
    opt = DSGD(pol.parameters(), lr=0.01)
    grad = np.random.RandomState(0).randn(theta.size)
    opt.zero_grad()
    pol.set_grad_from_flat(-grad)
    opt.step()
    ref, _ = olearn.dsgd_step(theta, grad, 0.01, 1.0, 0.0, 1.0, 1.0, 1.0)   # lr_scale = 1 (no adjust_lr)
    np.testing.assert_allclose(pol.get_trainable_flat(), ref, rtol=0, atol=1e-6)


def test_sequential_runner_trap(golden):
    from run_sequential import SequentialRunner
    g = golden("g6_runner_trap.npz")
    r = SequentialRunner(env_id="SimpleTrapEnv-v0", batch_size=16, random_seed=124, zeta_size=4,
                         max_strategy_history_size=4, noise_table_size=2 ** 22, verbose=False)
    assert np.array_equal(r.policy.get_trainable_flat(), g["theta0"])
    r.train(2)
    assert len(r.history) == 2
    # index stream and eval-coin schedule are the reference's
    assert np.array_equal(r.history[0]["idx"], g["e0_idx"])
    assert np.array_equal(r.history[1]["idx"], g["e1_idx"])
    assert abs(r.history[0]["Update Magnitude"] - g["update_magnitude_printed"][0]) < 1e-4
    assert all(float(x) == round(float(x)) for x in np.round(r.history[0]["rewards"], 6))  # integer trap rewards


def test_sequential_runner_antithetic_cheetah():
    from run_sequential import SequentialRunner
    r = SequentialRunner(env_id="HalfCheetah-v4", batch_size=64, random_seed=7, antithetic=True, episode_len=100,
                         noise_table_size=2 ** 22, verbose=False, eval_prob=0.1)
    r.train(3)
    assert len(r.history) == 3
    for h in r.history:
        assert np.isfinite(h["Noisy Reward"]) and h["Update Magnitude"] > 0


def test_compute_vbn_on_device_vs_torch_train_mode():
    """fdr_bn_refresh == one train-mode torch pass of the DiscretePolicy (policies/policy.py:31-34)."""
    import torch.nn as nn
    from policies import DiscretePolicy
    from oracle import policies as opol
    torch.manual_seed(124)
    pol = DiscretePolicy(4, 2, seed=124)
    ref = opol.TorchPolicy("discrete", 4, 2, seed=124)
    ref.set_flat(pol.get_trainable_flat())
    buf = (np.random.RandomState(3).randn(500, 4) * 2 + 0.5).astype(np.float32)
    for _ in range(2):                      # twice: the second pass starts from refreshed stats
        pol.compute_vbn(buf)
        ref.model.train()
        with torch.no_grad():
            ref.model(torch.as_tensor(buf))
        ref.model.eval()
    got = [m for m in pol.model if isinstance(m, nn.BatchNorm1d)]
    want = [m for m in ref.model if isinstance(m, nn.BatchNorm1d)]
    for g, w in zip(got, want):
        np.testing.assert_allclose(g.running_mean.cpu().numpy(), w.running_mean.numpy(), rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(g.running_var.cpu().numpy(), w.running_var.numpy(), rtol=1e-5, atol=1e-6)


def test_sequential_runner_trap_vs_oracle_runner():
    """The product SequentialRunner (batched GPU episodes, counter action stream) against the oracle's restated
    runner driven by the same stream (oracle/runner.py counter_seed): index streams and eval schedule equal,
    every epoch's (integer) trap returns equal up to the +-1e-12 jiggle, the final theta within 1e-6."""
    from run_sequential import SequentialRunner
    from oracle import runner as orunner
    r = SequentialRunner(env_id="SimpleTrapEnv-v0", batch_size=16, random_seed=124, zeta_size=4, eval_prob=0.2,
                         max_strategy_history_size=4, noise_table_size=2 ** 22, verbose=False)
    r.train(2)
    ref = orunner.run_trap(2, batch_size=16, seed=124, eval_prob=0.2, zeta_size=4, counter_seed=True)
    assert len(r.history) == 2
    for e in range(2):
        np.testing.assert_array_equal(r.history[e]["idx"], ref["log"][e]["idx"])
        np.testing.assert_allclose(r.history[e]["rewards"], ref["log"][e]["rewards"], rtol=0, atol=1e-9)
        assert abs(r.history[e]["Update Magnitude"] - ref["log"][e]["update"]) < 1e-5
    assert np.unique(np.round(np.concatenate([h["rewards"] for h in r.history]))).size > 1   # returns vary
    np.testing.assert_allclose(r.policy.get_trainable_flat(), ref["theta"], rtol=0, atol=1e-6)
    assert abs(r.policy_reward - ref["policy_reward"]) < 1e-9
