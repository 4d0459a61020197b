"""GPU: the reference runner's DEFAULT noise source (run_sequential.py:89, RNGNoiseSource) on
the device path, against G15 (tests/golden/g15_rng_noise_source.npz): the reference's Worker.collect_returns +
FiniteDifferences.step over two epochs with one shared RNGNoiseSource (SURVEY finding-3 patch: bit_generator.state)
and injected action draws (as G7).

A host noise source has no table to gather from: each lane's theta' = fl32(theta + sigma * noise) is formed on the
host in the reference's f64 arithmetic (worker.py:28) and handed to the kernels as a row (fdr_lanes_desc.base_stride
= P, utils/noise_sources.py HostNoiseRows); the learner gathers lambda = fl32(sigma fl32(noise)) from the fl32 noise
rows that decode() regenerates.  Tolerances: returns / entropies <= 1e-4 rel (as G7), theta <= 1e-6 abs, the
gradient rel-L2 <= 1e-5 (f32 noise rows against the reference's f64 vectors)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

SHAPES = {"cartpole": ("discrete", 4, 2), "cheetah": ("mujoco", 17, 6)}


def _stream(g, name):
    """The reference's draws in order: worker eval coins (RandomState(3)), RNGNoiseSource(P, 5) samples, the injected
    action stream (RandomState(31)) and the Agent's jiggle (RandomState(11)), over both epochs."""
    from utils.noise_sources import RNGNoiseSource
    kind, n_in, n_act = SHAPES[name]
    T = int(g[name + "_T"])
    P = g[name + "_theta0"].size
    src = RNGNoiseSource(P, random_seed=5)
    wr, ar, inj = np.random.RandomState(3), np.random.RandomState(11), np.random.RandomState(31)
    k = 1 if kind == "discrete" else n_act
    out = []
    for e in range(2):
        n = len(g["%s_e%d_reward" % (name, e)])
        ev, enc, noises, jig = [], [], [], []
        u = np.zeros((n, T, k), np.float32)
        for i in range(n):
            is_eval = wr.uniform(0, 1) < 0.25
            ev.append(is_eval)
            if not is_eval:
                s, z = src.sample()
                enc.append(s)
                noises.append(z)
                for t in range(T):
                    u[i, t] = np.float32(inj.uniform()) if kind == "discrete" else inj.randn(n_act).astype(np.float32)
            else:
                enc.append("0")
            jig.append(ar.choice((-1e-12, 1e-12)))
        out.append(dict(is_eval=np.array(ev), enc=enc, noises=noises, u=u, jig=np.array(jig)))
    return out


@pytest.mark.parametrize("name", ["cheetah", "cartpole"])
def test_rng_noise_rows_replay_reference_episodes(golden, name):
    """theta' rows from RNGNoiseSource draws through fdr_rollout (base_stride = P, no table) replay the reference's
    episodes of both epochs (the second from the theta the reference's learner produced)."""
    from envs import SyntheticEnv
    from fdr import engine
    from utils.noise_sources import HostNoiseRows
    g = golden("g15_rng_noise_source.npz")
    kind, n_in, n_act = SHAPES[name]
    T = int(g[name + "_T"])
    dev = torch.device("cuda", 0)
    env = SyntheticEnv(n_in, n_act, kind == "discrete", T, env_seed=0, device=dev)
    for e, st in enumerate(_stream(g, name)):
        pre = "%s_e%d_" % (name, e)
        theta = g[name + "_theta0"] if e == 0 else g["%s_e%d_theta" % (name, e - 1)]
        P = theta.size
        np.testing.assert_array_equal(st["is_eval"], g[pre + "is_eval"])
        assert st["enc"] == [str(x) for x in g[pre + "encoded"]]           # the PCG64 state stream
        sign = np.where(st["is_eval"], 0, 1).astype(np.int8)
        row = np.maximum(np.cumsum(~st["is_eval"]) - 1, 0)
        rows = HostNoiseRows(theta, np.stack(st["noises"]), row, sign, 0.02, dev)
        # theta' is the reference's f64 formula rounded once (worker.py:28 + set_trainable_flat)
        i0 = int(np.argmax(sign))
        np.testing.assert_array_equal(rows.theta[i0].cpu().numpy(),
                                      (theta.astype(np.float64) + 0.02 * st["noises"][0]).astype(np.float32))
        spec = engine.PolicySpec(kind, n_in, n_act, P)
        lanes = engine.lanes_desc(rows.theta, P, None, None, None, 0.0,
                                  torch.as_tensor(st["is_eval"].astype(np.int8), device=dev))
        res = engine.rollout(spec, env, lanes, len(sign), 99, jiggle=False, u_inject=torch.as_tensor(st["u"], device=dev))
        torch.cuda.synchronize()
        np.testing.assert_array_equal(res.timesteps.cpu().numpy(), g[pre + "timesteps"])
        np.testing.assert_allclose(res.reward.cpu().numpy() + st["jig"], g[pre + "reward"], rtol=1e-4, atol=1e-6)
        np.testing.assert_allclose(res.entropy.cpu().numpy(), g[pre + "entropy"], rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("name", ["cheetah", "cartpole"])
def test_learner_with_rng_noise_source_matches_reference(golden, name):
    """FiniteDifferences over an RNGNoiseSource: each return's lambda regenerated from its encoded state by decode()
    (finite_differences.py:94), two steps from the reference's returns -> the reference's theta, update, gradient."""
    from dsgd import DSGD
    from learner import FDReturn, FiniteDifferences
    from policies import DiscretePolicy, MujocoPolicy
    from utils import AdaptiveOmega
    from utils.noise_sources import RNGNoiseSource
    g = golden("g15_rng_noise_source.npz")
    kind, n_in, n_act = SHAPES[name]
    torch.manual_seed(124)
    pol = (DiscretePolicy if kind == "discrete" else MujocoPolicy)(n_in, n_act, seed=124)
    np.testing.assert_array_equal(pol.get_trainable_flat(), g[name + "_theta0"])
    P = pol.num_params
    learner = FiniteDifferences(pol, DSGD(pol.parameters(), lr=0.01), AdaptiveOmega(), RNGNoiseSource(P, 5),
                                noise_std=0.02, batch_size=8, max_delayed_return=10)
    for e in range(2):
        pre = "%s_e%d_" % (name, e)
        rets = []
        for enc, r, ev in zip(g[pre + "encoded"], g[pre + "reward"], g[pre + "is_eval"]):
            if ev:
                continue
            x = FDReturn()
            x.epoch, x.encoded_noise, x.reward = learner.epoch, str(enc), float(r)
            rets.append(x)
        upd = learner.step(rets, 0.25 * e, 0, 0)
        gm = learner.gradient_memory.cpu().numpy()
        assert np.linalg.norm(gm - g[pre + "g"]) <= 1e-5 * np.linalg.norm(g[pre + "g"])
        assert abs(upd - float(g[pre + "update"])) <= 1e-6 * float(g[pre + "update"]) + 1e-9
        np.testing.assert_allclose(pol.get_trainable_flat(), g[pre + "theta"], rtol=0, atol=1e-6)


def test_worker_and_runner_with_rng_noise_source(golden):
    """Worker.collect_returns / evaluate and SequentialRunner(noise_source="rng") drive the device path with the
    reference's default source: encoded states in the source's sample() order, eval lanes unperturbed, norm2 =
    ||fl32(sigma fl32(noise))||^2, and two training epochs whose updates are finite and nonzero."""
    from envs import SyntheticEnv
    from policies import MujocoPolicy
    from run_sequential import SequentialRunner
    from utils.noise_sources import RNGNoiseSource
    from worker import Agent, Worker
    g = golden("g15_rng_noise_source.npz")
    dev = torch.device("cuda", 0)
    torch.manual_seed(124)
    pol = MujocoPolicy(17, 6, seed=124)
    P = pol.num_params
    env = SyntheticEnv(17, 6, False, 40, env_seed=0, device=dev)
    w = Worker(pol, Agent(pol, env, random_seed=11), RNGNoiseSource(P, 5), None, sigma=0.02, eval_prob=0.25,
               random_seed=3)
    w.epoch = 0
    rets = w.collect_returns(8)
    assert [r.encoded_noise for r in rets] == [str(x) for x in g["cheetah_e0_encoded"]]
    assert [r.is_eval for r in rets] == list(g["cheetah_e0_is_eval"])
    ref = RNGNoiseSource(P, 5)
    for r in rets:
        if r.is_eval:
            assert r.norm2 == 0.0
        else:
            z = np.float32(0.02) * ref.decode(r.encoded_noise).astype(np.float32)
            assert abs(r.norm2 - float(np.dot(z.astype(np.float64), z))) <= 1e-9 * r.norm2
    b = w.evaluate(6, antithetic=True)
    assert b.noise_table is not None and b.noise_table.numel() == 6 * P and len(b.encoded) == 12
    np.testing.assert_array_equal(b.idx_host[0::2], b.idx_host[1::2])
    run = SequentialRunner(env_id="HalfCheetah-v4", batch_size=16, random_seed=7, episode_len=50, verbose=False,
                           eval_prob=0.1, noise_source="rng", zeta_size=8, max_strategy_history_size=4)
    th0 = run.policy.get_trainable_flat().copy()
    run.train(2)
    assert len(run.history) == 2 and all(np.isfinite(h["Update Magnitude"]) and h["Update Magnitude"] > 0
                                         for h in run.history)
    assert not np.array_equal(run.policy.get_trainable_flat(), th0)
    src = RNGNoiseSource(P, 7)
    assert run.history[0]["idx"] == [src.sample()[0] for _ in range(len(run.history[0]["idx"]))]
