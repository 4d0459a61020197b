"""GPU parity of the AtariPolicy path (fdr_atari_forward / fdr_atari_rollout) against the oracle and the
reference (tests/golden/g11_atari.npz).  Tolerances: features / probs 1e-5 relative to scale (f32 MFMA
vs torch-CPU summation order); actions and integer rewards exact; norm2 rel 1e-9."""
import numpy as np
import pytest
import torch

from oracle import atari as oa

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engine():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from fdr import engine
    return engine


def test_forward_matches_reference_golden(engine, golden):
    g = golden("g11_atari.npz")
    A = int(g["A"])
    theta = torch.tensor(oa.init_theta(A, 124), device="cuda")
    spec = engine.AtariSpec(A)
    probs, feat = engine.atari_forward(spec, theta, torch.tensor(g["frames"].astype(np.float32), device="cuda"),
                                       bn_mean=torch.tensor(g["rm"], device="cuda"),
                                       bn_var=torch.tensor(g["rv"], device="cuda"), feat=True)
    torch.cuda.synchronize()
    f = feat.cpu().numpy()
    assert np.abs(f - g["feat"]).max() <= 1e-5 * np.abs(g["feat"]).max()
    np.testing.assert_allclose(probs.cpu().numpy(), g["probs"], rtol=1e-5, atol=1e-7)


@pytest.mark.parametrize("E,det", [(2, 0), (1, 1)])
def test_rollout_vs_oracle(engine, E, det):
    A, T = 6, 3
    theta = oa.init_theta(A, 124)
    table = np.random.RandomState(124).randn(1 << 21).astype(np.float32)
    idx = np.array([11, 400000, 1000000], np.int64)
    sign = np.array([1, -1, 1], np.int8)
    dets = np.full(3, det, np.int8)
    dev = "cuda"
    lanes = engine.lanes_desc(torch.tensor(theta, device=dev), 0, torch.tensor(table, device=dev),
                              torch.tensor(idx, device=dev), torch.tensor(sign, device=dev), 0.02,
                              torch.tensor(dets, device=dev), lane_offset=3)
    out = engine.atari_rollout(engine.AtariSpec(A, E, T, env_seed=9), lanes, 3, 21, record=True)
    torch.cuda.synchronize()
    nb = 304
    ref = oa.evaluate_lanes(theta, table, idx, sign, 0.02, A, E, T, 21, 9, np.zeros(nb, np.float32),
                            np.ones(nb, np.float32), deterministic=dets.astype(bool), lane_offset=3, record=True)
    np.testing.assert_allclose(out.probs.cpu().numpy().reshape(3, E, T, A), ref["probs"], rtol=1e-5, atol=1e-7)
    np.testing.assert_array_equal(out.actions.cpu().numpy().reshape(3, E, T), ref["actions"])
    np.testing.assert_array_equal(out.reward.cpu().numpy().reshape(3, E), ref["ret"])
    np.testing.assert_allclose(out.entropy.cpu().numpy().reshape(3, E), ref["ent"], rtol=1e-6)
    np.testing.assert_allclose(out.norm2.cpu().numpy(), ref["norm2"], rtol=1e-9)


def test_host_policy_init_and_worker_batch(engine, golden):
    """AtariPolicy host class: normc init bit-exact with the reference; Worker.evaluate -> learner step."""
    import hashlib
    from dsgd import DSGD
    from envs import StackedFrameEnv
    from learner import FiniteDifferences
    from policies import AtariPolicy
    from utils import AdaptiveOmega, SharedNoiseTable
    from worker import Agent, Worker
    g = golden("g11_atari.npz")
    torch.manual_seed(124)
    pol = AtariPolicy((84, 84), 6, seed=124)
    flat = pol.get_trainable_flat()
    assert hashlib.sha256(np.ascontiguousarray(flat).tobytes()).hexdigest() == str(g["init_sha"])
    probs = pol.forward(g["frames"].astype(np.float32))
    assert probs.shape == (5, 6)
    nt = SharedNoiseTable(1 << 21, pol.num_params, random_seed=124)
    env = StackedFrameEnv(6, episode_len=3, envs_per_lane=2, env_seed=9)
    worker = Worker(pol, Agent(pol, env, random_seed=3), nt, None, sigma=0.02)
    learner = FiniteDifferences(pol, DSGD(pol.parameters(), lr=0.01), AdaptiveOmega(), nt, noise_std=0.02)
    batch = worker.evaluate(2, antithetic=True, seed=5)
    assert len(batch) == 8
    upd = learner.step(batch, 0.0, 0.0, 0.0)
    assert np.isfinite(upd) and upd > 0
