"""GPU parity of the HIP path (through the C ABI) against the oracle and the golden fixtures.

Tolerances (DESIGN.md "Parity"):
  theta' / noise indices / trap-env returns   bit-exact
  per-step forward                            <= 1e-5 abs (fp32)
  episode returns (contractive synthetic env) <= 1e-4 relative (+1e-4 abs)
  gradient                                    rel-L2 <= 1e-5;  theta after DSGD <= 1e-6 abs
"""
import numpy as np
import pytest
import torch

from oracle import agent as oagent
from oracle import envs as oenvs
from oracle import learner as olearn
from oracle import noise as onoise
from oracle import policies as opol

pytestmark = pytest.mark.gpu

IMPL_NAMES = {0: "pair", 1: "single", 2: "auto", 3: "wide"}   # FDR_ROLLOUT_*
SHAPES = {"trap": ("discrete", 2, 9), "cartpole": ("discrete", 4, 2), "cheetah": ("mujoco", 17, 6)}
# the other compiled rollout shapes (no golden vectors: oracle parity only)
ROLL_SHAPES = dict(SHAPES, lunar=("discrete", 8, 4), hopper=("mujoco", 11, 3))
DEV = "cuda"


@pytest.fixture(scope="module")
def eng():
    from fdr import engine
    return engine


def dev(a, dtype=None):
    t = torch.as_tensor(np.asarray(a))
    if dtype is not None:
        t = t.to(dtype)
    return t.to(DEV).contiguous()


_TABLES = {}


def table(P, seed=124, size=2 ** 22):
    k = (P, seed, size)
    if k not in _TABLES:
        t = onoise.NoiseTable(size, P, seed)
        _TABLES[k] = (t, dev(t.table))
    return _TABLES[k]


@pytest.mark.parametrize("name", list(SHAPES))
def test_perturb_bit_exact_vs_reference(golden, eng, name):
    g = golden("g2_perturb.npz")
    theta = g["%s_s124_theta" % name]
    t, tab = table(theta.size)
    idx = g[name + "_idx"]
    sign = np.array([1, 1, 1, 1], np.int8)
    out = eng.perturb(dev(theta), tab, dev(idx, torch.int64), dev(sign), 0.02).cpu().numpy()
    assert np.array_equal(out, g[name + "_perturbed"])
    # antithetic / eval lanes against the oracle's numpy arithmetic
    sign = np.array([-1, 1, 0, -1], np.int8)
    out = eng.perturb(dev(theta), tab, dev(idx, torch.int64), dev(sign), 0.02).cpu().numpy()
    assert np.array_equal(out, onoise.perturb(theta, t.table, idx, sign, 0.02))


@pytest.mark.parametrize("name", list(SHAPES))
def test_policy_forward_vs_reference(golden, eng, name):
    g = golden("g3_forward.npz")
    kind, n_in, n_act = SHAPES[name]
    P = opol.num_params(kind, n_in, n_act)
    t, tab = table(P)
    params = (t.decode(int(g[name + "_idx"])) * 0.1).astype(np.float32)
    x = g[name + "_x"]
    spec = eng.PolicySpec(kind, n_in, n_act, P)
    lanes = eng.lanes_desc(dev(params), 0)
    base = dev(params)
    lanes = eng.lanes_desc(base, 0)
    out = eng.policy_forward(spec, lanes, len(x), dev(x))
    if kind == "discrete":
        np.testing.assert_allclose(out.cpu().numpy(), g[name + "_probs"], atol=1e-5)
        stats = [(g["%s_vbn_rm%d" % (name, i)], g["%s_vbn_rv%d" % (name, i)]) for i in range(3)]
        bm = dev(np.concatenate([s[0] for s in stats]))
        bv = dev(np.concatenate([s[1] for s in stats]))
        out = eng.policy_forward(spec, lanes, len(x), dev(x), bm, bv)
        np.testing.assert_allclose(out.cpu().numpy(), g[name + "_vbn_probs"], atol=1e-5)
    else:
        m, s = out
        np.testing.assert_allclose(m.cpu().numpy(), g[name + "_mean"], atol=1e-5)
        np.testing.assert_allclose(s.cpu().numpy(), g[name + "_std"], atol=1e-5)


@pytest.mark.parametrize("name", list(SHAPES))
def test_policy_forward_perturbed_lanes(eng, name):
    kind, n_in, n_act = SHAPES[name]
    torch.manual_seed(124)
    pol = opol.TorchPolicy(kind, n_in, n_act, seed=124)
    theta = pol.get_flat()
    P = theta.size
    t, tab = table(P)
    L = 96
    idx = t.sample_indices(L)
    sign = np.tile(np.array([1, -1, 0], np.int8), L // 3)
    x = np.random.RandomState(3).randn(L, n_in).astype(np.float32)
    spec = eng.PolicySpec(kind, n_in, n_act, P)
    lanes = eng.lanes_desc(dev(theta), 0, tab, dev(idx, torch.int64), dev(sign), 0.02)
    out = eng.policy_forward(spec, lanes, L, dev(x))
    thetas = onoise.perturb(theta, t.table, idx, sign, 0.02)
    ref = opol.lanes_forward(kind, n_in, n_act, thetas, x)
    if kind == "discrete":
        np.testing.assert_allclose(out.cpu().numpy(), ref, atol=1e-5)
    else:
        np.testing.assert_allclose(out[0].cpu().numpy(), ref[0], atol=1e-5)
        np.testing.assert_allclose(out[1].cpu().numpy(), ref[1], atol=1e-5)


def _rollout_case(eng, name, L, T, det, seed=7, antithetic=True, idx_seed=None):
    kind, n_in, n_act = ROLL_SHAPES[name]
    torch.manual_seed(124)
    pol = opol.TorchPolicy(kind, n_in, n_act, seed=124)
    theta = pol.get_flat()
    P = theta.size
    t, tab = table(P)
    # idx_seed: a private index stream (the same lanes on every call), else the table's own stream
    draw = t.sample_indices if idx_seed is None else \
        (lambda n: np.random.RandomState(idx_seed).randint(0, t.max_idx, size=n).astype(np.int64))
    if antithetic:
        idx = np.repeat(draw(L // 2), 2)
        sign = np.tile(np.array([1, -1], np.int8), L // 2)
    else:
        idx = draw(L)
        sign = np.ones(L, np.int8)
    sign[-2:] = 0                              # two eval lanes
    dflag = np.full(L, 1 if det else 0, np.int8)
    dflag[-2:] = 1
    from envs import SyntheticEnv
    env = SyntheticEnv(n_in, n_act, kind == "discrete", T, env_seed=0)
    spec = eng.PolicySpec(kind, n_in, n_act, P)
    lanes = eng.lanes_desc(dev(theta), 0, tab, dev(idx, torch.int64), dev(sign), 0.02, dev(dflag))
    res = eng.rollout(spec, env, lanes, L, seed)
    oenv = oenvs.BatchedSyntheticEnv(n_in, n_act, kind == "discrete", T, L, env_seed=0)
    ref = oagent.evaluate_lanes(kind, n_in, n_act, theta, t.table, idx, sign, 0.02, oenv, seed,
                                deterministic=dflag.astype(bool))
    return res, ref


@pytest.mark.parametrize("name,det", [("cheetah", False), ("cheetah", True), ("cartpole", False),
                                      ("cartpole", True)])
def test_rollout_vs_oracle(eng, name, det):
    res, (r_ret, r_ent, r_steps, r_n2) = _rollout_case(eng, name, 64, 200, det)
    ret = res.reward.cpu().numpy()
    np.testing.assert_allclose(ret, r_ret, rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(res.entropy.cpu().numpy(), r_ent, rtol=1e-5, atol=1e-5)
    assert np.array_equal(res.timesteps.cpu().numpy(), r_steps)
    np.testing.assert_allclose(res.norm2.cpu().numpy(), r_n2, rtol=1e-9, atol=0)


@pytest.mark.parametrize("name,L,det,T", [("cheetah", 13, False, 120), ("cheetah", 7, True, 120),
                                          ("cartpole", 13, False, 120), ("cartpole", 9, True, 120),
                                          ("cheetah", 64, False, 120), ("cheetah", 10, False, 123),
                                          ("cheetah", 6, False, 3), ("cartpole", 6, False, 37),
                                          ("lunar", 13, False, 90), ("lunar", 8, True, 40), ("hopper", 11, False, 70)])
def test_rollout_pair_and_single_kernels_agree(eng, name, L, det, T):
    """rollout_pair_kernel (two lanes per wave), rollout_kernel (one lane per wave) and its register-rich
    WIDE variant against the oracle and each other, incl. odd lane counts (a wave whose second half is
    idle) and episode lengths that are not a multiple of the pair kernel's 5-step unroll (remainder loop)."""
    from fdr._lib import FDR_ROLLOUT_PAIR, FDR_ROLLOUT_SINGLE, FDR_ROLLOUT_WIDE
    out = {}
    try:
        for impl in (FDR_ROLLOUT_SINGLE, FDR_ROLLOUT_PAIR, FDR_ROLLOUT_WIDE):
            eng.context().set_rollout_impl(IMPL_NAMES[impl])
            out[impl] = _rollout_case(eng, name, L, T, det, antithetic=L % 2 == 0, idx_seed=L)
    finally:
        eng.context().set_rollout_impl("auto")
    for impl in (FDR_ROLLOUT_SINGLE, FDR_ROLLOUT_PAIR, FDR_ROLLOUT_WIDE):
        res, (ref_ret, ref_ent, ref_steps, ref_n2) = out[impl]
        assert res.reward.numel() == L
        np.testing.assert_allclose(res.reward.cpu().numpy(), ref_ret, rtol=1e-4, atol=1e-4)
        np.testing.assert_allclose(res.entropy.cpu().numpy(), ref_ent, rtol=1e-5, atol=1e-5)
        assert np.array_equal(res.timesteps.cpu().numpy(), ref_steps)
        np.testing.assert_allclose(res.norm2.cpu().numpy(), ref_n2, rtol=1e-9, atol=0)
    a, b, w = out[FDR_ROLLOUT_SINGLE][0], out[FDR_ROLLOUT_PAIR][0], out[FDR_ROLLOUT_WIDE][0]
    np.testing.assert_allclose(a.reward.cpu().numpy(), b.reward.cpu().numpy(), rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(a.reward.cpu().numpy(), w.reward.cpu().numpy(), rtol=1e-5, atol=1e-5)
    np.testing.assert_array_equal(a.norm2.cpu().numpy(), w.norm2.cpu().numpy())


@pytest.mark.parametrize("name", ["cheetah", "cartpole"])
def test_rollout_kernels_obs_norm_and_states_vs_oracle(eng, name):
    """FEAT paths of both synthetic-env kernels (observation normalisation, visited states, both) against
    the oracle, with the kernel forced (auto would pick the wide one-lane kernel at this lane count)."""
    from envs import SyntheticEnv
    from fdr._lib import FDR_ROLLOUT_PAIR, FDR_ROLLOUT_SINGLE, FDR_ROLLOUT_WIDE
    kind, n_in, n_act = SHAPES[name]
    torch.manual_seed(124)
    pol = opol.TorchPolicy(kind, n_in, n_act, seed=124)
    theta = pol.get_flat()
    t, tab = table(theta.size)
    L, T, seed = 13, 80, 5
    idx = np.random.RandomState(11).randint(0, t.max_idx, size=L).astype(np.int64)
    sign = np.ones(L, np.int8)
    sign[-1] = 0
    om = np.linspace(-0.2, 0.2, n_in).astype(np.float32)
    osd = np.linspace(0.5, 1.5, n_in).astype(np.float32)
    spec = eng.PolicySpec(kind, n_in, n_act, theta.size)
    lanes = eng.lanes_desc(dev(theta), 0, tab, dev(idx, torch.int64), dev(sign), 0.02)
    env = SyntheticEnv(n_in, n_act, kind == "discrete", T, env_seed=0)
    oenv = oenvs.BatchedSyntheticEnv(n_in, n_act, kind == "discrete", T, L, env_seed=0)
    ref = oagent.evaluate_lanes(kind, n_in, n_act, theta, t.table, idx, sign, 0.02, oenv, seed, obs_mean=om,
                                obs_std=osd, record_states=True)
    ref_states = ref[-1]
    try:
        for impl in (FDR_ROLLOUT_SINGLE, FDR_ROLLOUT_PAIR, FDR_ROLLOUT_WIDE):
            eng.context().set_rollout_impl(IMPL_NAMES[impl])
            for norm, rec in ((True, False), (False, True), (True, True)):
                states = torch.empty((L, T, n_in), dtype=torch.float32, device=DEV) if rec else None
                res = eng.rollout(spec, env, lanes, L, seed, obs_mean=dev(om) if norm else None,
                                  obs_std=dev(osd) if norm else None, states=states)
                torch.cuda.synchronize()
                if norm:
                    np.testing.assert_allclose(res.reward.cpu().numpy(), ref[0], rtol=1e-4, atol=1e-4)
                    np.testing.assert_allclose(res.entropy.cpu().numpy(), ref[1], rtol=1e-5, atol=1e-5)
                if rec and norm:
                    np.testing.assert_allclose(states.cpu().numpy(), ref_states, atol=1e-4)
                if rec and not norm:
                    S = states.cpu().numpy()
                    np.testing.assert_array_equal(S[:, 0], np.broadcast_to(ref_states[0, 0], S[:, 0].shape))
    finally:
        eng.context().set_rollout_impl("auto")


def test_rollout_reproducible_and_antithetic_norms(eng):
    torch.manual_seed(124)
    pol = opol.TorchPolicy("mujoco", 17, 6, seed=124)
    theta = pol.get_flat()
    t, tab = table(theta.size)
    L = 32
    idx = np.repeat(t.sample_indices(L // 2), 2)
    sign = np.tile(np.array([1, -1], np.int8), L // 2)
    sign[-2:] = 0
    from envs import SyntheticEnv
    env = SyntheticEnv(17, 6, False, 50)
    spec = eng.PolicySpec("mujoco", 17, 6, theta.size)
    lanes = eng.lanes_desc(dev(theta), 0, tab, dev(idx, torch.int64), dev(sign), 0.02)
    res1 = eng.rollout(spec, env, lanes, L, 7)
    res2 = eng.rollout(spec, env, lanes, L, 7)
    assert torch.equal(res1.reward, res2.reward) and torch.equal(res1.entropy, res2.entropy)
    n2 = res1.norm2.cpu().numpy()
    assert np.array_equal(n2[0:-2:2], n2[1:-2:2])     # +eps / -eps lanes share ||lambda||
    assert np.all(n2[-2:] == 0)                       # eval lanes are unperturbed


def test_trap_env_deterministic_vs_reference(golden, eng):
    g = golden("g5_trap.npz")
    from envs import TrapEnv
    env = TrapEnv()
    for seed in (124, 1, 2):
        theta = g["det_s%d_theta" % seed]
        spec = eng.PolicySpec("discrete", 2, 9, theta.size)
        lanes = eng.lanes_desc(dev(theta), 0, deterministic=dev(np.ones(1, np.int8)))
        res = eng.rollout(spec, env, lanes, 1, 0, jiggle=False)
        ref = g["det_s%d" % seed]
        assert res.reward.item() == round(ref[0])              # integer-exact (jiggle off)
        assert res.timesteps.item() == ref[2]
        assert abs(res.entropy.item() - ref[1]) < 1e-5


def test_trap_env_sampled_vs_oracle(eng):
    torch.manual_seed(124)
    pol = opol.TorchPolicy("discrete", 2, 9, seed=124)
    theta = pol.get_flat()
    t, tab = table(theta.size)
    L = 8
    idx = t.sample_indices(L)
    sign = np.ones(L, np.int8)
    from envs import TrapEnv
    from oracle import rng as crng
    spec = eng.PolicySpec("discrete", 2, 9, theta.size)
    lanes = eng.lanes_desc(dev(theta), 0, tab, dev(idx, torch.int64), dev(sign), 0.5)
    res = eng.rollout(spec, TrapEnv(), lanes, L, 99, jiggle=False)
    thetas = onoise.perturb(theta, t.table, idx, sign, 0.5)
    for l in range(L):
        pol.set_flat(thetas[l])
        env = oenvs.TrapEnv()
        r, e, steps, _ = oagent.collect_return(
            pol, env, env.reset(), False, lambda s, l=l: np.float32(crng.uniform(99, l, s, 0)), lambda: 0.0)
        assert res.reward[l].item() == r
        assert res.timesteps[l].item() == steps == 201
        assert abs(res.entropy[l].item() - e) < 1e-5


@pytest.mark.parametrize("case", ["cheetah_n16", "cheetah_n64", "trap_n16"])
def test_fd_step_vs_reference(golden, eng, case):
    """weights -> gradient reduce -> DSGD on the device vs the reference's FiniteDifferences.step."""
    g = golden("g4_fd_step.npz")
    theta0 = g[case + "_theta0"]
    P = theta0.size
    t, tab = table(P)
    idx = g[case + "_idx"]
    N = idx.size
    sign = np.ones(N, np.int8)
    s32 = np.float32(0.02)
    n2 = np.array([float(np.dot((t.decode(i) * s32).astype(np.float64), (t.decode(i) * s32).astype(np.float64)))
                   for i in idx])
    rewards = dev(g[case + "_rewards"])
    coef = eng.fd_weights(rewards, 0.25, 0, dev(sign), dev(n2), 1, 0.02)
    grad = eng.fd_grad(tab, dev(idx, torch.int64), coef, P)
    gref = g[case + "_g"]
    assert np.linalg.norm(grad.cpu().numpy() - gref) / np.linalg.norm(gref) < 1e-5
    theta = dev(theta0)
    om = float(g[case + "_omega"])
    lr_scale = olearn.affine_transform(om, 0, 1, 0.23, 1.0)
    out = eng.dsgd_step(theta, grad, 0.01, lr_scale).cpu().numpy()
    np.testing.assert_allclose(theta.cpu().numpy(), g[case + "_theta1"], rtol=0, atol=1e-6)
    assert abs(out[0] - float(g[case + "_update"])) < 1e-5


def test_fd_grad_matches_oracle_antithetic(eng):
    P = 6092
    t, tab = table(P)
    D = 300
    idx = t.sample_indices(D)
    rng = np.random.RandomState(4)
    r = rng.randn(2 * D)
    lidx = np.repeat(idx, 2)
    sign = np.tile(np.array([1, -1], np.int8), D)
    s32 = np.float32(0.02)
    n2 = np.array([float(np.dot((t.decode(i) * s32).astype(np.float64), (t.decode(i) * s32).astype(np.float64)))
                   for i in lidx])
    coef = eng.fd_weights(dev(r), -0.3, 0, dev(sign), dev(n2), 2, 0.02)
    grad = eng.fd_grad(tab, dev(idx, torch.int64), coef, P).cpu().numpy()
    gref, _ = olearn.fd_gradient(t.table, P, lidx, sign, r, -0.3, 0.02)
    assert np.linalg.norm(grad - gref) / np.linalg.norm(gref) < 1e-5


def test_dsgd_zero_gradient_reports_norm_zero(eng):
    theta = dev(np.ones(100, np.float32))
    out = eng.dsgd_step(theta, torch.zeros(100, dtype=torch.float64, device=DEV), 0.01, 1.0).cpu().numpy()
    assert out[1] == 0.0 and out[0] == 0.0
    assert torch.all(theta == 1)


def test_full_size_properties(eng):
    """BASELINE config 3 size (4096 lanes x T=1000): size-independent properties + sampled parity."""
    name = "cheetah"
    kind, n_in, n_act = SHAPES[name]
    torch.manual_seed(124)
    pol = opol.TorchPolicy(kind, n_in, n_act, seed=124)
    theta = pol.get_flat()
    P = theta.size
    t, tab = table(P, size=25_000_000)
    L, T = 4096, 1000
    idx = np.repeat(t.sample_indices(L // 2), 2)
    sign = np.tile(np.array([1, -1], np.int8), L // 2)
    from envs import SyntheticEnv
    env = SyntheticEnv(n_in, n_act, False, T)
    spec = eng.PolicySpec(kind, n_in, n_act, P)
    lanes = eng.lanes_desc(dev(theta), 0, tab, dev(idx, torch.int64), dev(sign), 0.02)
    res = eng.rollout(spec, env, lanes, L, 5)
    res2 = eng.rollout(spec, env, lanes, L, 5)
    ret = res.reward.cpu().numpy()
    assert np.isfinite(ret).all() and torch.equal(res.reward, res2.reward)
    assert (res.timesteps.cpu().numpy() == T).all()
    n2 = res.norm2.cpu().numpy()
    assert np.array_equal(n2[0::2], n2[1::2])
    # sampled lanes against the oracle at full episode length
    pick = np.array([0, 1, 777, 2048, 4095])
    oenv = oenvs.BatchedSyntheticEnv(n_in, n_act, False, T, len(pick), env_seed=0)
    # the counter stream is keyed by the lane id, so evaluate the picked lanes with their ids
    ref = _oracle_lanes_with_ids(kind, n_in, n_act, theta, t.table, idx[pick], sign[pick], oenv, 5, pick)
    np.testing.assert_allclose(ret[pick], ref, rtol=1e-4, atol=1e-4)
    # every lane: the auto-selected two-lanes-per-wave kernel against the one-lane kernel
    from fdr._lib import FDR_ROLLOUT_AUTO, FDR_ROLLOUT_SINGLE, check, lib
    try:
        eng.context().set_rollout_impl("single")
        res1 = eng.rollout(spec, env, lanes, L, 5)
        torch.cuda.synchronize()
    finally:
        eng.context().set_rollout_impl("auto")
    np.testing.assert_allclose(ret, res1.reward.cpu().numpy(), rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(res.entropy.cpu().numpy(), res1.entropy.cpu().numpy(), rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(n2, res1.norm2.cpu().numpy(), rtol=1e-12)


def test_pair_kernel_multi_round_launch(eng):
    """More lanes than one resident round of rollout_pair_kernel (16 lanes per CU): the lanes go out as
    consecutive launches (lane_base) -- here 2 x 16 x CUs + 10 lanes, three rounds with a ragged last one,
    odd L (an idle half wave at the end).  Every lane against the one-lane kernel, sampled lanes incl. each
    round's first and last lane against the oracle (bench.py's 4096-pair variant takes this path)."""
    name = "cheetah"
    kind, n_in, n_act = SHAPES[name]
    torch.manual_seed(124)
    pol = opol.TorchPolicy(kind, n_in, n_act, seed=124)
    theta = pol.get_flat()
    P = theta.size
    t, tab = table(P, size=25_000_000)
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    L, T = 2 * 16 * cus + 11, 60
    idx = np.random.RandomState(3).randint(0, t.max_idx, size=L).astype(np.int64)
    sign = np.where(np.arange(L) % 2 == 0, 1, -1).astype(np.int8)
    from envs import SyntheticEnv
    env = SyntheticEnv(n_in, n_act, False, T)
    spec = eng.PolicySpec(kind, n_in, n_act, P)
    lanes = eng.lanes_desc(dev(theta), 0, tab, dev(idx, torch.int64), dev(sign), 0.02)
    try:
        eng.context().set_rollout_impl("pair")
        res = eng.rollout(spec, env, lanes, L, 9)
        eng.context().set_rollout_impl("single")
        res1 = eng.rollout(spec, env, lanes, L, 9)
        torch.cuda.synchronize()
    finally:
        eng.context().set_rollout_impl("auto")
    ret = res.reward.cpu().numpy()
    assert (res.timesteps.cpu().numpy() == T).all()
    np.testing.assert_allclose(ret, res1.reward.cpu().numpy(), rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(res.entropy.cpu().numpy(), res1.entropy.cpu().numpy(), rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(res.norm2.cpu().numpy(), res1.norm2.cpu().numpy(), rtol=1e-12)
    per = ((L + 2) // 3 + 3) // 4 * 4     # launch_pair: equal rounds in whole workgroups (4 lanes)
    pick = np.unique(np.array([0, 1, per - 1, per, per + 1, 2 * per - 1, 2 * per, L - 2, L - 1]))
    oenv = oenvs.BatchedSyntheticEnv(n_in, n_act, False, T, len(pick), env_seed=0)
    ref = _oracle_lanes_with_ids(kind, n_in, n_act, theta, t.table, idx[pick], sign[pick], oenv, 9, pick)
    np.testing.assert_allclose(ret[pick], ref, rtol=1e-4, atol=1e-4)


def test_full_size_properties_config2(eng):
    """BASELINE config 2 size (1024 lanes x T=500, CartPole-shaped, discrete): the auto-selected WIDE one-lane
    kernel is reproducible, antithetic norms are symmetric, sampled lanes match the oracle over the full
    episode, and every lane matches the 128-VGPR one-lane kernel."""
    name = "cartpole"
    kind, n_in, n_act = SHAPES[name]
    torch.manual_seed(124)
    pol = opol.TorchPolicy(kind, n_in, n_act, seed=124)
    theta = pol.get_flat()
    P = theta.size
    t, tab = table(P, size=25_000_000)
    L, T = 1024, 500
    idx = np.repeat(t.sample_indices(L // 2), 2)
    sign = np.tile(np.array([1, -1], np.int8), L // 2)
    from envs import SyntheticEnv
    env = SyntheticEnv(n_in, n_act, True, T)
    spec = eng.PolicySpec(kind, n_in, n_act, P)
    lanes = eng.lanes_desc(dev(theta), 0, tab, dev(idx, torch.int64), dev(sign), 0.02)
    res = eng.rollout(spec, env, lanes, L, 9)
    res2 = eng.rollout(spec, env, lanes, L, 9)
    ret = res.reward.cpu().numpy()
    assert np.isfinite(ret).all() and torch.equal(res.reward, res2.reward)
    assert (res.timesteps.cpu().numpy() == T).all()
    n2 = res.norm2.cpu().numpy()
    assert np.array_equal(n2[0::2], n2[1::2])
    pick = np.array([0, 1, 333, 512, 1023])
    oenv = oenvs.BatchedSyntheticEnv(n_in, n_act, True, T, len(pick), env_seed=0)
    ref = oagent.evaluate_lanes(kind, n_in, n_act, theta, t.table, idx[pick], sign[pick], 0.02, oenv, 9,
                                lane_ids=pick)
    np.testing.assert_allclose(ret[pick], ref[0], rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(res.entropy.cpu().numpy()[pick], ref[1], rtol=1e-5, atol=1e-5)
    try:
        eng.context().set_rollout_impl("single")
        res1 = eng.rollout(spec, env, lanes, L, 9)
        torch.cuda.synchronize()
    finally:
        eng.context().set_rollout_impl("auto")
    np.testing.assert_allclose(ret, res1.reward.cpu().numpy(), rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(res.entropy.cpu().numpy(), res1.entropy.cpu().numpy(), rtol=1e-5, atol=1e-5)
    np.testing.assert_array_equal(n2, res1.norm2.cpu().numpy())


def _oracle_lanes_with_ids(kind, n_in, n_act, theta, tab, idx, sign, env, seed, ids):
    from oracle import rng as crng
    thetas = onoise.perturb(theta, tab, idx, sign, 0.02)
    obs = env.reset()
    ret = np.zeros(len(ids))
    lanes = np.asarray(ids, dtype=np.uint64)
    for s in range(env.episode_len):
        mean, std = opol.lanes_forward(kind, n_in, n_act, thetas, obs)
        z = crng.normal(seed, lanes[:, None], s, np.arange(n_act, dtype=np.uint64)[None, :])
        obs, r = env.step((mean + std * z).astype(np.float32))
        ret += r
    return ret + crng.jiggle(seed, lanes)


def test_lambda_drift_norms_and_grad_vs_oracle(eng):
    """Delayed returns (finite_differences.py:88-114): lambda = sign * fl32(sigma eps) + dist_map[epoch]."""
    P = 6092
    t, tab = table(P)
    rs = np.random.RandomState(4)
    n = 10
    idx = t.sample_indices(n)
    sign = rs.choice([-1, 1], n).astype(np.int8)
    drift = (rs.randn(2, P) * 0.01).astype(np.float32)
    slot = rs.choice([-1, 0, 1], n).astype(np.int32)
    s32 = np.float32(0.02)
    lam = np.stack([(np.float32(sg) * (t.table[i:i + P] * s32).astype(np.float32)).astype(np.float32)
                    + (drift[sl] if sl >= 0 else np.float32(0)) for i, sg, sl in zip(idx, sign, slot)]).astype(np.float32)
    n2_ref = (lam.astype(np.float64) ** 2).sum(1)
    n2 = eng.fd_lambda_norms(tab, dev(idx, torch.int64), dev(sign), dev(slot), 0.02, dev(drift), P).cpu().numpy()
    np.testing.assert_allclose(n2, n2_ref, rtol=1e-12)
    coef = rs.randn(n)
    g = eng.fd_grad_lambda(tab, dev(idx, torch.int64), dev(sign), dev(slot), dev(coef), 0.02, dev(drift), P)
    g_ref = coef @ lam.astype(np.float64)
    assert np.linalg.norm(g.cpu().numpy() - g_ref) <= 1e-12 * np.linalg.norm(g_ref)


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_fd_weights_and_grad_sum_to_unsharded(eng, world):
    """The multi-GPU learner's arithmetic on one GPU: a 512-direction antithetic batch split into the standard
    rank slices (fdr.dist.lane_range); each slice runs fdr_fd_weights(lane_lo = its first lane) over the
    all-gathered rewards and fdr_fd_grad over its directions.  The slices' gradients sum to the unsharded
    gradient (the all-reduce) within f64 reordering, and to the oracle's."""
    from fdr import dist as fdist
    from oracle import learner as olearn
    P, n_dirs, sigma = 6092, 512, 0.02
    rs = np.random.RandomState(21)
    table = rs.randn(1 << 22).astype(np.float32)
    idx_dirs = rs.randint(0, table.size - P, size=n_dirs).astype(np.int64)
    idx = np.repeat(idx_dirs, 2)
    sign = np.tile(np.array([1, -1], np.int8), n_dirs)
    rew = rs.randn(2 * n_dirs) * 3 + 1
    s32 = np.float32(sigma)
    n2 = np.array([float(np.dot((table[i:i + P] * s32).astype(np.float64), (table[i:i + P] * s32).astype(np.float64)))
                   for i in idx])
    tab = torch.as_tensor(table, device="cuda")
    rew_d = torch.as_tensor(rew, device="cuda")
    sign_d = torch.as_tensor(sign, device="cuda")
    n2_d = torch.as_tensor(n2, device="cuda")
    idx_d = torch.as_tensor(idx_dirs, device="cuda")
    coef = eng.fd_weights(rew_d, 0.25, 0, sign_d, n2_d, 2, sigma)
    g_full = eng.fd_grad(tab, idx_d, coef, P).cpu().numpy().copy()
    g_sum = np.zeros(P)
    for rank in range(world):
        lo, hi = fdist.lane_range(n_dirs, 2, world, rank)
        assert lo % 2 == 0 and hi % 2 == 0
        c = eng.fd_weights(rew_d, 0.25, lo, sign_d[lo:hi].contiguous(), n2_d[lo:hi].contiguous(), 2, sigma)
        g_sum += eng.fd_grad(tab, idx_d[lo // 2:hi // 2].contiguous(), c, P).cpu().numpy()
    assert np.linalg.norm(g_sum - g_full) / np.linalg.norm(g_full) <= 1e-12
    g_ref, _ = olearn.fd_gradient(table, P, idx, sign, rew, 0.25, sigma)
    assert np.linalg.norm(g_full - g_ref) / np.linalg.norm(g_ref) <= 1e-5


def test_two_contexts_hold_independent_rollout_selections(eng):
    """fdr_ctx carries the rollout kernel selection: two contexts on one device, one set to the pair kernel and
    one to the one-lane kernel, used alternately with no global state flipped, each reproduce (bitwise) the
    kernel they select; the default context is untouched."""
    from fdr import engine as E
    name = "cheetah"
    kind, n_in, n_act = SHAPES[name]
    torch.manual_seed(124)
    pol = opol.TorchPolicy(kind, n_in, n_act, seed=124)
    theta = pol.get_flat()
    P = theta.size
    t, tab = table(P)
    L = 64
    idx = np.repeat(t.sample_indices(L // 2), 2)
    sign = np.tile(np.array([1, -1], np.int8), L // 2)
    from envs import SyntheticEnv
    env = SyntheticEnv(n_in, n_act, False, 120, env_seed=0)
    lanes = eng.lanes_desc(dev(theta), 0, tab, dev(idx, torch.int64), dev(sign, torch.int8), 0.02)
    spec = eng.PolicySpec(kind, n_in, n_act, P)
    ca, cb = E.Context(DEV), E.Context(DEV)
    ca.set_rollout_impl("pair")
    cb.set_rollout_impl("single")
    outs = {}
    for rep in range(2):
        for name_, c in (("pair", ca), ("single", cb)):
            r = eng.rollout(spec, env, lanes, L, 5, ctx=c)
            outs.setdefault(name_, []).append(r.reward.cpu().numpy().copy())
    for k in outs:
        np.testing.assert_array_equal(outs[k][0], outs[k][1])
    assert not np.array_equal(outs["pair"][0], outs["single"][0])     # different kernels: different sum order
    np.testing.assert_allclose(outs["pair"][0], outs["single"][0], rtol=1e-4, atol=1e-4)
    # the engine's own context of the device was never switched: auto (64 lanes -> one-lane kernel)
    np.testing.assert_array_equal(eng.rollout(spec, env, lanes, L, 5).reward.cpu().numpy(), outs["single"][0])
