"""Generate the golden fixtures in tests/golden/ by running the REFERENCE itself.

Run in the build container only (needs /root/reference, read-only):
    python tests/golden/make_golden.py

What it does:
  * imports the reference (nexus-rl/dfd-starter @ /root/reference) with an in-script ``gym`` /
    ``wandb`` stub -- neither is installed -- and with bytecode writing disabled so nothing is
    written under /root/reference;
  * runs the reference's own classes (SharedNoiseTable, DiscretePolicy, MujocoPolicy, Worker,
    Agent, FiniteDifferences, DSGD, AdaptiveOmega, SequentialRunner, the trap env) on small
    seeded inputs and stores inputs + outputs as .npz DATA;
  * the only harness patches are the ones SURVEY.md section 8c lists (Worker.update,
    learner.noise_std, RNGNoiseSource -> SharedNoiseTable) plus action sampling replaced by
    injected noise (the torch multinomial / normal streams cannot be reproduced elsewhere).

Nothing here ships to the GPU box: the box only sees the .npz files.
"""
import hashlib
import io
import os
import sys
import types
import contextlib

import numpy as np

sys.dont_write_bytecode = True           # never write __pycache__ into /root/reference
REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)


# ------------------------------------------------------------------------------------------
# gym / wandb stubs (the reference imports them at module level; neither is installed)
# ------------------------------------------------------------------------------------------
def _install_stubs():
    gym = types.ModuleType("gym")
    spaces = types.ModuleType("gym.spaces")

    class Env(object):
        pass

    class Discrete(object):
        def __init__(self, n):
            self.n = n
            self._rng = np.random.RandomState(0)

        def seed(self, s):
            self._rng = np.random.RandomState(s)

        def sample(self):
            return int(self._rng.randint(self.n))

    class Box(object):
        def __init__(self, low, high, shape=None, dtype=np.float32):
            self.low, self.high, self.shape = low, high, tuple(shape)
            self._rng = np.random.RandomState(0)

        def seed(self, s):
            self._rng = np.random.RandomState(s)

        def sample(self):
            return self._rng.uniform(-1, 1, size=self.shape).astype(np.float32)

    registry = {}

    def register(id, entry_point, **kw):
        registry[id] = entry_point

    def make(env_id, **kw):
        return _ENV_FACTORY[env_id]()

    spaces.Discrete, spaces.Box = Discrete, Box
    gym.Env, gym.spaces, gym.register, gym.make = Env, spaces, register, make
    sys.modules["gym"] = gym
    sys.modules["gym.spaces"] = spaces
    sys.modules["wandb"] = types.ModuleType("wandb")
    return gym


_ENV_FACTORY = {}
gym = _install_stubs()
sys.path.insert(0, REF)

import torch  # noqa: E402
from utils.noise_sources import SharedNoiseTable  # noqa: E402  (reference)
from policies import DiscretePolicy, MujocoPolicy  # noqa: E402  (reference)
from worker import Agent, Worker  # noqa: E402  (reference)
from learner import FiniteDifferences, FDReturn, FDState  # noqa: E402  (reference)
from dsgd import DSGD  # noqa: E402  (reference)
from utils import AdaptiveOmega, math_helpers  # noqa: E402  (reference)
from strategy import StrategyHandler  # noqa: E402  (reference)
import run_sequential  # noqa: E402  (reference)

from oracle.envs import SyntheticEnv  # noqa: E402  (build-defined env; ours)


def _trap_env():
    """Reference trap env constructed with opt_id=None so it never writes action logs."""
    from custom_envs.simple_trap_env import Environment
    cwd = os.getcwd()
    os.chdir(REF)                      # map.txt is loaded by a relative path (read only)
    try:
        env = Environment(opt_id=None)
    finally:
        os.chdir(cwd)
    return env


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def save(name, **arrays):
    path = os.path.join(HERE, name)
    np.savez_compressed(path, **arrays)
    print("wrote", os.path.relpath(path, REPO), sum(np.asarray(v).nbytes for v in arrays.values()), "bytes")


def make_policy(kind, n_in, n_act, seed):
    torch.manual_seed(seed)
    if kind == "discrete":
        return DiscretePolicy(n_in, n_act, seed=seed)
    return MujocoPolicy(n_in, n_act, seed=seed)


SHAPES = {"trap": ("discrete", 2, 9), "cartpole": ("discrete", 4, 2), "cheetah": ("mujoco", 17, 6)}


# ------------------------------------------------------------------------------------------
def g1_noise():
    out = {}
    for seed in (124, 7):
        for P in (5197, 4874, 6092):
            t = SharedNoiseTable(2 ** 22, P, random_seed=seed)
            idx = np.array([int(t.sample()[0]) for _ in range(64)], dtype=np.int64)
            key = "s%d_p%d" % (seed, P)
            out[key + "_idx"] = idx
            out[key + "_spot"] = t._table[[0, 1, 2, 1000, 2 ** 21, 2 ** 22 - 1]]
            out[key + "_sha"] = np.array(sha(t._table))
    t = SharedNoiseTable(25_000_000, 6092, random_seed=124)
    out["big_idx"] = np.array([int(t.sample()[0]) for _ in range(256)], dtype=np.int64)
    out["big_sha"] = np.array(sha(t._table))
    out["big_spot"] = t._table[[0, 12_345_678, 24_999_999]]
    save("g1_noise.npz", **out)


def g2_perturb():
    out = {}
    for name, (kind, n_in, n_act) in SHAPES.items():
        for seed in (124, 123):
            pol = make_policy(kind, n_in, n_act, seed)
            out["%s_s%d_theta" % (name, seed)] = pol.get_trainable_flat().copy()
        pol = make_policy(kind, n_in, n_act, 124)
        P = pol.num_params
        table = SharedNoiseTable(2 ** 22, P, random_seed=124)
        flat = pol.get_trainable_flat()
        idx, new = [], []
        for _ in range(4):
            enc, noise = table.sample()
            idx.append(int(enc))
            new.append(flat + 0.02 * noise)          # worker/worker.py:28
        out[name + "_idx"] = np.array(idx, dtype=np.int64)
        out[name + "_perturbed"] = np.stack(new).astype(np.float32)
    save("g2_perturb.npz", **out)


def g3_forward():
    out = {}
    obs_rng = np.random.RandomState(5)
    for name, (kind, n_in, n_act) in SHAPES.items():
        pol = make_policy(kind, n_in, n_act, 124)
        P = pol.num_params
        table = SharedNoiseTable(2 ** 22, P, random_seed=124)
        idx = int(table.sample()[0])
        params = (table.decode(idx) * 0.1).astype(np.float32)
        pol.set_trainable_flat(params)
        x = obs_rng.randn(8, n_in).astype(np.float32)
        out[name + "_idx"] = np.array(idx)
        out[name + "_x"] = x
        with torch.no_grad():
            if kind == "discrete":
                out[name + "_probs"] = pol.forward(x).numpy()
                out[name + "_entropy"] = np.array(pol.get_entropy(x))
                out[name + "_argmax"] = np.array([pol.get_action(x[i], deterministic=True) for i in range(8)])
                # non-trivial BN running stats via the reference's own compute_vbn (policy.py:31-34)
                buf = obs_rng.randn(32, n_in).astype(np.float32) * 2 + 0.5
                pol.compute_vbn(buf)
                bns = [m for m in pol.model if isinstance(m, torch.nn.BatchNorm1d)]
                for i, m in enumerate(bns):
                    out["%s_vbn_rm%d" % (name, i)] = m.running_mean.numpy().copy()
                    out["%s_vbn_rv%d" % (name, i)] = m.running_var.numpy().copy()
                out[name + "_vbn_buf"] = buf
                out[name + "_vbn_probs"] = pol.forward(x).numpy()
            else:
                mean, std = pol.forward(x)
                out[name + "_mean"] = mean.numpy()
                out[name + "_std"] = std.numpy()
                out[name + "_entropy"] = np.array(pol.get_entropy(x))
                out[name + "_det_action"] = np.array([pol.get_action(x[i], deterministic=True) for i in range(8)])
    save("g3_forward.npz", **out)


def _fd_case(kind, n_in, n_act, N, omega_value, seed):
    pol = make_policy(kind, n_in, n_act, 124)
    P = pol.num_params
    opt = DSGD(pol.parameters(), lr=0.01)
    omega = AdaptiveOmega()
    omega.omega = omega_value
    table = SharedNoiseTable(2 ** 22, P, random_seed=124)
    learner = FiniteDifferences(pol, opt, omega, table, noise_std=0.02, batch_size=N,
                                max_delayed_return=10)
    theta0 = pol.get_trainable_flat().copy()
    rng = np.random.RandomState(seed)
    rewards = rng.randn(N) * 3 + 1
    batch, idx = [], []
    for i in range(N):
        r = FDReturn()
        r.epoch = 0
        r.encoded_noise = table.sample()[0]
        r.reward = float(rewards[i])
        batch.append(r)
        idx.append(int(r.encoded_noise))
    upd = learner.step(batch, 0.25, 0, 0)
    g = learner.gradient_memory.copy()
    theta1 = pol.get_trainable_flat().copy()
    # second step: half the returns are one epoch stale -> lambda drift (finite_differences.py:88-89)
    rewards2 = rng.randn(N)
    batch2, idx2, ep2 = [], [], []
    for i in range(N):
        r = FDReturn()
        r.epoch = 0 if i % 2 else 1
        r.encoded_noise = table.sample()[0]
        r.reward = float(rewards2[i])
        batch2.append(r)
        idx2.append(int(r.encoded_noise))
        ep2.append(r.epoch)
    upd2 = learner.step(batch2, -0.5, 0, 0)
    return dict(theta0=theta0, idx=np.array(idx), rewards=rewards, update=np.array(upd), g=g, theta1=theta1,
                idx2=np.array(idx2), ep2=np.array(ep2), rewards2=rewards2, update2=np.array(upd2),
                g2=learner.gradient_memory.copy(), theta2=pol.get_trainable_flat().copy(),
                omega=np.array(omega_value))


def g4_fd_step():
    out = {}
    for name, N, om in (("cheetah", 16, 0.0), ("cheetah", 64, 0.5), ("trap", 16, 0.25)):
        kind, n_in, n_act = SHAPES[name]
        case = _fd_case(kind, n_in, n_act, N, om, seed=N)
        for k, v in case.items():
            out["%s_n%d_%s" % (name, N, k)] = v
    save("g4_fd_step.npz", **out)


def g5_trap():
    env = _trap_env()
    out = {"walkable": np.array([[n.walkable for n in row] for row in env.map.nodes], dtype=bool)}
    rets, cols, rows = [], [], []
    for a in range(9):
        env.reset()
        tot, done, steps = 0, False, 0
        while not done:
            _, r, done, _ = env.step(a)
            tot += r
            steps += 1
        rets.append(tot)
        cols.append(env.current_node.x // 7)
        rows.append(env.current_node.y // 7)
        assert steps == 201
    out["const_return"] = np.array(rets)
    out["const_col"] = np.array(cols)
    out["const_row"] = np.array(rows)
    out["start_obs"] = env.reset()
    # deterministic DiscretePolicy episodes through the reference Agent (worker/agent.py:20-71)
    for seed in (124, 1, 2):
        pol = make_policy("discrete", 2, 9, seed)
        agent = Agent(pol, env, random_seed=seed)
        rew, ent, steps = agent.collect_return(eval_run=True)
        out["det_s%d" % seed] = np.array([rew, ent, steps])
        out["det_s%d_theta" % seed] = pol.get_trainable_flat().copy()
    save("g5_trap.npz", **out)
    np.savez_compressed(os.path.join(HERE, "trap_map.npz"), walkable=out["walkable"])
    # the same bitmap ships with the product's GPU trap env (data, not code)
    np.savez_compressed(os.path.join(REPO, "dfd-starter_amd", "custom_envs", "simple_trap_env", "trap_map.npz"),
                        walkable=out["walkable"])


class _InjectedDiscrete(object):
    """Replaces DiscretePolicy.get_action: inverse CDF at a uniform from a fixed RandomState."""

    def __init__(self, seed):
        self.rng = np.random.RandomState(seed)

    def __call__(self, policy, x, deterministic=False):
        probs = policy.forward(x)
        if deterministic:
            return probs.argmax().item()
        from oracle.policies import categorical_inverse_cdf   # ours: the rule being pinned
        return categorical_inverse_cdf(probs[0].numpy(), np.float32(self.rng.uniform()))


class _InjectedNormal(object):
    def __init__(self, seed):
        self.rng = np.random.RandomState(seed)

    def __call__(self, policy, x, deterministic=False):
        mean, std = policy.forward(x)
        if deterministic:
            return mean.flatten().tolist()
        z = torch.as_tensor(self.rng.randn(mean.shape[-1]).astype(np.float32))
        return (mean + std * z).flatten().tolist()


def g6_runner_trap():
    """Patched SequentialRunner on the trap env, 2 epochs x batch 16."""
    _ENV_FACTORY["SimpleTrapEnv-v0"] = _trap_env
    inj = _InjectedDiscrete(777)
    orig_get_action = DiscretePolicy.get_action
    DiscretePolicy.get_action = lambda self, x, deterministic=False: inj(self, x, deterministic)
    orig_rng_src = run_sequential.RNGNoiseSource
    run_sequential.RNGNoiseSource = lambda n, random_seed=123: SharedNoiseTable(2 ** 22, n, random_seed)
    orig_update = Worker.update

    def update(self, state):                                 # SURVEY 8c patch (1)
        self.policy.set_trainable_flat(state.policy_params)
        self.epoch = state.epoch
        if state.obs_stats is not None:
            self.fixed_obs_stats.deserialize(state.obs_stats)
    Worker.update = update

    idx_log = []
    orig_sample = SharedNoiseTable.sample

    def sample(self):
        enc, noise = orig_sample(self)
        idx_log.append(int(enc))
        return enc, noise
    SharedNoiseTable.sample = sample
    step_log = []
    orig_step = FiniteDifferences.step

    def step(self, batch, pr, pn, pe):
        step_log.append(dict(rewards=[r.reward for r in batch], idx=[int(r.encoded_noise) for r in batch],
                             policy_reward=pr, omega=self.omega.omega))
        return orig_step(self, batch, pr, pn, pe)
    FiniteDifferences.step = step
    try:
        runner = run_sequential.SequentialRunner(env_id="SimpleTrapEnv-v0", batch_size=16, random_seed=124,
                                                 zeta_size=4, max_strategy_history_size=4)
        runner.learner.noise_std = 0.02                      # SURVEY 8c patch (2)
        theta0 = runner.policy.get_trainable_flat().copy()
        with contextlib.redirect_stdout(io.StringIO()) as buf:
            runner.train(2)
        report = buf.getvalue()
        theta = runner.policy.get_trainable_flat().copy()
        out = dict(theta0=theta0, theta_final=theta, sample_idx=np.array(idx_log),
                   cum_steps=np.array(runner.agent.cumulative_timesteps),
                   policy_reward=np.array(runner.policy_reward))
        for e, s in enumerate(step_log):
            out["e%d_rewards" % e] = np.array(s["rewards"])
            out["e%d_idx" % e] = np.array(s["idx"])
            out["e%d_policy_reward" % e] = np.array(s["policy_reward"])
            out["e%d_omega" % e] = np.array(s["omega"])
        mags = [float(l.split()[-1]) for l in report.splitlines() if l.startswith("Update Magnitude")]
        out["update_magnitude_printed"] = np.array(mags)
        save("g6_runner_trap.npz", **out)
    finally:
        DiscretePolicy.get_action = orig_get_action
        run_sequential.RNGNoiseSource = orig_rng_src
        Worker.update = orig_update
        SharedNoiseTable.sample = orig_sample
        FiniteDifferences.step = orig_step


def g7_worker_synthetic():
    """Reference Worker/Agent on the build's synthetic envs with injected noise (episode loop)."""
    out = {}
    for name, (kind, n_in, n_act), T in (("cheetah", SHAPES["cheetah"], 60), ("cartpole", SHAPES["cartpole"], 50)):
        env = SyntheticEnv(n_in, n_act, kind == "discrete", T, env_seed=0)
        pol = make_policy(kind, n_in, n_act, 124)
        P = pol.num_params
        cls = DiscretePolicy if kind == "discrete" else MujocoPolicy
        inj = _InjectedDiscrete(31) if kind == "discrete" else _InjectedNormal(31)
        orig = cls.get_action
        cls.get_action = lambda self, x, deterministic=False: inj(self, x, deterministic)
        try:
            table = SharedNoiseTable(2 ** 22, P, random_seed=124)
            agent = Agent(pol, env, random_seed=11)
            handler = StrategyHandler(pol, math_helpers.categorical_tvd)
            worker = Worker(pol, agent, table, handler, sigma=0.02, eval_prob=0.25, random_seed=3)
            rets = worker.collect_returns(8)
        finally:
            cls.get_action = orig
        out[name + "_theta"] = pol.get_trainable_flat().copy()
        out[name + "_reward"] = np.array([r.reward for r in rets])
        out[name + "_entropy"] = np.array([r.entropy for r in rets])
        out[name + "_timesteps"] = np.array([r.timesteps for r in rets])
        out[name + "_is_eval"] = np.array([r.is_eval for r in rets])
        out[name + "_idx"] = np.array([int(r.encoded_noise) for r in rets])
        out[name + "_T"] = np.array(T)
    save("g7_worker_synthetic.npz", **out)


TERM_ENVS = {"cartpole_term": (("discrete", 4, 2), 500, 0.4, 1), "hopper_term": (("mujoco", 11, 3), 1000, 0.5, 1)}


def g13_worker_terminating():
    """Reference Worker/Agent on TERMINATING synthetic envs (episodes end before T: worker/agent.py:35-52) with
    injected draws, as G7: per-episode steps, rewards over the steps taken, entropy over the visited states, and
    the Agent's cumulative_timesteps (agent.py:55).  The envs are the build's (oracle/envs.py, done_threshold)."""
    out = {}
    for name, ((kind, n_in, n_act), T, thr, dim) in TERM_ENVS.items():
        env = SyntheticEnv(n_in, n_act, kind == "discrete", T, env_seed=0, done_threshold=thr, done_dim=dim)
        pol = make_policy(kind, n_in, n_act, 124)
        P = pol.num_params
        cls = DiscretePolicy if kind == "discrete" else MujocoPolicy
        inj = _InjectedDiscrete(31) if kind == "discrete" else _InjectedNormal(31)
        orig = cls.get_action
        cls.get_action = lambda self, x, deterministic=False: inj(self, x, deterministic)
        try:
            table = SharedNoiseTable(2 ** 22, P, random_seed=124)
            agent = Agent(pol, env, random_seed=11)
            handler = StrategyHandler(pol, math_helpers.categorical_tvd)
            worker = Worker(pol, agent, table, handler, sigma=0.02, eval_prob=0.25, random_seed=3)
            rets = worker.collect_returns(12)
        finally:
            cls.get_action = orig
        out[name + "_theta"] = pol.get_trainable_flat().copy()
        out[name + "_reward"] = np.array([r.reward for r in rets])
        out[name + "_entropy"] = np.array([r.entropy for r in rets])
        out[name + "_timesteps"] = np.array([r.timesteps for r in rets])
        out[name + "_is_eval"] = np.array([r.is_eval for r in rets])
        out[name + "_idx"] = np.array([int(r.encoded_noise) for r in rets])
        out[name + "_T"] = np.array(T)
        out[name + "_done"] = np.array([thr, dim], np.float64)
        out[name + "_cumulative_timesteps"] = np.array(agent.cumulative_timesteps)
    save("g13_worker_terminating.npz", **out)


def g8_impala():
    """G3 for the ImpalaCNN (policies/impala.py:48-186): reference module, B=1 sequences.

    Params = 0.1 * table slice (seed 7, size 2^22) so they need not be committed; BN running stats
    are set to non-trivial values so the eval-mode BN folding is exercised.  Two env sequences of
    3 steps each (B=1 per call, the reference's own usage -- with B>1 its done-mask uses env 0's
    flag for every env), one with a mid-sequence done.  Also the entropy pass of worker/agent.py:66
    (all visited obs as one batch through the end-of-episode LSTM state)."""
    from policies.impala import ImpalaCNN
    A = 6
    torch.manual_seed(124)
    net = ImpalaCNN(A, use_lstm=True)
    net.eval()
    P = sum(p.numel() for p in net.parameters())
    rs = np.random.RandomState(7)
    table = rs.randn(2 ** 22).astype(np.float32)
    flat = (table[1000:1000 + P] * np.float32(0.1)).astype(np.float32)
    with torch.no_grad():
        torch.nn.utils.vector_to_parameters(torch.as_tensor(flat), net.parameters())
        bns = [m for m in net.modules() if isinstance(m, (torch.nn.BatchNorm1d, torch.nn.BatchNorm2d))]
        nbn = sum(m.num_features for m in bns)
        rm = (table[2000000:2000000 + nbn] * np.float32(0.1)).astype(np.float32)
        rv = (1.0 + 0.5 * np.abs(table[3000000:3000000 + nbn])).astype(np.float32)
        off = 0
        for m in bns:
            n = m.num_features
            m.running_mean.copy_(torch.as_tensor(rm[off:off + n]))
            m.running_var.copy_(torch.as_tensor(rv[off:off + n]))
            off += n
    feats = []
    hook = net.fc[0].register_forward_hook(lambda mod, inp, out: feats.append(inp[0].detach().clone()))
    frng = np.random.RandomState(5)
    n_seq, T = 2, 3
    frames = frng.randint(0, 256, size=(n_seq, T, 3, 64, 64)).astype(np.float32)
    rewards = np.array([[0.0, 2.5, -0.25], [0.0, -3.0, 0.75]], np.float32)
    dones = np.array([[False, False, False], [False, True, False]])
    probs = np.zeros((n_seq, T, A), np.float32)
    hs = np.zeros((n_seq, T, 256), np.float32)
    cs = np.zeros((n_seq, T, 256), np.float32)
    feat = np.zeros((n_seq, T, 2048), np.float32)
    ent_probs = np.zeros((n_seq, T, A), np.float32)
    with torch.no_grad():
        for q in range(n_seq):
            net.state = net.initial_state()
            for t in range(T):
                obs = {"frame": torch.as_tensor(frames[q, t]).view(1, 1, 3, 64, 64),
                       "reward": torch.as_tensor(rewards[q, t]).view(1, 1),
                       "done": torch.as_tensor(bool(dones[q, t])).view(1, 1)}
                logits = net(obs)
                probs[q, t] = torch.softmax(logits, dim=-1).view(-1).numpy()
                hs[q, t] = net.state[0].view(-1).numpy()
                cs[q, t] = net.state[1].view(-1).numpy()
                feat[q, t] = feats[-1].view(-1).numpy()
            # entropy pass: every visited obs, one batch, through the end-of-sequence state
            batch = {"frame": torch.as_tensor(frames[q]).view(T, 1, 3, 64, 64),
                     "reward": torch.as_tensor(rewards[q]).view(T, 1),
                     "done": torch.as_tensor(np.zeros(T, bool)).view(T, 1)}
            ent_probs[q] = torch.softmax(net(batch), dim=-1).view(T, A).numpy()
    hook.remove()
    save("g8_impala.npz", A=np.array(A), P=np.array(P), table_seed=np.array(7), param_offset=np.array(1000),
         rm=rm, rv=rv, frames=frames.astype(np.uint8), rewards=rewards, dones=dones, probs=probs, h=hs, c=cs,
         feat=feat, ent_probs=ent_probs,
         param_shapes=np.array([str(tuple(p.shape)) for p in net.parameters()]))


def g9_novelty():
    """Strategy distances / novelty (utils/math_helpers.py:147-222) on seeded strategies."""
    rs = np.random.RandomState(9)
    out = {}
    Z, A, K, H = 7, 5, 3, 6
    p = rs.rand(Z, A).astype(np.float32); p /= p.sum(-1, keepdims=True)
    P = rs.rand(H, Z, A).astype(np.float32); P /= P.sum(-1, keepdims=True)
    g = np.concatenate([rs.randn(Z, K), 0.1 + rs.rand(Z, K)], -1).astype(np.float32)
    G = np.concatenate([rs.randn(H, Z, K), 0.1 + rs.rand(H, Z, K)], -1).astype(np.float32)
    out.update(cat_a=p, cat_b=P, gau_a=g, gau_b=G)
    out["tvd"] = np.asarray(math_helpers.categorical_tvd(p, P))
    out["l2"] = np.asarray(math_helpers.l2_dist(p, P))
    out["w2"] = np.asarray(math_helpers.gaussian_wasserstein_dist_from_strategies(g, G))
    out["nov_tvd"] = np.asarray(math_helpers.compute_strategy_novelty(p, P, distance_fn=math_helpers.categorical_tvd))
    out["nov_l2"] = np.asarray(math_helpers.compute_strategy_novelty(p, P))
    out["nov_w2"] = np.asarray(math_helpers.compute_strategy_novelty(
        g, G, distance_fn=math_helpers.gaussian_wasserstein_dist_from_strategies))
    # pairwise archive distances as SparseHistoryManager._construct_table computes them (:55-66)
    out["pair_tvd"] = np.array([[math_helpers.compute_strategy_distance(P[i], P[j], distance_fn=math_helpers.categorical_tvd)
                                 for j in range(H)] for i in range(H)])
    save("g9_novelty.npz", **out)


def g10_welford():
    """WelfordRunningStat (utils/math_helpers.py:7-124): sequential updates, std/mean properties and the
    increment_from_obs_stats_update merge that run_server.py:143 applies to every return."""
    rs = np.random.RandomState(10)
    d = 5
    parts = []
    for n in (0, 1, 3, 7, 12):
        w = math_helpers.WelfordRunningStat(d)
        xs = (rs.randn(n, d) * 3 + 1).astype(np.float32)
        for x in xs:
            w.increment(x, 1)
        parts.append((xs, w.serialize()))
    acc = math_helpers.WelfordRunningStat(d)
    for _, ser in parts:
        acc.increment_from_obs_stats_update(ser)
    out = {"d": np.array(d)}
    for i, (xs, ser) in enumerate(parts):
        out["x%d" % i] = xs
        out["ser%d" % i] = np.asarray(ser, np.float64)
    out["acc_ser"] = np.asarray(acc.serialize(), np.float64)
    out["acc_mean"] = np.asarray(acc.mean, np.float32)
    out["acc_std"] = np.asarray(acc.std, np.float32)
    save("g10_welford.npz", **out)


def g11_atari():
    """AtariPolicy (policies/atari.py:7-51): normc init fingerprint (policy.py:88-115 over conv, BN and
    linear weights) and eval-mode forwards.  The reference's Policy.forward views non-tensor input with
    a tuple input_shape (policy.py:27-28), which torch rejects, so the forward is fed tensors."""
    from policies import AtariPolicy
    A = 6
    torch.manual_seed(124)
    pol = AtariPolicy((84, 84), A, seed=124)
    flat = pol.get_trainable_flat().copy()
    P = flat.size
    rs = np.random.RandomState(11)
    # forward at the (normc) init theta: every layer with a weight is normc'd and its bias zeroed, so
    # theta depends on RandomState(seed) only and the oracle can rebuild it
    bns = [m for m in pol.model if isinstance(m, (torch.nn.BatchNorm1d, torch.nn.BatchNorm2d))]
    nbn = sum(m.num_features for m in bns)
    scale = np.concatenate([np.full(16, 3e3), np.full(32, 3e2), np.full(256, 1.0)]).astype(np.float32)
    rm = (rs.randn(nbn) * scale).astype(np.float32)
    rv = ((1.0 + rs.rand(nbn)) * scale * scale).astype(np.float32)
    off = 0
    with torch.no_grad():
        for m in bns:
            n = m.num_features
            m.running_mean.copy_(torch.as_tensor(rm[off:off + n]))
            m.running_var.copy_(torch.as_tensor(rv[off:off + n]))
            off += n
    frames = rs.randint(0, 256, size=(5, 4, 84, 84)).astype(np.float32)
    feats = []
    hook = pol.model[7].register_forward_hook(lambda mod, inp, out: feats.append(inp[0].detach().clone()))
    with torch.no_grad():
        probs = pol.forward(torch.as_tensor(frames)).numpy()
    hook.remove()
    save("g11_atari.npz", A=np.array(A), P=np.array(P), init_sha=np.array(sha(flat)), init_head=flat[:64],
         init_tail=flat[-64:], init_sum=np.array(float(np.float64(flat).sum())), rm=rm, rv=rv,
         frames=frames.astype(np.uint8), probs=probs, feat=feats[0].numpy(),
         param_shapes=np.array([str(tuple(p.shape)) for p in pol.parameters()]))


def g12_history():
    """SparseHistoryManager replacement (strategy/sparse_history_manager.py:17-148 via StrategyHandler): a
    DiscretePolicy (categorical_tvd) and a MujocoPolicy (gaussian_wasserstein_dist_from_strategies) archive of
    6 points, filled, evaluated on zeta, then 14 more submit_policy calls that replace -- or not -- the less
    novel member of the closest pair.  Records every submission's return value and worst_point_idx, the final
    strategy tensor and the known-distance table."""
    out = {}
    rs = np.random.RandomState(12)
    table = rs.randn(1 << 20).astype(np.float32)
    for tag, Pol, n_in, n_act, dist in (("disc", DiscretePolicy, 4, 2, math_helpers.categorical_tvd),
                                        ("mj", MujocoPolicy, 17, 6,
                                         math_helpers.gaussian_wasserstein_dist_from_strategies)):
        torch.manual_seed(124)
        pol = Pol(n_in, n_act, seed=124)
        theta = pol.get_trainable_flat().copy()
        P = theta.size
        H, N = 6, 20
        scales = rs.choice([0.02, 0.05, 0.1, 0.2, 0.4], size=N).astype(np.float32)
        offs = rs.randint(0, table.size - P, size=N)
        flats = np.stack([(theta + scales[k] * table[offs[k]:offs[k] + P]).astype(np.float32) for k in range(N)])
        zeta = rs.randn(10, n_in).astype(np.float32)
        handler = StrategyHandler(pol, dist, max_history_size=H)
        mgr = handler.strategy_history_manager
        for k in range(H):
            pol.set_trainable_flat(flats[k])
            handler.add_policy(pol)
        handler.set_zeta(zeta)
        worst = [mgr.worst_point_idx]
        rets = []
        for k in range(H, N):
            pol.set_trainable_flat(flats[k])
            r = mgr.submit_policy(pol)
            rets.append(-2 if r is None else int(r))
            worst.append(mgr.worst_point_idx)
        D = np.full((H, H), np.inf)
        for (i, j), d in mgr.known_dists.items():
            D[i, j] = D[j, i] = d
        out.update({tag + "_flats": flats, tag + "_zeta": zeta, tag + "_returns": np.array(rets),
                    tag + "_worst": np.array(worst), tag + "_strategies": np.asarray(mgr.strategy_tensor, np.float32),
                    tag + "_dists": D, tag + "_H": np.array(H)})
    save("g12_history.npz", **out)


def g12_impala(patched=True):
    """G12 for ImpalaPolicy (config 5's archive): the reference StrategyHandler / SparseHistoryManager
    (strategy/strategy_handler.py:6-31, sparse_history_manager.py:17-148) over a reference ImpalaPolicy
    (policies/impala.py:8-45) with categorical_tvd -- 6 points added, zeta set (8 obs dicts), 14 more
    submit_policy calls.  Harness patch: ImpalaPolicy.get_strategy resets the LSTM state first, the build's
    documented zero-state rule (StrategyPoint.evaluate_strategy would otherwise start
    each point from the state the previous call left in the shared policy object, policies/impala.py:24-27).
    The parameter vectors are not committed (4.6 MB each): theta = 0.1 * table[1000:], point k =
    theta + scale_k * table[off_k:] with table = RandomState(7).randn(2^22) f32; BN running stats as G8.
    patched=False (g12_impala_unpatched.npz): the same run with the reference's get_strategy as it is, so the
    size of the zero-state rule's divergence from the reference's carried-over LSTM state is recorded."""
    from policies.impala import ImpalaPolicy
    A, H, N, Z = 4, 6, 20, 8
    orig = ImpalaPolicy.get_strategy

    def get_strategy_from_reset(self, x):
        self.reset()
        return orig(self, x)

    if patched:
        ImpalaPolicy.get_strategy = get_strategy_from_reset
    try:
        torch.manual_seed(124)
        pol = ImpalaPolicy((64, 64, 3), A, seed=124)
        P = pol.num_params
        rs = np.random.RandomState(7)
        table = rs.randn(2 ** 22).astype(np.float32)
        theta = (table[1000:1000 + P] * np.float32(0.1)).astype(np.float32)
        bns = [m for m in pol.modules() if isinstance(m, (torch.nn.BatchNorm1d, torch.nn.BatchNorm2d))]
        nbn = sum(m.num_features for m in bns)
        rm = (table[2000000:2000000 + nbn] * np.float32(0.1)).astype(np.float32)
        rv = (1.0 + 0.5 * np.abs(table[3000000:3000000 + nbn])).astype(np.float32)
        with torch.no_grad():
            o = 0
            for m in bns:
                n = m.num_features
                m.running_mean.copy_(torch.as_tensor(rm[o:o + n]))
                m.running_var.copy_(torch.as_tensor(rv[o:o + n]))
                o += n
        prs = np.random.RandomState(12)
        scales = prs.choice([0.02, 0.05, 0.1, 0.2, 0.4], size=N).astype(np.float32)
        offs = prs.randint(0, table.size - P, size=N)
        frames = prs.randint(0, 256, size=(Z, 3, 64, 64)).astype(np.uint8)
        zrew = prs.choice([-1.0, 0.0, 1.0], size=Z).astype(np.float32)
        zeta = [{"frame": torch.as_tensor(frames[z].astype(np.float32)).view(1, 1, 3, 64, 64),
                 "reward": torch.as_tensor(zrew[z]).view(1, 1),
                 "done": torch.as_tensor(False).view(1, 1)} for z in range(Z)]
        handler = StrategyHandler(pol, math_helpers.categorical_tvd, max_history_size=H)
        mgr = handler.strategy_history_manager
        for k in range(H):
            pol.set_trainable_flat((theta + scales[k] * table[offs[k]:offs[k] + P]).astype(np.float32))
            handler.add_policy(pol)
        handler.set_zeta(zeta)
        worst, rets = [mgr.worst_point_idx], []
        for k in range(H, N):
            pol.set_trainable_flat((theta + scales[k] * table[offs[k]:offs[k] + P]).astype(np.float32))
            r = mgr.submit_policy(pol)
            rets.append(-2 if r is None else int(r))
            worst.append(mgr.worst_point_idx)
        D = np.full((H, H), np.inf)
        for (i, j), d in mgr.known_dists.items():
            D[i, j] = D[j, i] = d
        # novelty of two more policies against the final archive (strategy_handler.py:26-31)
        nov = []
        for k in (0, N - 1):
            pol.set_trainable_flat((theta - scales[k] * table[offs[k]:offs[k] + P]).astype(np.float32))
            nov.append(handler.compute_novelty(pol))
    finally:
        ImpalaPolicy.get_strategy = orig
    save("g12_impala.npz" if patched else "g12_impala_unpatched.npz", A=np.array(A), H=np.array(H), P=np.array(P), table_seed=np.array(7),
         param_offset=np.array(1000), rm=rm, rv=rv, scales=scales, offs=offs, zeta_frames=frames, zeta_rewards=zrew,
         returns=np.array(rets), worst=np.array(worst), strategies=np.asarray(mgr.strategy_tensor, np.float32),
         dists=D, novelty=np.array(nov))


def g14_impala_vbn():
    """ImpalaPolicy.compute_vbn (policies/impala.py:12-16; called every epoch by run_sequential.py:156-157 with
    the VBN buffer of :198-213): the stacked buffer (B = n obs, T = 1) runs through ImpalaCNN in train mode, so
    every BatchNorm normalises with its batch statistics and folds them into its running stats, and the
    batch_first LSTM reads the n obs as ONE sequence from the carried self.state, masked by the FIRST obs' done
    flag (impala.py:165-176), leaving self.state at the sequence end (:184).  Params / initial running stats as
    G8 (0.1 * table[1000:], table = RandomState(7).randn(2^22)).  Cases, each from the same starting running
    stats and carried state (h0, c0):
      a  done[0] = False            (the carried state enters the sequence)
      b  done[0] = True             (the state is zeroed first)
      a2 case a, then compute_vbn again on the same buffer (stats and state chained)
    Records every BN running_mean / running_var (modules() order) and self.state after each case."""
    from policies.impala import ImpalaPolicy
    A, N = 6, 16
    torch.manual_seed(124)
    pol = ImpalaPolicy((64, 64, 3), A, seed=124)
    P = pol.num_params
    rs = np.random.RandomState(7)
    table = rs.randn(2 ** 22).astype(np.float32)
    flat = (table[1000:1000 + P] * np.float32(0.1)).astype(np.float32)
    pol.set_trainable_flat(flat)
    net = pol.model[0]
    bns = [m for m in pol.modules() if isinstance(m, (torch.nn.BatchNorm1d, torch.nn.BatchNorm2d))]
    nbn = sum(m.num_features for m in bns)
    rm = (table[2000000:2000000 + nbn] * np.float32(0.1)).astype(np.float32)
    rv = (1.0 + 0.5 * np.abs(table[3000000:3000000 + nbn])).astype(np.float32)
    brs = np.random.RandomState(14)
    frames = brs.randint(0, 256, size=(N, 3, 64, 64)).astype(np.uint8)
    rewards = brs.choice([-2.0, -1.0, -0.5, 0.0, 0.25, 1.0, 3.0], size=N).astype(np.float32)
    dones = brs.rand(N) < 0.25
    h0 = (0.5 * brs.randn(256)).astype(np.float32)
    c0 = (0.5 * brs.randn(256)).astype(np.float32)

    def set_stats():
        with torch.no_grad():
            o = 0
            for m in bns:
                n = m.num_features
                m.running_mean.copy_(torch.as_tensor(rm[o:o + n]))
                m.running_var.copy_(torch.as_tensor(rv[o:o + n]))
                m.num_batches_tracked.zero_()
                o += n
        net.state = (torch.as_tensor(h0).view(1, 1, 256).clone(), torch.as_tensor(c0).view(1, 1, 256).clone())

    def buffer(first_done):
        d = dones.copy()
        d[0] = first_done
        return [{"frame": torch.as_tensor(frames[i].astype(np.float32)).view(1, 1, 3, 64, 64),
                 "reward": torch.as_tensor(rewards[i]).view(1, 1),
                 "done": torch.as_tensor(bool(d[i])).view(1, 1)} for i in range(N)], d

    def record(tag, out):
        out[tag + "_rm"] = torch.cat([m.running_mean for m in bns]).numpy().copy()
        out[tag + "_rv"] = torch.cat([m.running_var for m in bns]).numpy().copy()
        out[tag + "_h"] = net.state[0].reshape(-1).numpy().copy()
        out[tag + "_c"] = net.state[1].reshape(-1).numpy().copy()

    out = {}
    with torch.no_grad():
        for tag, first_done in (("a", False), ("b", True)):
            set_stats()
            buf, d = buffer(first_done)
            pol.compute_vbn(buf)
            assert not pol.training
            record(tag, out)
            out[tag + "_dones"] = d
            if tag == "a":
                pol.compute_vbn(buf)
                record("a2", out)
    save("g14_impala_vbn.npz", A=np.array(A), P=np.array(P), N=np.array(N), table_seed=np.array(7),
         param_offset=np.array(1000), rm=rm, rv=rv, frames=frames, rewards=rewards, h0=h0, c0=c0,
         momentum=np.array(0.1), **out)


def g16_atari_vbn():
    """AtariPolicy.compute_vbn (policy.py:31-34: train(); forward(buffer); eval()) over a VBN buffer of N = 12
    stacked-frame obs, fed as a tensor (policy.py:27-28's tuple view is rejected by torch, as in G11): every
    BatchNorm (2d(16), 2d(32), 1d(256)) normalises with its batch statistics and folds them into its running stats.
    theta = 0.05 * RandomState(16).randn(P) (f32), running stats as G11's scales; records the running stats after
    one call (a) and after a second call on the same buffer (a2)."""
    from policies import AtariPolicy
    A, N = 6, 12
    torch.manual_seed(124)
    pol = AtariPolicy((84, 84), A, seed=124)
    P = pol.num_params
    flat = (np.random.RandomState(16).randn(P) * 0.05).astype(np.float32)
    pol.set_trainable_flat(flat)
    rs = np.random.RandomState(116)
    bns = [m for m in pol.model if isinstance(m, (torch.nn.BatchNorm1d, torch.nn.BatchNorm2d))]
    nbn = sum(m.num_features for m in bns)
    scale = np.concatenate([np.full(16, 3e1), np.full(32, 1e1), np.full(256, 1.0)]).astype(np.float32)
    rm = (rs.randn(nbn) * scale).astype(np.float32)
    rv = ((1.0 + rs.rand(nbn)) * scale * scale).astype(np.float32)
    frames = rs.randint(0, 256, size=(N, 4, 84, 84)).astype(np.uint8)
    off = 0
    with torch.no_grad():
        for m in bns:
            n = m.num_features
            m.running_mean.copy_(torch.as_tensor(rm[off:off + n]))
            m.running_var.copy_(torch.as_tensor(rv[off:off + n]))
            off += n
    out = {}
    with torch.no_grad():
        for tag in ("a", "a2"):
            pol.compute_vbn(torch.as_tensor(frames.astype(np.float32)))
            assert not pol.training
            out[tag + "_rm"] = torch.cat([m.running_mean for m in bns]).numpy().copy()
            out[tag + "_rv"] = torch.cat([m.running_var for m in bns]).numpy().copy()
    save("g16_atari_vbn.npz", A=np.array(A), P=np.array(P), N=np.array(N), param_seed=np.array(16),
         param_scale=np.array(0.05), rm=rm, rv=rv, frames=frames, momentum=np.array(0.1), **out)


def _patch_rng_noise_source():
    """SURVEY finding 3: RNGNoiseSource reads Generator.__getstate__(), which returns None on numpy >= 2; the
    harness patch reads / writes bit_generator.state instead -- otherwise the reference's code as it is
    (utils/noise_sources.py:4-20: sample() reports the PCG64 state, then draws; decode() restores it and redraws)."""
    from utils import noise_sources as ns
    cls = ns.RNGNoiseSource
    orig = (cls.__init__, cls.sample, cls.decode)

    def __init__(self, n_params, random_seed=123):
        self.rng = np.random.default_rng(np.random.SeedSequence(random_seed))
        self.base_state = self.rng.bit_generator.state
        self.n_params = n_params

    def sample(self):
        st = self.rng.bit_generator.state
        state = "{},{}".format(st['state']['state'], st['state']['inc'])
        noise = self.rng.standard_normal(size=self.n_params)
        return state, noise

    def decode(self, state):
        state_data = state.split(",")
        self.base_state['state']['state'] = int(state_data[0])
        self.base_state['state']['inc'] = int(state_data[1])
        self.rng.bit_generator.state = self.base_state
        return self.rng.standard_normal(size=self.n_params)
    cls.__init__, cls.sample, cls.decode = __init__, sample, decode
    return cls, orig


def g15_rng_noise_source():
    """The reference's DEFAULT noise source (run_sequential.py:89: RNGNoiseSource, one noise source object shared
    by the Worker and the learner) through Worker.collect_returns + FiniteDifferences.step, two epochs, with the
    finding-3 patch and injected action draws as G7: every return's encoded PCG64 state, reward, entropy, steps,
    eval flag; the learner's update magnitude, gradient and theta after each step."""
    from utils.noise_sources import RNGNoiseSource
    cls, orig = _patch_rng_noise_source()
    out = {}
    try:
        for name, (kind, n_in, n_act), T in (("cheetah", SHAPES["cheetah"], 40), ("cartpole", SHAPES["cartpole"], 30)):
            env = SyntheticEnv(n_in, n_act, kind == "discrete", T, env_seed=0)
            pol = make_policy(kind, n_in, n_act, 124)
            P = pol.num_params
            pcls = DiscretePolicy if kind == "discrete" else MujocoPolicy
            inj = _InjectedDiscrete(31) if kind == "discrete" else _InjectedNormal(31)
            orig_act = pcls.get_action
            pcls.get_action = lambda self, x, deterministic=False: inj(self, x, deterministic)
            try:
                src = RNGNoiseSource(P, random_seed=5)
                agent = Agent(pol, env, random_seed=11)
                handler = StrategyHandler(pol, math_helpers.categorical_tvd)
                worker = Worker(pol, agent, src, handler, sigma=0.02, eval_prob=0.25, random_seed=3)
                opt = DSGD(pol.parameters(), lr=0.01)
                omega = AdaptiveOmega()
                learner = FiniteDifferences(pol, opt, omega, src, noise_std=0.02, batch_size=8, max_delayed_return=10)
                out[name + "_theta0"] = pol.get_trainable_flat().copy()
                for e in range(2):
                    worker.epoch = learner.epoch          # what run_sequential.py:168's worker.update(state) sets
                    rets = worker.collect_returns(8)
                    train = [r for r in rets if not r.is_eval]
                    pre = "%s_e%d_" % (name, e)
                    out[pre + "reward"] = np.array([r.reward for r in rets])
                    out[pre + "entropy"] = np.array([r.entropy for r in rets])
                    out[pre + "timesteps"] = np.array([r.timesteps for r in rets])
                    out[pre + "is_eval"] = np.array([r.is_eval for r in rets])
                    out[pre + "encoded"] = np.array([str(r.encoded_noise) for r in rets])
                    out[pre + "update"] = np.array(learner.step(train, 0.25 * e, 0, 0))
                    out[pre + "g"] = learner.gradient_memory.copy()
                    out[pre + "theta"] = pol.get_trainable_flat().copy()
            finally:
                pcls.get_action = orig_act
            out[name + "_T"] = np.array(T)
    finally:
        cls.__init__, cls.sample, cls.decode = orig
    save("g15_rng_noise_source.npz", **out)


GENERATORS = {"g16": g16_atari_vbn, "g15": g15_rng_noise_source, "g1": g1_noise, "g2": g2_perturb, "g3": g3_forward, "g4": g4_fd_step, "g5": g5_trap,
              "g6": g6_runner_trap, "g7": g7_worker_synthetic, "g13": g13_worker_terminating, "g8": g8_impala,
              "g9": g9_novelty, "g10": g10_welford, "g11": g11_atari, "g12": g12_history,
              "g12i": g12_impala, "g12iu": lambda: g12_impala(patched=False), "g14": g14_impala_vbn}

if __name__ == "__main__":
    torch.set_num_threads(1)
    for name in (sys.argv[1:] or sorted(GENERATORS)):
        GENERATORS[name]()
