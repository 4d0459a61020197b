"""FD learner restatement: return weighting, noise-weighted gradient, DSGD update.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

  standardize      utils/math_helpers.py:127-134  (f64, population std, unchanged if std == 0)
  affine_transform utils/math_helpers.py:137-144
  lambda / v       learner/finite_differences.py:80-114
                   lambda_i = fl32(eps_i * fl32(sigma)) [* sign_i] + dist_map[epoch_i]
                   v_i = lambda_i / (||lambda_i|| ** 2)            (f32)
  gradient         learner/finite_differences.py:40-49   g = standardize(r - r_pol) . V   (f64;
                   the "/ len(batch)" on :49 is discarded by the reference and so here too)
  DSGD             dsgd/dynamic_sgd.py:19-51 + policies/policy.py:63-70
                   grad = fl32(-g); coef = lr * sqrt(P) * lr_scale / ||grad||;
                   theta <- fl32(theta - fl32(fl32(coef) * grad))
  update size      learner/finite_differences.py:54-59   ||theta_old - theta_new||
  policy history   learner/finite_differences.py:66-78   (delayed-return drift)
"""
import numpy as np
import torch


def standardize(x):
    x = np.asarray(x, dtype=np.float64)
    m, s = x.mean(), x.std()
    if s == 0:
        return x
    return (x - m) / s


def affine_transform(value, from_min, from_max, to_min, to_max):
    if from_max == from_min or to_max == to_min:
        return to_min
    return (value - from_min) * (to_max - to_min) / (from_max - from_min) + to_min


def perturbation_vectors(table, P, idx, sign, sigma, drift=None):
    """V [N, P] f32 rows v_i = lambda_i / ||lambda_i||^2, and the squared norms (f32)."""
    s32 = np.float32(sigma)
    V = np.empty((len(idx), P), dtype=np.float32)
    n2 = np.empty(len(idx), dtype=np.float64)
    for i, (ix, sg) in enumerate(zip(idx, sign)):
        lam = (table[int(ix):int(ix) + P] * s32).astype(np.float32)
        if sg < 0:
            lam = -lam
        if drift is not None and drift[i] is not None:
            lam = (lam + drift[i]).astype(np.float32)
        nrm = np.linalg.norm(lam)
        n2[i] = float(nrm) * float(nrm)
        V[i] = lam / (nrm * nrm)
    return V, n2


def fd_gradient(table, P, idx, sign, rewards, policy_reward, sigma, drift=None):
    V, _ = perturbation_vectors(table, P, idx, sign, sigma, drift)
    z = standardize(np.subtract(rewards, policy_reward))
    g = np.dot(z, V)
    return g, z


def centred_ranks(x):
    """Centred-rank weights (build extension; the standard ES transform -- the reference's weighting is the
    z-score): rank of x_i among all returns, ties broken by index (stable sort), / (n - 1) - 0.5."""
    x = np.asarray(x, dtype=np.float64)
    n = x.size
    r = np.empty(n, dtype=np.float64)
    r[np.argsort(x, kind="stable")] = np.arange(n)
    return r / (n - 1) - 0.5 if n > 1 else np.zeros(n)


def fd_gradient_weights(table, P, idx, sign, weights, sigma):
    """g = sum_i w_i v_i for given per-return weights (the centred-rank form of fd_gradient)."""
    V, _ = perturbation_vectors(table, P, idx, sign, sigma)
    return np.dot(np.asarray(weights, np.float64), V)


def fd_moments(table, P, idx, sign, rewards, policy_reward, sigma, lane_lo=0, n_all=None, lanes_per_dir=1):
    """One rank's share of the one-collective z-score step: [A | B | n_local | r' slots [n_all]] with
    r' = r - policy_reward, A = sum r'_i v_i, B = sum v_i (f64); this rank's r' sit at its global lanes
    [lane_lo, lane_lo + n_local), zeros elsewhere, so the all-reduce's sum holds every lane's r'.
    A is accumulated per direction as sum_k (r'_k - r'_0) v_k + r'_0 sum_k v_k (the build's fdr_fd_grad_fused
    order: for an antithetic pair sum_k v_k = 0 exactly and the near-constant-return products do not cancel)."""
    V, _ = perturbation_vectors(table, P, idx, sign, sigma)
    V = V.astype(np.float64)
    r = np.subtract(rewards, policy_reward).astype(np.float64)
    R = r.reshape(-1, lanes_per_dir)
    VB = V.reshape(R.shape[0], lanes_per_dir, P).sum(1)
    A = np.dot((R - R[:, :1]).reshape(-1), V) + np.dot(R[:, 0], VB)
    n_all = r.size + lane_lo if n_all is None else n_all
    slots = np.zeros(n_all)
    slots[lane_lo:lane_lo + r.size] = r
    return np.concatenate([A, VB.sum(0), [float(r.size)], slots])


def grad_from_moments(mom, P):
    """g = (A - m B) / sd from summed moments; m, sd over the r' slots as standardize (utils/math_helpers.py:127-134:
    two-pass, population std; sd == 0: A, as standardize returns its input unchanged)."""
    A, B = mom[:P], mom[P:2 * P]
    n = int(mom[2 * P])
    r = mom[2 * P + 1:2 * P + 1 + n]
    m, sd = r.mean(), r.std()
    return A if sd == 0 else (A - m * B) / sd


def dsgd_step(theta, g, lr, omega=0.0, omega_min=0.0, omega_max=1.0, min_scale=0.23, max_scale=1.0):
    theta = torch.as_tensor(np.asarray(theta, dtype=np.float32)).clone()
    P = theta.numel()
    lr_scale = affine_transform(omega, omega_min, omega_max, min_scale, max_scale)
    grad = torch.as_tensor(-np.asarray(g, dtype=np.float64), dtype=torch.float32)
    norm = grad.norm().item()
    assert norm > 0, "DSGD ENCOUNTERED GRADIENT WITH NORM OF ZERO"
    coef = lr * np.sqrt(P) * lr_scale / norm
    new = theta - coef * grad
    old = theta.numpy()
    update = float(np.linalg.norm(old - new.numpy()))
    return new.numpy(), update


class FDLearner(object):
    """finite_differences.FiniteDifferences restated (epoch bookkeeping + drift map)."""

    def __init__(self, theta, table, P, noise_std, lr, max_delayed_return=10):
        self.theta = np.asarray(theta, dtype=np.float32).copy()
        self.table, self.P = table, P
        self.noise_std, self.lr = noise_std, lr
        self.max_delayed_return = max_delayed_return
        self.history = [(self.theta.copy(), 0)]
        self.epoch = 0
        self.dist_map = {0: None}
        self.discarded = 0

    def step(self, epochs, idx, sign, rewards, policy_reward, omega=0.0, omega_min=0.0, omega_max=1.0):
        keep = [i for i, e in enumerate(epochs) if e in self.dist_map]
        self.discarded += len(epochs) - len(keep)
        if not keep:
            return 0.0, None
        drift = [self.dist_map[epochs[i]] for i in keep]
        g, _ = fd_gradient(self.table, self.P, [idx[i] for i in keep], [sign[i] for i in keep],
                           [rewards[i] for i in keep], policy_reward, self.noise_std, drift)
        self.theta, update = dsgd_step(self.theta, g, self.lr, omega, omega_min, omega_max)
        self.epoch += 1
        self.dist_map = {self.epoch: None}
        for params, ep in self.history:
            self.dist_map[ep] = (params - self.theta).astype(np.float32)
        self.history.append((self.theta.copy(), self.epoch))
        while len(self.history) > self.max_delayed_return:
            self.history.pop(0)
        return update, g
