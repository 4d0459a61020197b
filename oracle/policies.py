"""Policy restatement: architectures, flat-parameter layout, normc init, forwards.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Two forms of the same arithmetic:
  * ``TorchPolicy`` -- torch-CPU nn.Sequential with the reference's exact layer order, used
    one observation at a time like the reference (policies/policy.py:26-29); this is the
    CPU-baseline form (``bench.py`` cpu_baseline leg).
  * ``lanes_forward`` -- numpy f32, batched over lanes that each own a parameter vector;
    the fast form used to check the HIP kernels at hundreds of lanes.

Reference citations:
  DiscretePolicy  policies/discrete.py:34-48 (BN -> Linear -> ReLU -> BN -> Linear -> ReLU -> BN
                  -> Linear -> Softmax, eval-mode BN), get_action :16-24, get_entropy :26-29
  MujocoPolicy    policies/mujoco.py:32-41 + utils/torch_helpers.py:15-25 (tanh; mean = first A,
                  std = 0.55 + 0.45 * t), get_action :15-22, get_entropy :24-26
  flat layout     policies/policy.py:36-42 (parameters_to_vector order)
  normc init      policies/policy.py:88-115
"""
import numpy as np
import torch
import torch.nn as nn

HIDDEN = 64
BN_EPS = 1e-5


class _MapContinuousToAction(nn.Module):
    # utils/torch_helpers.py:15-25
    def forward(self, x):
        x = torch.tanh(x)
        n = x.shape[-1] // 2
        return x[..., :n], 0.55 + 0.45 * x[..., n:]


def build_model(kind, n_in, n_act):
    if kind == "discrete":
        return nn.Sequential(
            nn.BatchNorm1d(n_in), nn.Linear(n_in, HIDDEN), nn.ReLU(),
            nn.BatchNorm1d(HIDDEN), nn.Linear(HIDDEN, HIDDEN), nn.ReLU(),
            nn.BatchNorm1d(HIDDEN), nn.Linear(HIDDEN, n_act), nn.Softmax(dim=-1))
    if kind == "mujoco":
        return nn.Sequential(
            nn.Linear(n_in, HIDDEN), nn.Tanh(),
            nn.Linear(HIDDEN, HIDDEN), nn.Tanh(),
            nn.Linear(HIDDEN, 2 * n_act), _MapContinuousToAction())
    raise ValueError(kind)


def layout(kind, n_in, n_act):
    """[(name, shape)] in parameters() order -- the flat vector order."""
    H = HIDDEN
    if kind == "discrete":
        return [("bn0.w", (n_in,)), ("bn0.b", (n_in,)), ("l1.w", (H, n_in)), ("l1.b", (H,)),
                ("bn1.w", (H,)), ("bn1.b", (H,)), ("l2.w", (H, H)), ("l2.b", (H,)),
                ("bn2.w", (H,)), ("bn2.b", (H,)), ("l3.w", (n_act, H)), ("l3.b", (n_act,))]
    return [("l1.w", (H, n_in)), ("l1.b", (H,)), ("l2.w", (H, H)), ("l2.b", (H,)),
            ("l3.w", (2 * n_act, H)), ("l3.b", (2 * n_act,))]


def num_params(kind, n_in, n_act):
    return int(sum(np.prod(s) for _, s in layout(kind, n_in, n_act)))


def unflatten(kind, n_in, n_act, flat):
    """flat [..., P] -> dict name -> array [..., *shape] (views)."""
    out, off = {}, 0
    flat = np.asarray(flat)
    for name, shape in layout(kind, n_in, n_act):
        n = int(np.prod(shape))
        out[name] = flat[..., off:off + n].reshape(flat.shape[:-1] + shape)
        off += n
    return out


def normc_init(model, rng):
    """policies/policy.py:88-115 -- applied to every layer with a .weight (BN included)."""
    layers = [m for m in model if hasattr(m, "weight")]
    std = 1.0
    for i, layer in enumerate(layers):
        if i == len(layers) - 1:
            std = 0.01
        w = layer.weight.data
        out = rng.randn(*w.shape).astype(np.float32)
        out *= std / np.sqrt(np.square(out).sum(axis=0, keepdims=True))
        new_w = (torch.as_tensor(out, dtype=torch.float32) - w).reshape_as(w)
        new_b = -layer.bias.data.reshape_as(layer.bias.data)
        layer.weight.data += new_w
        layer.bias.data += new_b


class TorchPolicy(object):
    """Reference-shaped CPU policy (one nn.Sequential, eval mode)."""

    def __init__(self, kind, n_in, n_act, seed=124):
        self.kind, self.n_in, self.n_act = kind, n_in, n_act
        self.model = build_model(kind, n_in, n_act)
        self.model.eval()
        self.rng = np.random.RandomState(seed)     # policies/policy.py:15
        normc_init(self.model, self.rng)
        self.num_params = num_params(kind, n_in, n_act)

    def forward(self, x):
        # policies/policy.py:26-29
        x = torch.as_tensor(np.asarray(x), dtype=torch.float32).view(-1, self.n_in)
        return self.model(x)

    @torch.no_grad()
    def get_flat(self):
        return nn.utils.parameters_to_vector(self.model.parameters()).numpy().copy()

    @torch.no_grad()
    def set_flat(self, flat):
        nn.utils.vector_to_parameters(torch.as_tensor(np.asarray(flat), dtype=torch.float32),
                                      self.model.parameters())

    def bn_stats(self):
        """[(running_mean, running_var)] for the three BN layers (discrete only)."""
        return [(m.running_mean.numpy().copy(), m.running_var.numpy().copy())
                for m in self.model if isinstance(m, nn.BatchNorm1d)]

    @torch.no_grad()
    def act(self, x, deterministic, noise):
        """get_action with an injected noise value (uniform for discrete, normals for mujoco).

        discrete: deterministic -> argmax (discrete.py:18-19); else inverse CDF of the
                  normalised probs at uniform u (DESIGN.md "Random streams").
        mujoco:   deterministic -> mean (mujoco.py:17-18); else mean + std * z.
        Returns (action, per-step entropy term) -- entropy is returned for the online
        accumulation check; the reference's end-of-episode form is ``entropy``.
        """
        if self.kind == "discrete":
            p = self.forward(x)[0].numpy()
            if deterministic:
                return int(np.argmax(p))
            return categorical_inverse_cdf(p, noise)
        mean, std = self.forward(x)
        mean, std = mean[0].numpy(), std[0].numpy()
        if deterministic:
            return mean.astype(np.float32)
        return (mean + std * np.asarray(noise, dtype=np.float32)).astype(np.float32)

    @torch.no_grad()
    def entropy(self, states):
        # discrete.py:26-29 / mujoco.py:24-26
        if self.kind == "discrete":
            probs = self.forward(states)
            return torch.distributions.Categorical(probs=probs).entropy().mean().item()
        mean, std = self.forward(states)
        return torch.distributions.Normal(mean, std).entropy().sum(dim=-1).mean().item()


def categorical_inverse_cdf(p, u):
    """Smallest i with cumsum(p)[i] > u * sum(p) (f32, sequential cumsum); last index if none."""
    p = np.asarray(p, dtype=np.float32)
    total = np.float32(0)
    for v in p:
        total = np.float32(total + v)
    target = np.float32(np.float32(u) * total)
    c = np.float32(0)
    for i, v in enumerate(p):
        c = np.float32(c + v)
        if c > target:
            return i
    return len(p) - 1


# ----------------------------------------------------------------------------------------------
# numpy batched-over-lanes forward (f32), each lane with its own parameter vector
# ----------------------------------------------------------------------------------------------

def _bn(x, w, b, rm, rv):
    # torch eval BN: alpha = w / sqrt(rv + eps); out = x * alpha + (b - rm * alpha)
    alpha = (w / np.sqrt(rv + np.float32(BN_EPS), dtype=np.float32)).astype(np.float32)
    return (x * alpha + (b - rm * alpha)).astype(np.float32)


def lanes_forward(kind, n_in, n_act, thetas, x, bn_stats=None):
    """thetas [L, P] f32, x [L, n_in] f32 -> probs [L, A] (discrete) | (mean, std) [L, A]."""
    p = unflatten(kind, n_in, n_act, np.asarray(thetas, dtype=np.float32))
    x = np.asarray(x, dtype=np.float32)

    def lin(h, name):
        return (np.einsum("lok,lk->lo", p[name + ".w"], h).astype(np.float32) + p[name + ".b"]).astype(np.float32)

    if kind == "discrete":
        if bn_stats is None:
            bn_stats = [(np.zeros(n_in, np.float32), np.ones(n_in, np.float32))] + \
                       [(np.zeros(HIDDEN, np.float32), np.ones(HIDDEN, np.float32))] * 2
        h = _bn(x, p["bn0.w"], p["bn0.b"], *bn_stats[0])
        h = np.maximum(lin(h, "l1"), 0)
        h = _bn(h, p["bn1.w"], p["bn1.b"], *bn_stats[1])
        h = np.maximum(lin(h, "l2"), 0)
        h = _bn(h, p["bn2.w"], p["bn2.b"], *bn_stats[2])
        z = lin(h, "l3")
        z = z - z.max(axis=-1, keepdims=True)
        e = np.exp(z).astype(np.float32)
        return (e / e.sum(axis=-1, keepdims=True)).astype(np.float32)
    h = np.tanh(lin(x, "l1")).astype(np.float32)
    h = np.tanh(lin(h, "l2")).astype(np.float32)
    t = np.tanh(lin(h, "l3")).astype(np.float32)
    return t[:, :n_act], (np.float32(0.55) + np.float32(0.45) * t[:, n_act:]).astype(np.float32)


def categorical_entropy(probs):
    """torch Categorical(probs).entropy(): p normalised, logits = log p clamped, -sum p*logits."""
    p = np.asarray(probs, dtype=np.float64)
    p = p / p.sum(axis=-1, keepdims=True)
    with np.errstate(divide="ignore"):
        lg = np.log(p)
    lg = np.maximum(lg, np.finfo(np.float32).min)
    return -(p * lg).sum(axis=-1)


def normal_entropy(std):
    """torch Normal entropy summed over action dims: sum(0.5 + 0.5 ln(2 pi) + ln std)."""
    std = np.asarray(std, dtype=np.float64)
    return (0.5 + 0.5 * np.log(2 * np.pi) + np.log(std)).sum(axis=-1)
