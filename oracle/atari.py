"""AtariPolicy restatement (policies/atari.py:7-51) + its batched rollout semantics on the build's
synthetic stacked-frame env.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py); pinned by tests/golden/g11_atari.npz (the
reference AtariPolicy: normc init fingerprint and eval-mode forwards) and g16_atari_vbn.npz (compute_vbn).

Network, eval mode (atari.py:36-51), input [4, 84, 84] (no /255 scaling in the reference):
  conv 4->16 k8 s4 -> BN2d -> ReLU -> conv 16->32 k4 s2 -> BN2d -> ReLU -> flatten (C,H,W) 2592
  -> Linear 256 -> BN1d -> ReLU -> Linear A -> Softmax
normc (policy.py:88-115) touches every layer with a weight (convs and BNs included) and zeroes the
biases; the `w + (out - w)` update rounds, so the torch default init (torch.manual_seed) matters.
"""
import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from . import impala as oi
from . import rng as crng
from .noise import perturb
from .policies import categorical_inverse_cdf, normc_init

FRAME_C, FRAME_H, FRAME_W = 4, 84, 84
FRAME_PIX = FRAME_C * FRAME_H * FRAME_W
FEAT = 2592
BN_EPS = 1e-5


def build_model(n_act):
    return nn.Sequential(
        nn.Conv2d(4, 16, kernel_size=[8, 8], stride=[4, 4]), nn.BatchNorm2d(16), nn.ReLU(),
        nn.Conv2d(16, 32, kernel_size=[4, 4], stride=[2, 2]), nn.BatchNorm2d(32), nn.ReLU(),
        nn.Flatten(), nn.Linear(FEAT, 256), nn.BatchNorm1d(256), nn.ReLU(),
        nn.Linear(256, n_act), nn.Softmax(dim=-1))


def init_theta(n_act, seed=124):
    """AtariPolicy(., n_act, seed) parameters after torch.manual_seed(seed) + normc(RandomState(seed))."""
    torch.manual_seed(seed)
    m = build_model(n_act)
    m.eval()
    normc_init(m, np.random.RandomState(seed))
    return nn.utils.parameters_to_vector(m.parameters()).detach().numpy().copy()


def layout(n_act):
    return [("c1.w", (16, 4, 8, 8)), ("c1.b", (16,)), ("bn1.w", (16,)), ("bn1.b", (16,)),
            ("c2.w", (32, 16, 4, 4)), ("c2.b", (32,)), ("bn2.w", (32,)), ("bn2.b", (32,)),
            ("fc.w", (256, FEAT)), ("fc.b", (256,)), ("bn3.w", (256,)), ("bn3.b", (256,)),
            ("head.w", (n_act, 256)), ("head.b", (n_act,))]


def num_params(n_act):
    return int(sum(np.prod(s) for _, s in layout(n_act)))


def unflatten(flat, n_act):
    flat = torch.as_tensor(np.asarray(flat, np.float32))
    out, off = {}, 0
    for name, shape in layout(n_act):
        n = int(np.prod(shape))
        out[name] = flat[off:off + n].view(shape)
        off += n
    return out


def split_bn(rm, rv):
    rm = torch.as_tensor(np.asarray(rm, np.float32))
    rv = torch.as_tensor(np.asarray(rv, np.float32))
    return {"bn1": (rm[:16], rv[:16]), "bn2": (rm[16:48], rv[16:48]), "bn3": (rm[48:304], rv[48:304])}


def _bn(x, p, bn, name):
    return F.batch_norm(x, bn[name][0], bn[name][1], p[name + ".w"], p[name + ".b"], training=False, eps=BN_EPS)


@torch.no_grad()
def features(p, bn, frames):
    x = torch.as_tensor(np.asarray(frames, np.float32)).reshape(-1, FRAME_C, FRAME_H, FRAME_W)
    x = F.relu(_bn(F.conv2d(x, p["c1.w"], p["c1.b"], stride=4), p, bn, "bn1"))
    x = F.relu(_bn(F.conv2d(x, p["c2.w"], p["c2.b"], stride=2), p, bn, "bn2"))
    return x.reshape(x.shape[0], -1)


@torch.no_grad()
def forward(p, bn, frames):
    f = features(p, bn, frames)
    h = F.relu(_bn(F.linear(f, p["fc.w"], p["fc.b"]), p, bn, "bn3"))
    return torch.softmax(F.linear(h, p["head.w"], p["head.b"]), dim=-1), f


@torch.no_grad()
def compute_vbn(p, rm, rv, frames, momentum=0.1):
    """AtariPolicy.compute_vbn (policies/policy.py:31-34 on atari.py:36-51): one train-mode pass of the buffer -- every
    BN normalises with its batch statistics (biased variance) and updates its running stats (unbiased variance,
    momentum).  Returns the new (rm, rv) flat [16 | 32 | 256]; pinned by tests/golden/g16_atari_vbn.npz."""
    rm = torch.as_tensor(np.array(rm, np.float32))
    rv = torch.as_tensor(np.array(rv, np.float32))
    bn = {"bn1": (rm[:16], rv[:16]), "bn2": (rm[16:48], rv[16:48]), "bn3": (rm[48:304], rv[48:304])}

    def tbn(x, name):
        return F.batch_norm(x, bn[name][0], bn[name][1], p[name + ".w"], p[name + ".b"], training=True,
                            momentum=momentum, eps=BN_EPS)
    x = torch.as_tensor(np.asarray(frames, np.float32)).reshape(-1, FRAME_C, FRAME_H, FRAME_W)
    x = F.relu(tbn(F.conv2d(x, p["c1.w"], p["c1.b"], stride=4), "bn1"))
    x = F.relu(tbn(F.conv2d(x, p["c2.w"], p["c2.b"], stride=2), "bn2"))
    tbn(F.linear(x.reshape(x.shape[0], -1), p["fc.w"], p["fc.b"]), "bn3")
    return rm.numpy(), rv.numpy()


# synthetic stacked-frame env: the Impala frame env's hash (oracle/impala.py) over a 4 x 84 x 84 image
FRAME_WORDS = FRAME_PIX // 8


def frames(env_seed, env_ids, t):
    key = crng.mix64(np.uint64((env_seed ^ oi.FRAME_SALT) & crng.M64))
    env_ids = np.asarray(env_ids, dtype=np.uint64).reshape(-1, 1)
    h = oi._keyed(key, oi._ctr(env_ids, t, np.arange(FRAME_WORDS, dtype=np.uint64)[None, :]))
    return np.ascontiguousarray(h).view(np.uint8).reshape(-1, FRAME_C, FRAME_H, FRAME_W)


def evaluate_lanes(theta, table, idx, sign, sigma, n_act, envs_per_lane, T, seed, env_seed, rm, rv,
                   deterministic=False, jiggle=True, lane_offset=0, record=False):
    """Batched semantics of fdr_atari_rollout: lane l (theta'_l) drives envs l*E .. l*E+E-1 for T
    steps; entropy = mean of the per-step Categorical entropies (atari.py:25-28 on the visited
    states, eval-mode BN: per-state); actions/rewards as oracle/impala.py."""
    L, E = len(idx), int(envs_per_lane)
    thetas = perturb(theta, table, idx, sign, sigma)
    P = thetas.shape[1]
    s32 = np.float32(sigma)
    norm2 = np.array([float(np.dot((table[int(i):int(i) + P] * s32).astype(np.float64),
                                   (table[int(i):int(i) + P] * s32).astype(np.float64)))
                      if sg != 0 else 0.0 for i, sg in zip(idx, sign)])
    bn = split_bn(rm, rv)
    det = np.broadcast_to(np.asarray(deterministic, dtype=bool), (L,))
    ret = np.zeros((L, E), np.float64)
    ent = np.zeros((L, E), np.float64)
    acts = np.zeros((L, E, T), np.int32)
    probs_rec = np.zeros((L, E, T, n_act), np.float32) if record else None
    for l in range(L):
        p = unflatten(thetas[l], n_act)
        envs = (np.uint64(lane_offset + l) * np.uint64(E) + np.arange(E, dtype=np.uint64))
        for t in range(T):
            pr, _ = forward(p, bn, frames(env_seed, envs, t).astype(np.float32))
            pn = pr.numpy()
            if record:
                probs_rec[l, :, t] = pn
            if det[l]:
                a = pn.argmax(-1)
            else:
                u = crng.uniform(seed, envs, t, 0)
                a = np.array([categorical_inverse_cdf(pn[e], u[e]) for e in range(E)])
            acts[l, :, t] = a
            ret[l] += oi.rewards(env_seed, envs, t, a, n_act)
            ent[l] += oi.categorical_entropy(pr).double().numpy()
        ent[l] /= T
        if jiggle:
            ret[l] += crng.jiggle(seed, envs)
    out = dict(ret=ret, ent=ent, steps=np.full((L, E), T, np.int32), norm2=norm2, actions=acts)
    if record:
        out["probs"] = probs_rec
    return out
