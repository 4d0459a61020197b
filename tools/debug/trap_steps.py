"""Debug: trap-env sampled rollout, GPU vs oracle, per episode length T (first divergence)."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "dfd-starter_amd")]
import numpy as np, torch
from fdr import engine, _lib
from envs import TrapEnv
from oracle import policies as opol, noise as onoise, envs as oenvs, rng as crng

torch.manual_seed(124)
pol = opol.TorchPolicy("discrete", 2, 9, seed=124)
theta = pol.get_flat()
t = onoise.NoiseTable(1 << 22, theta.size, 124)
L = 4
idx = t.sample_indices(L)
sign = np.ones(L, np.int8)
dev = "cuda"
tab = torch.from_numpy(t.table).to(dev)
spec = engine.PolicySpec("discrete", 2, 9, theta.size)
th_d, idx_d, sg_d = torch.from_numpy(theta).to(dev), torch.from_numpy(idx).to(dev), torch.from_numpy(sign).to(dev)
lanes = engine.lanes_desc(th_d, 0, tab, idx_d, sg_d, 0.5)
env = TrapEnv()
thetas = onoise.perturb(theta, t.table, idx, sign, 0.5)

class ShortTrap(object):
    def __init__(self, T): self.T = T
    def desc(self):
        return _lib.EnvDesc(_lib.FDR_ENV_TRAP, 2, 9, self.T, None, None, None, env.walkable.data_ptr(), env.map_w, env.map_h)

for T in [1, 2, 3, 5, 8, 20, 64, 65, 70, 130, 201]:
    res = engine.rollout(spec, ShortTrap(T), lanes, L, 99, jiggle=False)
    out = []
    for l in range(L):
        pol.set_flat(thetas[l])
        e = oenvs.TrapEnv(); obs = e.reset(); r = 0; acts = []
        for s in range(T):
            p = pol.forward(obs)[0].detach().numpy()
            a = opol.categorical_inverse_cdf(p, np.float32(crng.uniform(99, l, s, 0)))
            acts.append(a)
            obs, rew, _, _ = e.step(a); r += rew
        out.append(r)
    print(T, res.reward.cpu().numpy().tolist(), out)
