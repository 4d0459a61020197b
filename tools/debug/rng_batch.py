"""Debug: does the rollout use u(t) at step t?  Uniform policy on the trap env -> dx_t = f(u_t)."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "dfd-starter_amd")]
import numpy as np, torch
from fdr import engine, _lib
from envs import TrapEnv, SyntheticEnv
from oracle import policies as opol, rng as crng

P = opol.num_params("discrete", 2, 9)
theta = np.zeros(P, np.float32)        # all-zero params: BN w=0 -> logits = bias = 0 -> uniform probs
dev = "cuda"
spec = engine.PolicySpec("discrete", 2, 9, P)
env = TrapEnv()
class ShortTrap(object):
    def __init__(self, T): self.T = T
    def desc(self):
        return _lib.EnvDesc(_lib.FDR_ENV_TRAP, 2, 9, self.T, None, None, None, env.walkable.data_ptr(), env.map_w, env.map_h)
L = 3
th = torch.from_numpy(theta).to(dev)
lanes = engine.lanes_desc(th, 0)
prev = np.zeros(L)
for T in range(1, 12):
    res = engine.rollout(spec, ShortTrap(T), lanes, L, 99, jiggle=False)
    r = res.reward.cpu().numpy()
    dx_gpu = (r - prev) / 7; prev = r
    dx_orc = [opol.categorical_inverse_cdf(np.full(9, 1/9, np.float32), np.float32(crng.uniform(99, l, T - 1, 0))) // 3 - 1
              for l in range(L)]
    print(T - 1, "gpu dx", dx_gpu.tolist(), "oracle dx", dx_orc,
          "u", [round(float(crng.uniform(99, l, T - 1, 0)), 3) for l in range(L)])
# synthetic (2, 9) env, sampled, vs oracle batched evaluation
from oracle import agent as oagent, envs as oenvs, noise as onoise
torch.manual_seed(124)
pol = opol.TorchPolicy("discrete", 2, 9, seed=124)
theta = pol.get_flat(); t = onoise.NoiseTable(1 << 22, P, 124)
idx = t.sample_indices(8); sign = np.ones(8, np.int8)
tab = torch.from_numpy(t.table).to(dev)
lanes = engine.lanes_desc(torch.from_numpy(theta).to(dev), 0, tab, torch.from_numpy(idx).to(dev),
                          torch.from_numpy(sign).to(dev), 0.5)
for T in (5, 70, 200):
    senv = SyntheticEnv(2, 9, True, T)
    res = engine.rollout(spec, senv, lanes, 8, 99, jiggle=False)
    ref = oagent.evaluate_lanes("discrete", 2, 9, theta, t.table, idx, sign, 0.5,
                                oenvs.BatchedSyntheticEnv(2, 9, True, T, 8), 99, jiggle=False)
    print("synth T=%d" % T, np.abs(res.reward.cpu().numpy() - ref[0]).max())
