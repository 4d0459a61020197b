"""Launch gaps around the rollout kernel (GPU box, under rocprofv3 --kernel-trace): 4 back-to-back rollouts, then
rollout / tiny kernel alternation.  python tools/gap_probe.py"""
import os
import sys

import numpy as np
import torch

sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "dfd-starter_amd")]
from envs import SyntheticEnv  # noqa: E402
from fdr import engine  # noqa: E402
from policies import MujocoPolicy  # noqa: E402

dev = torch.device("cuda", 0)
pol = MujocoPolicy(17, 6, seed=124, device=dev)
env = SyntheticEnv.named("halfcheetah", device=dev)
table = torch.randn(25_000_000, device=dev)
L = 4096
idx = torch.as_tensor(np.repeat(np.random.RandomState(0).randint(0, 24_000_000, size=L // 2), 2), device=dev)
sign = torch.as_tensor(np.tile(np.array([1, -1], np.int8), L // 2), device=dev)
lanes = engine.lanes_desc(pol.flat, 0, table, idx, sign, 0.02)
x = torch.zeros(16, device=dev)
for _ in range(3):
    engine.rollout(pol.spec, env, lanes, L, 1, device=dev)
torch.cuda.synchronize()
for _ in range(4):
    engine.rollout(pol.spec, env, lanes, L, 1, device=dev)
for _ in range(4):
    engine.rollout(pol.spec, env, lanes, L, 1, device=dev)
    x.add_(1.0)
torch.cuda.synchronize()
print("gap probe done")
