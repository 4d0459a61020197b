"""Rollout launch time vs episode length at config 3's shape (4096 lanes, MujocoPolicy(17, 6), table gather) or, with
argument 'cartpole', config 2's (1024 lanes, DiscretePolicy(4, 2)): t(T) = prologue + T x step.  HIP events around
back-to-back launches; prints ms per launch for each T."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, "dfd-starter_amd")
from envs import SyntheticEnv  # noqa: E402
from fdr import engine  # noqa: E402
from policies import DiscretePolicy, MujocoPolicy  # noqa: E402

dev = torch.device("cuda", 0)
cart = len(sys.argv) > 1 and sys.argv[1] == "cartpole"
pol = DiscretePolicy(4, 2, seed=124, device=dev) if cart else MujocoPolicy(17, 6, seed=124, device=dev)
P = pol.num_params
table = torch.as_tensor(np.random.RandomState(124).randn(25_000_000).astype(np.float32), device=dev)
n = 1024 if cart else 4096
rs = np.random.RandomState(5)
idx = torch.as_tensor(np.repeat(rs.randint(0, 25_000_000 - P, size=n // 2), 2).astype(np.int64), device=dev)
sign = torch.as_tensor(np.tile([1, -1], n // 2).astype(np.int8), device=dev)
lanes = engine.lanes_desc(pol.flat, 0, table, idx, sign, 0.02)
for T in (1, 2, 5, 50, 200, 1000):
    env = SyntheticEnv(4, 2, True, T, device=dev) if cart else SyntheticEnv(17, 6, False, T, device=dev)
    for _ in range(3):
        engine.rollout(pol.spec, env, lanes, n, 11)
    torch.cuda.synchronize()
    reps = 20 if T < 100 else 5
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        engine.rollout(pol.spec, env, lanes, n, 11)
    e1.record()
    torch.cuda.synchronize()
    print("T=%5d  %.4f ms per launch" % (T, e0.elapsed_time(e1) / reps), flush=True)
