"""Learner-kernel timings (GPU box): staged (fd_weights + fd_grad + dsgd) vs fused (fd_grad_fused [+ dsgd]) vs
one-launch fdr_fd_step, at BASELINE config 3's shape (2048 directions x +-, P = 6092), HIP events over 50 calls.
    python tools/learner_bench.py [n_dirs P]"""
import os
import sys

import numpy as np
import torch

sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "dfd-starter_amd")]
from fdr import engine  # noqa: E402

n_dirs = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
P = int(sys.argv[2]) if len(sys.argv) > 2 else 6092
dev = "cuda"
rs = np.random.RandomState(0)
table = torch.randn(25_000_000, device=dev)
idx_dirs = torch.as_tensor(rs.randint(0, 25_000_000 - P, size=n_dirs), device=dev)
idx = idx_dirs.repeat_interleave(2)
sign = torch.as_tensor(np.tile(np.array([1, -1], np.int8), n_dirs), device=dev)
rew = torch.randn(2 * n_dirs, dtype=torch.float64, device=dev)
n2 = torch.rand(2 * n_dirs, dtype=torch.float64, device=dev) + 1.0
theta = torch.randn(P, device=dev)
g = torch.empty(P, dtype=torch.float64, device=dev)


def timeit(name, fn, n=50):
    for _ in range(5):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    print("%-40s %8.2f us / call" % (name, e0.elapsed_time(e1) * 1e3 / n), flush=True)


def staged():
    c = engine.fd_weights(rew, 0.0, 0, sign, n2, 2, 0.02)
    gg = engine.fd_grad(table, idx_dirs, c, P, g)
    engine.dsgd_step(theta, gg, 0.01, 0.5)


timeit("staged weights+grad+dsgd (7 launches)", staged)
timeit("fd_weights only", lambda: engine.fd_weights(rew, 0.0, 0, sign, n2, 2, 0.02))
timeit("fd_grad_fused zscore", lambda: engine.fd_grad_fused(table, idx, rew, 0.0, 0, sign, n2, 2, 0.02, P, out=g))
timeit("fd_grad_fused moments", lambda: engine.fd_grad_fused(table, idx, rew, 0.0, 0, sign, n2, 2, 0.02, P,
                                                             mode="moments"))
timeit("dsgd_step_ex (fused single WG)", lambda: engine.dsgd_step_ex(theta, g, False, 0.01, 0.5))
if P <= 65536:
    timeit("fd_step (one launch)", lambda: engine.fd_step(table, idx, rew, 0.0, sign, n2, 2, 0.02, theta, 0.01, 0.5,
                                                          g=g))
