"""Debug: rollout kernels vs the oracle over lane counts / antithetic layouts (GPU box)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dfd-starter_amd"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402

import test_gpu_kernels as tg  # noqa: E402
from fdr import engine  # noqa: E402
from fdr._lib import lib  # noqa: E402

for name in ("cheetah", "cartpole"):
    for L, anti in ((13, False), (14, False), (14, True), (64, False), (64, True)):
        for det in (False, True):
            row = []
            for impl in (1, 0):
                lib.fdr_rollout_set_impl(impl)
                res, ref = tg._rollout_case(engine, name, L, 120, det, antithetic=anti)
                d = np.abs(res.reward.cpu().numpy() - ref[0])
                row.append("%s max %.2e bad %d" % ("single" if impl else "pair", d.max(), int((d > 1e-3).sum())))
            print(name, "L=%d anti=%d det=%d:" % (L, anti, det), " | ".join(row), flush=True)
lib.fdr_rollout_set_impl(2)
