"""Where do the ~6 us idle gaps before the rollout and before the learner come from?  Config 3's FD step three
ways under rocprofv3 --kernel-trace (GPU box), separated by marker kernels: (A) Worker.evaluate(prefetch=True) +
FiniteDifferences.step_async (the bench loop), (B) the same without prefetch, (C) engine.rollout + engine.fd_step on
static device lanes.  Then: python tools/worker_gaps.py --analyse <run_kernel_trace.csv>"""
import csv
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run():
    import torch
    sys.path[:0] = [os.path.join(ROOT, "dfd-starter_amd")]
    from dsgd import DSGD
    from envs import SyntheticEnv
    from fdr import engine
    from learner import FiniteDifferences
    from policies import MujocoPolicy
    from utils import AdaptiveOmega, SharedNoiseTable
    from worker import Agent, Worker
    dev = torch.device("cuda", 0)
    torch.manual_seed(124)
    pol = MujocoPolicy(17, 6, seed=124, device=dev)
    env = SyntheticEnv.named("halfcheetah", device=dev)
    tab = SharedNoiseTable(25_000_000, pol.num_params, random_seed=124)
    table = tab.device_table(dev)
    worker = Worker(pol, Agent(pol, env, random_seed=124), tab, None, sigma=0.02, random_seed=124)
    learner = FiniteDifferences(pol, DSGD(pol.parameters(), lr=0.01), AdaptiveOmega(), tab, noise_std=0.02)
    x = torch.zeros(16, device=dev)
    L = 4096
    modes = ("A", "B", "C", "A")
    for mode in modes:
        for _ in range(3):
            torch.cumsum(x, 0, out=x)  # marker (a scan kernel)
        for k in range(12):
            if mode == "C":
                if k == 0:
                    idx = torch.as_tensor(tab.sample_batch(L // 2), device=dev).repeat_interleave(2).contiguous()
                    sign = torch.tensor([1, -1], dtype=torch.int8, device=dev).repeat(L // 2).contiguous()
                    lanes = engine.lanes_desc(pol.flat, 0, table, idx, sign, 0.02, torch.zeros(L, dtype=torch.int8,
                                                                                               device=dev))
                    g = torch.empty(pol.num_params, dtype=torch.float64, device=dev)
                res = engine.rollout(pol.spec, env, lanes, L, 7 + k, device=dev)
                engine.fd_step(table, idx, res.reward, 0.0, sign, res.norm2, 2, 0.02, pol.flat, 1e-6, 1.0, g=g)
            else:
                b = worker.evaluate(L // 2, antithetic=True, seed=k, prefetch=(mode == "A"))
                learner.step_async(b, 0.0, 0.0, 0.0)
        torch.cuda.synchronize()


def analyse(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    seg, segs, prev = [], [], None
    for r in rows:
        name = r["Kernel_Name"]
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if "scan" in name.lower() or "cumsum" in name.lower():  # marker
            if seg:
                segs.append(seg)
            seg, prev = [], e
            continue
        if prev is not None:
            seg.append((name[:40], (s - prev) / 1e3))
        prev = e
    if seg:
        segs.append(seg)
    for i, sg in enumerate(s for s in segs if s):
        by = {}
        for n, gp in sg[6:]:  # skip the first steps of a mode
            by.setdefault(n, []).append(gp)
        print("mode %s: " % ("ABCA"[i] if i < 4 else "?") + "; ".join("%s gap %.2f us" % (n, np.median(v)) for n, v in by.items()))


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--analyse":
        analyse(sys.argv[2])
    else:
        run()
