"""Host-side cost of one FD step of the MLP configs (GPU box): perf_counter around the phases of
Worker.evaluate + FiniteDifferences.step_async (the same objects bench.py builds), the GPU running behind.
    python tools/host_phases.py [--config cartpole] [--steps 300]"""
import argparse
import collections
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "dfd-starter_amd")]

from dsgd import DSGD  # noqa: E402
from envs import SyntheticEnv  # noqa: E402
from learner import FiniteDifferences  # noqa: E402
from policies import DiscretePolicy, MujocoPolicy  # noqa: E402
from utils import AdaptiveOmega, SharedNoiseTable  # noqa: E402
from worker import Agent, Worker  # noqa: E402
import worker.worker as wmod  # noqa: E402

SHAPES = {"cartpole": (DiscretePolicy, 4, 2, 500, 1024), "halfcheetah": (MujocoPolicy, 17, 6, 1000, 4096)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cartpole", choices=list(SHAPES))
    ap.add_argument("--steps", type=int, default=300)
    args = ap.parse_args()
    Pol, n_in, n_act, T, L = SHAPES[args.config]
    dev = torch.device("cuda", 0)
    torch.manual_seed(124)
    policy = Pol(n_in, n_act, seed=124, device=dev)
    env = SyntheticEnv.named(args.config, device=dev, episode_len=T)
    table = SharedNoiseTable(25_000_000, policy.num_params, random_seed=124)
    table.device_table(dev)
    agent = Agent(policy, env, random_seed=124)
    worker = Worker(policy, agent, table, None, sigma=0.02, random_seed=124)
    learner = FiniteDifferences(policy, DSGD(policy.parameters(), lr=0.01), AdaptiveOmega(), table, noise_std=0.02)
    acc = collections.defaultdict(float)

    def timed(name, fn):
        def wrap(*a, **k):
            t = time.perf_counter()
            try:
                return fn(*a, **k)
            finally:
                acc[name] += time.perf_counter() - t
        return wrap

    # phases: wrap the methods the step calls (instance attributes shadow the class methods)
    for name in ("_lanes_of", "_lanes_to_device", "launch", "lane_novelty"):
        setattr(worker, name, timed("worker." + name, getattr(worker, name)))
    table.sample_batch = timed("noise.sample_batch", table.sample_batch)
    table.peek_batch = timed("noise.peek_batch", table.peek_batch)
    eng = wmod.engine
    for name in ("rollout", "lanes_desc", "fd_step"):
        setattr(eng, name, timed("engine." + name, getattr(eng, name)))
    n_dirs = L // 2
    for k in range(20):
        b = worker.evaluate(n_dirs, antithetic=True, seed=k, prefetch=True)
        learner.step_async(b, 0.0, 0.0, 0.0)
    torch.cuda.synchronize()
    acc.clear()
    t0 = time.perf_counter()
    t_eval = t_learn = 0.0
    for k in range(args.steps):
        t = time.perf_counter()
        b = worker.evaluate(n_dirs, antithetic=True, seed=100 + k, prefetch=True)
        t1 = time.perf_counter()
        learner.step_async(b, 0.0, 0.0, 0.0)
        t_learn += time.perf_counter() - t1
        t_eval += t1 - t
    host = time.perf_counter() - t0
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    us = 1e6 / args.steps
    print("%s: host enqueue %.1f us / step (evaluate %.1f, learner %.1f); wall %.1f us / step"
          % (args.config, host * us, t_eval * us, t_learn * us, wall * us))
    for name, v in sorted(acc.items(), key=lambda x: -x[1]):
        print("  %-28s %7.1f us / step" % (name, v * us))


if __name__ == "__main__":
    main()
