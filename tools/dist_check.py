"""Multi-rank rehearsal of the sharded FD step on ONE GPU (all ranks share cuda:0, gloo backend).

    python tools/dist_check.py single                  # 1 process  -> gpurun_out/dist/theta_single.npy
    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
        tools/dist_check.py multi                      # 2 ranks   -> gpurun_out/dist/theta_rank{r}.npy
    python tools/dist_check.py compare

Every rank draws the full index stream, evaluates its lane slice, all-gathers rewards, all-reduces
the gradient and applies the replicated DSGD step: all ranks must end bit-identical, and equal to
the single-process run up to the all-reduce summation order.
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "dfd-starter_amd")]
OUT = os.path.join(REPO, "gpurun_out", "dist")


def run(mode):
    import numpy as np
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if mode == "multi":
        dist.init_process_group("gloo")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    from dsgd import DSGD
    from envs import SyntheticEnv
    from learner import FiniteDifferences
    from policies import MujocoPolicy
    from utils import AdaptiveOmega, SharedNoiseTable
    from worker import Agent, Worker
    torch.manual_seed(124)
    policy = MujocoPolicy(17, 6, seed=124, device=dev)
    env = SyntheticEnv(17, 6, False, 200, device=dev)
    table = SharedNoiseTable(1 << 22, policy.num_params, random_seed=124)
    agent = Agent(policy, env, random_seed=7)
    worker = Worker(policy, agent, table, None, sigma=0.02, random_seed=124)
    learner = FiniteDifferences(policy, DSGD(policy.parameters(), lr=0.01), AdaptiveOmega(), table, noise_std=0.02)
    n_dirs = 96
    for step in range(3):
        # the same counter-stream key for a lane whatever rank evaluates it: seed by step only,
        # and lanes are keyed by their GLOBAL index through lane_base
        batch = worker.evaluate(n_dirs, antithetic=True, lane_range="auto", seed=1000 + step)
        learner.step(batch, 0.0, 0.0, 0.0)
    os.makedirs(OUT, exist_ok=True)
    name = "theta_single.npy" if mode == "single" else "theta_rank%d.npy" % rank
    np.save(os.path.join(OUT, name), policy.get_trainable_flat())
    if mode == "multi":
        dist.destroy_process_group()


def compare():
    import numpy as np
    single = np.load(os.path.join(OUT, "theta_single.npy"))
    r0 = np.load(os.path.join(OUT, "theta_rank0.npy"))
    r1 = np.load(os.path.join(OUT, "theta_rank1.npy"))
    assert np.array_equal(r0, r1), "ranks diverged"
    err = np.abs(r0 - single).max()
    print("max |theta_2rank - theta_1rank| = %.3e" % err)
    assert err < 1e-5, err
    print("dist_check ok")


if __name__ == "__main__":
    mode = sys.argv[1]
    compare() if mode == "compare" else run(mode)
