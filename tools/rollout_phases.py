"""Phase breakdown of the MLP rollout kernel: s_memtime cycles per env step of wave 0 of block 0,
split into policy L1 (+ draws, gather), L2, head, action, env.  Needs the diagnostics build:

    make -C dfd-starter_amd/csrc stamps
    python tools/rollout_phases.py [--config halfcheetah] [--lanes 4096]
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("FDR_LIB", os.path.join(ROOT, "dfd-starter_amd", "fdr", "libfdr_stamps.so"))
sys.path.insert(0, os.path.join(ROOT, "dfd-starter_amd"))

import torch  # noqa: E402

from envs import SyntheticEnv  # noqa: E402
from fdr._lib import lib  # noqa: E402
from policies import DiscretePolicy, MujocoPolicy  # noqa: E402
from utils import SharedNoiseTable  # noqa: E402
from worker import Agent, Worker  # noqa: E402

SHAPES = {"halfcheetah": (MujocoPolicy, 17, 6, 1000), "cartpole": (DiscretePolicy, 4, 2, 500)}
NAMES = ["draws + gather + L1", "gather + L2", "head + row reduce", "action + entropy", "env step"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="halfcheetah", choices=list(SHAPES))
    ap.add_argument("--lanes", type=int, default=4096)
    ap.add_argument("--iters", type=int, default=12)
    args = ap.parse_args()
    Pol, n_in, n_act, T = SHAPES[args.config]
    dev = torch.device("cuda", 0)
    torch.manual_seed(124)
    policy = Pol(n_in, n_act, seed=124, device=dev)
    env = SyntheticEnv.named(args.config, device=dev, episode_len=T)
    table = SharedNoiseTable(2_000_000, policy.num_params, random_seed=124)
    table.device_table(dev)
    worker = Worker(policy, Agent(policy, env, random_seed=124), table, None, sigma=0.02, random_seed=124)
    read = getattr(lib, "fdr_debug_phase_read", None)  # only in the stamps build
    if read is not None:
        read.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    times = []
    for it in range(args.iters):
        e0.record()
        worker.evaluate(args.lanes // 2, antithetic=True)
        e1.record()
        torch.cuda.synchronize()
        times.append(e0.elapsed_time(e1))
    ms = sorted(times[1:])[len(times[1:]) // 2]
    print("evaluate: %.3f ms (median of %d) for %d lanes x %d steps" % (ms, len(times) - 1, args.lanes, T))
    if read is None:
        return
    buf = (ctypes.c_ulonglong * 5)()
    assert read(buf) == 0
    tot = sum(buf)
    for k in range(5):
        print("%-22s %8.1f cycles/step  %5.1f %%" % (NAMES[k], buf[k] / T, 100.0 * buf[k] / max(tot, 1)))
    print("%-22s %8.1f cycles/step (wave 0 of block 0)" % ("total", tot / T))


if __name__ == "__main__":
    main()
