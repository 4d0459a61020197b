"""A/B timing of MLP rollout builds on the GPU box: one config's rollout launch (lanes resident on the device),
timed with HIP events after the clocks have settled; alternate builds in separate processes.

    python tools/ab_pair.py --lib dfd-starter_amd/fdr/libfdr_v1.so [--config halfcheetah] [--lanes 4096]

Prints one line: build, config, median / min ms per launch over the timed launches, and the check-sum of the
returns (builds must agree up to the kernel's own rounding -- parity is the GPU test suite's job).
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", required=True)
    ap.add_argument("--config", default="halfcheetah", choices=["halfcheetah", "cartpole"])
    ap.add_argument("--lanes", type=int, default=None)
    ap.add_argument("--settle-ms", type=float, default=300.0)
    ap.add_argument("--iters", type=int, default=60)
    ap.add_argument("--impl", default=None, help="pair | single | wide | auto")
    args = ap.parse_args()
    os.environ["FDR_LIB"] = os.path.abspath(args.lib)
    sys.path.insert(0, os.path.join(ROOT, "dfd-starter_amd"))
    import numpy as np
    import torch
    from envs import SyntheticEnv
    from fdr import engine
    from policies import DiscretePolicy, MujocoPolicy
    from utils import SharedNoiseTable
    Pol, n_in, n_act, T, lanes_default = {"halfcheetah": (MujocoPolicy, 17, 6, 1000, 4096),
                                          "cartpole": (DiscretePolicy, 4, 2, 500, 1024)}[args.config]
    L = args.lanes or lanes_default
    dev = torch.device("cuda", 0)
    torch.manual_seed(124)
    policy = Pol(n_in, n_act, seed=124, device=dev)
    env = SyntheticEnv.named(args.config, device=dev, episode_len=T)
    nt = SharedNoiseTable(25_000_000, policy.num_params, random_seed=124)
    table = nt.device_table(dev)
    idx = torch.as_tensor(np.repeat(nt.sample_batch(L // 2), 2), device=dev)
    sign = torch.as_tensor(np.tile(np.array([1, -1], np.int8), L // 2), device=dev)
    lanes = engine.lanes_desc(policy.flat, 0, table, idx, sign, 0.02)
    ctx = engine.Context(dev)
    if args.impl:
        ctx.set_rollout_impl(args.impl)
    bm, bv = policy.bn_stats()
    out = engine.rollout(policy.spec, env, lanes, L, 7, bn_mean=bm, bn_var=bv, device=dev, ctx=ctx)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    while (time.perf_counter() - t0) * 1e3 < args.settle_ms:
        engine.rollout(policy.spec, env, lanes, L, 7, bn_mean=bm, bn_var=bv, device=dev, ctx=ctx, out=out)
        torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.iters)]
    for e0, e1 in ev:
        e0.record()
        engine.rollout(policy.spec, env, lanes, L, 7, bn_mean=bm, bn_var=bv, device=dev, ctx=ctx, out=out)
        e1.record()
    torch.cuda.synchronize()
    ms = np.array([e0.elapsed_time(e1) for e0, e1 in ev])
    chk = float(out.reward.double().sum().item())
    print("%s %s lanes=%d: median %.4f ms  min %.4f ms  sum(ret) %.9e" % (os.path.basename(args.lib), args.config, L,
                                                                        np.median(ms), ms.min(), chk))


if __name__ == "__main__":
    main()
