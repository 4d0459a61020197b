"""Multi-rank rehearsal of the sharded FD step on ONE GPU (all ranks share cuda:0, gloo backend).

    python tools/dist_check.py single <weighting> <out_dir>        # 1 process -> <out_dir>/theta_single.npy
    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
        tools/dist_check.py multi <weighting> <out_dir>            # 2 ranks  -> <out_dir>/theta_rank{r}.npy
    python tools/dist_check.py compare <weighting> <out_dir>
    FDR_FORCE_COLLECTIVES=1 python -m torch.distributed.run --nproc-per-node 1 ... tools/dist_check.py nccl1 <w> <out>
                                                                   # RCCL, one rank, the sharded exchange forced on
    ... <mode> <weighting> <out_dir> bench                         # BASELINE config 3 size (below)

weighting: "zscore" (the default one-collective moments form) or "centred_rank" (all-gather + all-reduce).
The product path end to end: every rank draws the full index stream (SharedNoiseTable), Worker.evaluate runs its
lane slice (lane_range="auto", lanes keyed by their GLOBAL index), FiniteDifferences.step exchanges and applies
the replicated DSGD step -- for STEPS FD steps.  All ranks must end bit-identical, and equal to the
single-process run up to the collective's summation order.  tests/test_gpu_dist_equivalence.py drives it.
Preset "stale": from step 1 on, lists of FDReturn with the previous step's returns again as one-epoch-old
(delayed) returns -- the sharded drift path of FiniteDifferences.
Preset "uneven" (ADVICE r4): lists of FDReturn split unevenly over the ranks -- step 0: rank 1 holds none, step 1:
30 % / 70 %, step 2: rank 0 holds none -- the count exchange, the padded unequal all-gather and the zero-gradient
branch of a rank without returns, against the single process holding every return.
Preset "bench": bench.py's step at BASELINE config 3 size -- 2048 directions (4096 lanes) PER RANK, T = 1000, the
25 M-entry table, 2 FD steps through Worker.evaluate(prefetch=True) + FiniteDifferences.step_async.
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "dfd-starter_amd")]
STEPS = 3


PRESETS = {"small": dict(dirs_per_rank=48, T=200, table=1 << 22, steps=STEPS, bench=False),
           "bench": dict(dirs_per_rank=2048, T=1000, table=25_000_000, steps=2, bench=True),
           "stale": dict(dirs_per_rank=24, T=100, table=1 << 22, steps=STEPS, bench=False, stale=True),
           "uneven": dict(dirs_per_rank=24, T=100, table=1 << 22, steps=STEPS, bench=False, uneven=True)}


def run(mode, weighting, out, preset="small"):
    import numpy as np
    import torch
    import torch.distributed as dist
    rank = int(os.environ.get("RANK", "0"))
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    if mode == "multi":
        dist.init_process_group("gloo")
    elif mode == "nccl1":   # RCCL with ONE rank; FDR_FORCE_COLLECTIVES=1 keeps the sharded exchange on
        dist.init_process_group("nccl", device_id=dev)
    from dsgd import DSGD
    from envs import SyntheticEnv
    from learner import FiniteDifferences
    from policies import MujocoPolicy
    from utils import AdaptiveOmega, SharedNoiseTable
    from worker import Agent, Worker
    torch.manual_seed(124)
    policy = MujocoPolicy(17, 6, seed=124, device=dev)
    cfg = PRESETS[preset]
    env = SyntheticEnv(17, 6, False, cfg["T"], device=dev)
    table = SharedNoiseTable(cfg["table"], policy.num_params, random_seed=124)
    agent = Agent(policy, env, random_seed=7)
    worker = Worker(policy, agent, table, None, sigma=0.02, random_seed=124)
    learner = FiniteDifferences(policy, DSGD(policy.parameters(), lr=0.01), AdaptiveOmega(), table, noise_std=0.02,
                                weighting=weighting)
    # the global direction count is the 2-rank job's, whichever mode runs it
    n_dirs = 2 * cfg["dirs_per_rank"]
    upd = []
    for step in range(cfg["steps"]):
        # the same counter-stream key for a lane whatever rank evaluates it: seed by step only,
        # and lanes are keyed by their GLOBAL index through lane_offset
        if cfg.get("stale"):
            # delayed returns (the reference's async server, learner/finite_differences.py:66-92): from step 1 on,
            # the learner gets a list of FDReturn -- this step's returns (current epoch) + the previous step's
            # returns again (one epoch old: lambda carries the drift theta_prev - theta_now); each rank holds its
            # own lanes of both
            batch = worker.evaluate(n_dirs, antithetic=True, lane_range="auto", seed=1000 + step)
            if step == 0:
                upd.append(learner.step(batch, 0.25, 0.0, 0.0))
            else:
                cur = batch.to_returns()
                for r in cur:
                    r.epoch = learner.epoch
                for r in prev:
                    r.epoch = learner.epoch - 1
                upd.append(learner.step(cur + prev, 0.25, 0.0, 0.0))
            prev = batch.to_returns()
            continue
        if cfg.get("uneven"):
            # every process evaluates all lanes (global lane keys: identical returns everywhere), then each rank keeps
            # its share of the list; the single process keeps all of it
            rets = worker.evaluate(n_dirs, antithetic=True, seed=1000 + step).to_returns()
            for r in rets:
                r.epoch = learner.epoch
            if mode != "single":
                cut = [len(rets), (3 * len(rets)) // 10, 0][step % 3]
                rets = rets[:cut] if rank == 0 else rets[cut:]
            upd.append(learner.step(rets, 0.25, 0.0, 0.0))
            continue
        if cfg["bench"]:    # bench.py's fd_step: prefetched indices, the learner's no-sync step
            batch = worker.evaluate(n_dirs, antithetic=True, lane_range="auto", seed=1000 + step, prefetch=True)
            upd.append(learner.step_async(batch, 0.0, 0.0, 0.0).tolist()[0])
        else:
            batch = worker.evaluate(n_dirs, antithetic=True, lane_range="auto", seed=1000 + step)
            upd.append(learner.step(batch, 0.25, 0.0, 0.0))
    os.makedirs(out, exist_ok=True)
    name = "single" if mode == "single" else "rank%d" % rank
    np.save(os.path.join(out, "theta_%s.npy" % name), policy.get_trainable_flat())
    np.save(os.path.join(out, "upd_%s.npy" % name), np.asarray(upd))
    if mode in ("multi", "nccl1"):
        dist.destroy_process_group()


def compare(out, world=2):
    """-> max |theta_Nrank - theta_1rank|; raises if the ranks differ."""
    import numpy as np
    single = np.load(os.path.join(out, "theta_single.npy"))
    ranks = [np.load(os.path.join(out, "theta_rank%d.npy" % r)) for r in range(world)]
    for r in ranks[1:]:
        assert np.array_equal(r, ranks[0]), "ranks diverged"
    err = float(np.abs(ranks[0] - single).max())
    print("max |theta_%drank - theta_1rank| = %.3e" % (world, err))
    return err


if __name__ == "__main__":
    mode, weighting, out = sys.argv[1], sys.argv[2], sys.argv[3]
    if mode == "compare":
        assert compare(out) <= 1e-6
        print("dist_check ok")
    else:
        run(mode, weighting, out, sys.argv[4] if len(sys.argv) > 4 else "small")
