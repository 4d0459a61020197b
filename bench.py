"""bench.py -- FD perturbation-evaluation hot path on MI355X (BASELINE.json metric).

One "step" = one full FD step of BASELINE config 3 per GPU:
  host index draw (SharedNoiseTable stream) -> one fdr_rollout launch over 4096 lanes
  (2048 directions x {+eps, -eps}, HalfCheetah-shaped MujocoPolicy(17, 6), T = 1000 steps)
  -> [all-gather rewards] -> fdr_fd_weights -> fdr_fd_grad -> [RCCL all-reduce of g] -> fdr_dsgd_step.
Per-GPU work is fixed as N grows ("weak" scaling): the global batch is 4096 * N perturbations.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

`--gpus N > 1` without an external launcher (no WORLD_SIZE in the environment) starts the N ranks itself: the
parent never touches the GPU, runs `torch.distributed.run --nproc-per-node N` as a child, relays its output and
checks that rank 0's line reports N GPUs.  Under an external launcher `--gpus` must equal WORLD_SIZE, and N must
not exceed the visible devices: either mismatch exits non-zero before any GPU work.

Prints ONE JSON line on rank 0.  The cpu_baseline leg (rank 0, N = 1) times the oracle's
reference-shaped per-lane CPU loop (torch CPU forward per step, as worker/agent.py does) on a
bounded sample, BEFORE the GPU is initialised.
"""
import argparse
import json
import multiprocessing
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "dfd-starter_amd")
for _p in (REPO, PKG):
    if _p not in sys.path:
        sys.path.insert(0, _p)

METRIC = "env steps/sec (whole node) + sec/FD-grad-step, 4096 antithetic perturbations"
FP32_PEAK_TFLOPS = 157.3          # MI355X_MICROARCH.md: FP32 vector = FP32 matrix peak
FP16_PEAK_TFLOPS = 2516.6         # MI355X_MICROARCH.md: dense FP16/BF16 MFMA peak (no sparsity)
HBM_PEAK_GBS = 8000.0

CONFIGS = {
    # name: (policy kind, n_in, n_act, env shape name, episode_len)
    "halfcheetah": ("mujoco", 17, 6, "halfcheetah", 1000),
    "cartpole": ("discrete", 4, 2, "cartpole", 500),
    # BASELINE config 4 per GPU: 8192 perturbations x 4 envs over 8 GPUs -> 1024 lanes x 4 envs each
    "impala": ("impala", (64, 64, 3), 6, "frames", 1000),
    # BASELINE config 5 per GPU: as config 4 with A = 4 and fp16 rollouts
    "impala_fp16": ("impala", (64, 64, 3), 4, "frames", 1000),
}
DEFAULT_LANES = {"halfcheetah": 4096, "cartpole": 1024}   # BASELINE configs 3 and 2
IMPALA_ENVS = 4
ZETA_SIZE = 200           # run_sequential.py:30 default zeta_size
IMPALA_LANES = 1024
# ImpalaCNN conv stack, algorithmic FLOPs per env step: sum over the 15 convs of 2*Cin*9*Cout*Ho*Wo
IMPALA_CONV_FLOP = 2 * 9 * (3 * 16 * 64 * 64 + 4 * 16 * 16 * 32 * 32 + 16 * 32 * 32 * 32 + 4 * 32 * 32 * 16 * 16
                            + 32 * 32 * 16 * 16 + 4 * 32 * 32 * 8 * 8)
# fc + LSTM + head weights streamed per (lane, step) by the core kernel (f32)
IMPALA_CORE_BYTES = 4 * (2048 * 256 + 257 * 1024 + 256 * 1024)
# oracle CPU loop rate / the reference's own loop rate, same machine, one thread (tools/cpu_calibrate.py,
# profiles/r06_cpu_calibration.txt): the cpu_baseline's reference-equivalent rate = measured / ratio
CPU_CALIBRATION = {"halfcheetah": 1.06, "cartpole": 0.91, "trap": 1.60}


def rollout_kernel_name(kind, n_in, n_act, lanes, dev):
    """Which synthetic-env rollout kernel fdr_rollout picks (FDR_ROLLOUT / auto rule, include/fdr.h)."""
    import torch
    mode = os.environ.get("FDR_ROLLOUT", "auto")
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    pair = mode == "pair" or (mode != "single" and lanes >= 16 * cus)
    return ("rollout_pair_kernel<%d,%d,%s> (two lanes per wave)" if pair else
            "rollout_kernel<%d,%d,%s,synth> (one lane per wave)") % (n_in, n_act, kind)


def lane_step_flops(kind, n_in, n_act):
    """Algorithmic FLOPs per (lane, env step): 2 x MACs of the policy MLP + the env dynamics."""
    nout = n_act if kind == "discrete" else 2 * n_act
    policy = n_in * 64 + 64 * 64 + 64 * nout
    env = n_in * n_in + (0 if kind == "discrete" else n_in * n_act)
    return 2 * (policy + env)


# ------------------------------------------------------------------------------------------------
# CPU baseline (oracle restatement of the reference's per-lane loop), forked before any GPU use
# ------------------------------------------------------------------------------------------------
def _cpu_worker_impala(wid, seconds, T):
    """Per-env reference loop on one core, WHOLE episodes (at least one, then until `seconds`): ImpalaCNN torch-CPU
    forward per step (oracle restatement of policies/impala.py + worker/agent.py:35-55), perturbed theta, synthetic
    frames, then the end-of-episode entropy pass over every visited obs (worker/agent.py:60-66, the LSTM replayed
    from the end state).  -> (env steps, whole episodes, elapsed s)."""
    import numpy as np
    import torch
    from oracle import impala as oi
    from oracle import rng as crng
    torch.manual_seed(124)
    P = oi.num_params(6)
    theta = (torch.randn(P) * 0.01).numpy()
    bn = oi.split_bn(np.zeros(oi.num_bn(), np.float32), np.ones(oi.num_bn(), np.float32))
    rs = np.random.RandomState(wid)
    steps = episodes = 0
    t0 = time.perf_counter()
    while episodes == 0 or time.perf_counter() - t0 < seconds:
        p = oi.unflatten((theta + np.float32(0.02) * rs.randn(P).astype(np.float32)).astype(np.float32), 6)
        h, c, r = torch.zeros(1, 256), torch.zeros(1, 256), np.zeros(1, np.float32)
        cis = []
        for t in range(T):
            fr = oi.frames(5, [wid], t).astype(np.float32)
            pr, h, c, _, ci = oi.forward(p, bn, fr, r, h, c)
            cis.append(ci)
            a = oi.categorical_inverse_cdf(pr.numpy()[0], crng.uniform(7, wid, t, 0))
            r = oi.rewards(5, [wid], t, [a], 6)
        eh, ec = h, c
        for t in range(T):
            pe, eh, ec = oi.lstm_head(p, bn, cis[t], eh, ec)
            oi.categorical_entropy(pe)
        steps += T
        episodes += 1
    return steps, episodes, time.perf_counter() - t0


def _cpu_worker(args):
    wid, seconds, cfg = args
    import torch
    torch.set_num_threads(1)                      # run_client.py:15
    kind, n_in, n_act, _, T = CONFIGS[cfg]
    if kind == "impala":
        return _cpu_worker_impala(wid, seconds, T)
    from oracle import agent
    return agent.reference_collect_loop(kind, n_in, n_act, T, seconds, wid)


def _cpu_learner(args):
    P, n = args
    import torch
    torch.set_num_threads(1)
    from oracle import agent
    return agent.reference_learner_step_seconds(P, n)


def cpu_cores():
    """Host cores this process may use: the affinity set, capped by the harness's CPU share
    (OMP_NUM_THREADS = 16 per GPU on the box; os.cpu_count() there reports the whole machine)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    share = os.environ.get("OMP_NUM_THREADS")
    return max(1, min(n, int(share))) if share and share.isdigit() else max(1, n)


def cpu_baseline(cfg, seconds, cores, lanes, n_params, T):
    """Oracle restatement of SequentialRunner.train's worker + learner (run_sequential.py:113-179) on `cores`
    processes: env steps/s from whole reference-shaped episodes, and sec per FD step = lanes x T env steps at
    that rate + the restated FiniteDifferences.step on `lanes` returns (one core)."""
    ctx = multiprocessing.get_context("fork")
    with ctx.Pool(cores) as pool:
        res = pool.map(_cpu_worker, [(i, seconds, cfg) for i in range(cores)])
        n_learn = lanes if n_params * lanes <= 64e6 else 64
        learn_s = pool.apply(_cpu_learner, ((n_params, n_learn),)) * lanes / n_learn
    steps = sum(r[0] for r in res)
    episodes = sum(r[1] for r in res)
    wall = max(r[2] for r in res)
    rate = steps / wall
    return rate, steps, episodes, lanes * T / rate + learn_s, learn_s, n_learn


def bench_trap(args):
    """BASELINE config 1: run_sequential.py on custom_envs.simple_trap_env, DiscretePolicy(2, 9), 16 perturbations.
    The reference runs it on the CPU only; its cpu_baseline here is the restated SequentialRunner.train loop
    (oracle/runner.run_trap, run_sequential.py:113-179) timed epoch by epoch on one core (the reference's runner is
    one single-threaded process), and `value` is the product SequentialRunner (one rollout launch of the trap env
    per epoch + the device learner) on cuda:0.  A step is one train epoch."""
    import numpy as np
    cpu = None
    if not args.no_cpu_baseline:
        import torch
        torch.set_num_threads(1)
        from oracle import runner as orun
        secs = []
        n_ep = max(3, int(args.cpu_seconds / 0.6))
        t0 = time.perf_counter()
        out = orun.run_trap(n_ep, epoch_seconds=secs)
        wall = time.perf_counter() - t0
        rate = out["cum_steps"] / sum(secs)
        cpu = {"value": round(rate, 1), "unit": "env steps/s", "cores": 1, "kind": "port",
               "sec_per_fd_step": round(float(np.median(secs)), 4),
               "sample": "%d epochs of oracle/runner.run_trap (SequentialRunner.train restated: 16 returns per epoch, "
                         "per-step torch forward + injected-uniform sampling, learner step; %.1f s incl. setup), "
                         "%d env steps; sec_per_fd_step = median epoch" % (n_ep, wall, out["cum_steps"]),
               "reference_equivalent": {"value": round(rate / CPU_CALIBRATION["trap"], 1),
                                        "oracle_over_reference": CPU_CALIBRATION["trap"],
                                        "note": "the reference's own SequentialRunner.train on the trap env timed beside "
                                                "run_trap in the build container (profiles/r06_cpu_calibration.txt)"}}
    import torch
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    from run_sequential import SequentialRunner
    runner = SequentialRunner(env_id="SimpleTrapEnv-v0", batch_size=16, random_seed=124, zeta_size=4,
                              max_strategy_history_size=4, device=dev, verbose=False)
    for _ in range(max(1, args.warmup)):
        runner.train(1)
    torch.cuda.synchronize()
    s0 = runner.agent.cumulative_timesteps
    t0 = time.perf_counter()
    for _ in range(args.steps):
        runner.train(1)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    steps = runner.agent.cumulative_timesteps - s0
    line = {"metric": METRIC, "value": round(steps / el, 1), "unit": "env steps/s", "n_gpus": 1, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(el / args.steps * 1e3, 4),
            "sec_per_fd_step": round(el / args.steps, 6), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f32", "data": "synthetic",
            "config": {"workload": "BASELINE config 1: run_sequential.py SequentialRunner on custom_envs.simple_trap_env "
                                   "(the reference's map, integer-exact GPU env), DiscretePolicy(2, 9) P=%d, 16 "
                                   "perturbations per epoch, T=201; a step = one train epoch (rollout launch + FD "
                                   "step + the host bookkeeping of run_sequential.py:113-179)" % runner.policy.num_params,
                       "parallelism": "dp1"},
            "roofline": None, "cpu_baseline": cpu,
            "note": "plumbing config (the reference's CPU-only smoke test): launch- and host-bound by construction"}
    print(json.dumps(line), flush=True)


# ------------------------------------------------------------------------------------------------
def check_devices(n):
    """Exit non-zero unless n GPUs are visible.  torch.cuda.device_count() counts devices without starting the
    HIP runtime on this image, so the self-launching parent stays GPU-free."""
    import torch
    have = torch.cuda.device_count()
    if n > have:
        sys.exit("bench.py: %d GPU(s) requested but %d visible" % (n, have))


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def self_launch(n, rehearse):
    """`bench.py --gpus N` with no external launcher: one fresh process per GPU through torch.distributed.run
    (the replacement for the reference's N worker clients, run_client.py:46-53 / run_server.py:135-167).  This
    process never touches the GPU (no exec from a GPU-initialised process); it relays the children's output and
    exits with their status, non-zero also when rank 0's line is missing or does not report N GPUs."""
    import subprocess
    if not rehearse:
        check_devices(n)
    port = os.environ.get("MASTER_PORT") or str(_free_port())
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", port, os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True, env=env, cwd=REPO)
    lines = []
    for line in p.stdout:
        sys.stdout.write(line)
        sys.stdout.flush()
        if line.startswith("{"):
            lines.append(line)
    rc = p.wait()
    if rc != 0:
        sys.exit(rc)
    if len(lines) != 1:
        sys.exit("bench.py: expected ONE JSON line from rank 0, got %d" % len(lines))
    got = json.loads(lines[0]).get("n_gpus")
    if got != n:
        sys.exit("bench.py: rank 0 reports n_gpus=%s, %d were requested" % (got, n))
    return 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (ranks) of the run; default 1, or WORLD_SIZE under an external launcher")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="halfcheetah", choices=list(CONFIGS) + ["trap"])
    ap.add_argument("--perturbations", type=int, default=None,
                    help="antithetic lanes per GPU (default: the BASELINE config's -- 4096 halfcheetah, "
                         "1024 cartpole, 1024 x 4 envs impala)")
    ap.add_argument("--episode-len", type=int, default=None)
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-variant", action="store_true", help="skip the 4096-pair variant line (config 3)")
    ap.add_argument("--settle-ms", type=float, default=100.0,
                    help="after the W warmup steps, further untimed FD steps until this much wall time has passed "
                         "since the first warmup step: the GPU's clocks ramp over the first ~30 ms of sustained load "
                         "(config 3 rollout 1.24 -> 1.06 ms over its first 25 launches, rocprofv3 trace, DESIGN.md 7); "
                         "0 disables")
    ap.add_argument("--timing-steps", type=int, default=10,
                    help="FD steps of the rollout-timing pass that follows the timed region (HIP events around "
                         "each rollout; Impala: the in-rollout conv/core phase events)")
    ap.add_argument("--no-novelty", action="store_true", help="config 5 without the novelty archive / omega "
                    "(rocprof passes: the archive's conv launches would mix into the rollout conv's average)")
    args = ap.parse_args()
    rehearse = os.environ.get("FDR_BENCH_REHEARSE") == "1"
    ext_world = os.environ.get("WORLD_SIZE")
    if ext_world is None:
        n = 1 if args.gpus is None else args.gpus
        if n < 1:
            sys.exit("bench.py: --gpus must be >= 1 (got %d)" % n)
        if n > 1:
            if args.config == "trap":
                sys.exit("bench.py: --config trap is BASELINE config 1, a single-process run (--gpus 1)")
            return self_launch(n, rehearse)
    else:
        if args.gpus is not None and args.gpus != int(ext_world):
            sys.exit("bench.py: --gpus %d disagrees with WORLD_SIZE=%s set by the launcher" % (args.gpus, ext_world))
    if args.config == "trap":
        return bench_trap(args)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if not rehearse:
        check_devices(max(world, local_rank + 1))
    kind, n_in, n_act, env_name, T = CONFIGS[args.config]
    if args.episode_len:
        T = args.episode_len

    L = args.perturbations or (IMPALA_LANES if kind == "impala" else DEFAULT_LANES.get(args.config, 4096))
    E = IMPALA_ENVS if kind == "impala" else 1
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle import impala as oimp
        from oracle import policies as opol
        P = oimp.num_params(n_act) if kind == "impala" else opol.num_params(kind, n_in, n_act)
        cores = cpu_cores()
        v, steps, eps, fd_s, learn_s, n_learn = cpu_baseline(args.config, args.cpu_seconds, cores, L * E, P, T)
        ratio = CPU_CALIBRATION.get(args.config)
        cpu = {"value": round(v, 1), "unit": "env steps/s", "cores": cores, "kind": "port",
               "sec_per_fd_step": round(fd_s, 3), "per_core": round(v / cores, 1),
               "reference_equivalent": None if ratio is None else {
                   "value": round(v / ratio, 1), "per_core": round(v / cores / ratio, 1), "oracle_over_reference": ratio,
                   "note": "the reference's own Worker.collect_returns timed beside this loop in the build container "
                           "(tools/cpu_calibrate.py, profiles/r06_cpu_calibration.txt); SURVEY 6's 9.5 k/core was "
                           "measured on that container's CPU, not this host's"},
               "whole_episodes": eps,
               "sample": ("%d processes x %.0f s of the oracle's reference-shaped loop (worker/worker.py:20-57 + "
                          "worker/agent.py:20-71: perturb, per-step batch-1 torch forward + torch %s sampling, "
                          "env.step, end-of-episode entropy forward; 1 thread each as run_client.py:15; T=%d): "
                          "%d env steps, %d whole episodes; sec_per_fd_step = %d lanes x T env steps at that rate "
                          "+ FiniteDifferences.step restated on %d returns (%.3f s%s)"
                          % (cores, args.cpu_seconds, "Categorical" if kind != "mujoco" else "Normal", T, steps,
                             eps, L * E, n_learn, learn_s,
                             ", scaled linearly from the sample" if n_learn != L * E else ""))}

    import numpy as np
    import torch
    import torch.distributed as dist

    # FDR_BENCH_REHEARSE=1: rehearse the N-rank path on a one-GPU box (every rank on cuda:0, gloo) -- the
    # exchange protocol, the collective settle and the max-over-ranks timing; not a scaling measurement
    dev_index = 0 if rehearse else local_rank
    torch.cuda.set_device(dev_index)
    dev = torch.device("cuda", dev_index)
    # FDR_FORCE_COLLECTIVES=1 under a one-rank launcher: the N > 1 exchange on a process group of one (RCCL path check)
    from fdr import dist as fdist
    if world > 1 or (fdist.FORCE and "WORLD_SIZE" in os.environ):
        if rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)

    from dsgd import DSGD
    from envs import FrameEnv, SyntheticEnv
    from fdr import engine
    from learner import FiniteDifferences
    from policies import DiscretePolicy, ImpalaPolicy, MujocoPolicy
    from utils import AdaptiveOmega, SharedNoiseTable
    from worker import Agent, Worker

    torch.manual_seed(124)
    impala = kind == "impala"
    fp16 = False
    if impala:
        policy = ImpalaPolicy(n_in, n_act, seed=124, device=dev)
        fp16 = args.config == "impala_fp16"
        env = FrameEnv(n_act, episode_len=T, envs_per_lane=IMPALA_ENVS, env_seed=5, fp16=fp16)
    else:
        Pol = DiscretePolicy if kind == "discrete" else MujocoPolicy
        policy = Pol(n_in, n_act, seed=124, device=dev)
        env = SyntheticEnv.named(env_name, device=dev, episode_len=T)
    table = SharedNoiseTable(25_000_000, policy.num_params, random_seed=124)
    table.device_table(dev)
    agent = Agent(policy, env, random_seed=124)   # rank-independent: lane streams are keyed by global lane id
    worker = Worker(policy, agent, table, None, sigma=0.02, random_seed=124)
    omega = AdaptiveOmega()
    learner = FiniteDifferences(policy, DSGD(policy.parameters(), lr=0.01), omega, table, noise_std=0.02)

    novelty = args.config == "impala_fp16" and not args.no_novelty     # config 5: strategy.sparse_history_manager + utils.adaptive_omega
    if novelty:
        from strategy import StrategyHandler
        from utils import math_helpers
        from run_sequential import SequentialRunner
        handler = StrategyHandler(policy, math_helpers.categorical_tvd, max_history_size=200, fp16=True)
        # zeta: ZETA_SIZE obs of random-action steps (run_sequential.py:198-213); archive: the policy + 3 nearby
        zeta = SequentialRunner._random_action_obs(_ZetaSource(env, dev), ZETA_SIZE)
        flat = policy.get_trainable_flat()
        rs = np.random.RandomState(0)
        handler.points = [flat] + [(flat + 0.02 * rs.randn(flat.size)).astype(np.float32) for _ in range(3)]
        handler.set_zeta(zeta)
        worker.strategy_handler = handler

    n_dirs_global = (L // 2) * world
    from fdr import dist as fdist
    lane_range = fdist.lane_range(n_dirs_global, 2, world, rank)
    roll_ms = []
    phase_ms = []
    step_no = [0]
    # HIP event pairs bracketing each rollout, created and first recorded before the timed region (a fresh
    # event's first record allocates its signal: that is not work of the step)
    ev_pool = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
               for _ in range(max(args.steps, 10) + 1)]
    for a_, b_ in ev_pool:
        a_.record()
        b_.record()
    torch.cuda.synchronize()
    cur = [None]
    host_ms = [None]  # the timed loop's host enqueue time per step (before the closing synchronize)

    def fd_step(timed, n_dirs=n_dirs_global, rng=lane_range):
        timed = timed and cur[0] is not None
        # the action stream is keyed by (step seed, global lane id): every rank evaluates the lanes of a
        # 1-GPU run bit-identically, whatever the shard (include/fdr.h lane_offset)
        seed = 1000 + step_no[0]
        step_no[0] += 1
        # the events bracket the rollout launch alone (Worker.launch), not the host index draw before it
        batch = worker.evaluate(n_dirs, antithetic=True, lane_range=rng, seed=seed, novelty=novelty, prefetch=True,
                                timing=cur[0] if timed else None)
        out = learner.step_async(batch, 0.0, 0.0, 0.0)
        if novelty:
            # run_sequential.py:149-151 (the noisy mean reward; one host read per FD step) and :160
            omega.step(float(batch.reward.mean().item()))
            handler.add_policy(policy)
        if timed and impala:
            phase_ms.append(engine.impala_profile_read())
        return out, batch

    def timed_loop(steps, events=False, **kw):
        # events=False: the timed region carries no instrumentation (an event record on the stream costs
        # ~5 us of barrier processing at each kernel boundary it sits on: rocprofv3 trace);
        # the rollout's own time comes from a separate pass with events=True
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        prof = None
        if os.environ.get("FDR_HOST_PROFILE") and not events:  # diagnostics: the host side of the timed steps
            import cProfile
            prof = cProfile.Profile()
            prof.enable()
        t0 = time.perf_counter()
        pairs = []
        out = None
        for i in range(steps):
            cur[0] = ev_pool[i % len(ev_pool)] if events else None
            out, _ = fd_step(True, **kw)
            if cur[0] is not None:
                pairs.append(cur[0])
        t_host = time.perf_counter() - t0
        host_ms[0] = t_host / steps * 1e3
        if prof is not None:
            prof.disable()
            prof.dump_stats(os.environ["FDR_HOST_PROFILE"])
            print("host time of the timed loop (enqueue only): %.1f us per step" % (t_host / steps * 1e6),
                  file=sys.stderr)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        return el, [a_.elapsed_time(b_) for a_, b_ in pairs], out

    t_warm = time.perf_counter()
    for _ in range(args.warmup):
        out, _ = fd_step(False)
    # clock settle: untimed steps in chunks of 5 (one sync per chunk) until settle_ms of sustained load
    # (N > 1: the ranks decide together, so every rank runs the same FD steps and collectives)
    settle_steps = 0
    while args.settle_ms > 0:
        torch.cuda.synchronize()
        go = (time.perf_counter() - t_warm) * 1e3 < args.settle_ms
        if world > 1:
            t = torch.tensor([1 if go else 0], dtype=torch.int64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            go = bool(t.item())
        if not go:
            break
        for _ in range(5):
            out, _ = fd_step(False)
        settle_steps += 5
    elapsed, _, out = timed_loop(args.steps)
    host_enqueue_ms = host_ms[0]
    # rollout-timing pass (outside the timed region): HIP events bracketing each rollout on its stream,
    # and for Impala the per-step-loop phase events of fdr_impala_profile
    if impala:
        engine.impala_profile(True)
    _, roll_ms, _ = timed_loop(max(1, min(args.steps, args.timing_steps)), events=True)
    if impala:
        engine.impala_profile(False)
    rollout_ms = float(np.mean(roll_ms))
    if world > 1:
        t = torch.tensor([elapsed, rollout_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, rollout_ms = t.tolist()
    upd, gnorm = out.tolist()
    assert gnorm > 0 and np.isfinite(upd)
    conv_phase = None
    if impala:
        conv_phase = [float(np.mean([p[i] for p in phase_ms])) for i in range(3)]
        phase_ms.clear()

    variants = {}
    if not impala and args.config == "halfcheetah" and not args.no_variant:
        # also report the 4096-pair variant (4096 directions x +-, 8192 lanes per GPU)
        nv = 2 * n_dirs_global
        rng2 = fdist.lane_range(nv, 2, world, rank)
        fd_step(False, n_dirs=nv, rng=rng2)
        k = max(1, min(args.steps, 10))
        el2, _, out2 = timed_loop(k, n_dirs=nv, rng=rng2)
        _, ms2, _ = timed_loop(k, events=True, n_dirs=nv, rng=rng2)
        r2 = float(np.mean(ms2))
        if world > 1:
            t = torch.tensor([el2, r2], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el2, r2 = t.tolist()
        lanes2 = 2 * L
        variants["4096_pairs"] = {
            "value": round(lanes2 * T * world * k / el2, 1), "unit": "env steps/s", "steps": k,
            "ms_per_step": round(el2 / k * 1e3, 4), "sec_per_fd_step": round(el2 / k, 6),
            "perturbations_per_gpu": lanes2, "directions_per_gpu": lanes2 // 2, "rollout_ms": round(r2, 4),
            "roofline_frac": round(lane_step_flops(kind, n_in, n_act) * lanes2 * T / (r2 * 1e-3) / 1e12
                                   / FP32_PEAK_TFLOPS, 4),
            "kernel": rollout_kernel_name(kind, n_in, n_act, lanes2, dev)}

    lane_steps = L * E * T * world * args.steps
    value = lane_steps / elapsed
    prof = None
    pmc = os.path.join(REPO, "profiles", "pmc_rollout_%s.json" % args.config)
    if os.path.exists(pmc):
        with open(pmc) as f:
            prof = json.load(f)
    traffic = None if prof is None else prof.get("hbm_bytes_per_launch")
    if impala:
        conv_ms, core_ms, replay_ms = conv_phase
        if world > 1:
            t = torch.tensor([conv_ms, core_ms, replay_ms], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            conv_ms, core_ms, replay_ms = t.tolist()
        conv_launch_ms = conv_ms / T
        achieved_tf = IMPALA_CONV_FLOP * L * E / (conv_launch_ms * 1e-3) / 1e12
        core_bytes = IMPALA_CORE_BYTES // (2 if fp16 else 1)
        # antithetic pairs (fdr_impala_desc.pairs): one sigma-eps stream per pair from HBM + theta's shared pack
        # (L2 / MALL-resident) -- the algorithmic HBM bytes are half the per-lane stream's
        core_hbm = core_bytes * (L // 2 + 1)
        core_gbs = core_hbm / (core_ms / T * 1e-3) / 1e9
        peak = FP16_PEAK_TFLOPS if fp16 else FP32_PEAK_TFLOPS
        core_prof = None if prof is None else prof.get("core_kernel")
        roofline = {"bound": "mfma", "achieved": round(achieved_tf, 3), "peak": peak, "unit": "TFLOP/s",
                    "frac": round(achieved_tf / peak, 4), "traffic": traffic,
                    "kernel": ("impala conv_kernel_h2 (15 convs, v_mfma_f32_16x16x32_f16; 2 x 8 waves / CU)"
                               if fp16 else "impala conv_kernel (15 convs, v_mfma_f32_16x16x4_f32)"),
                    "conv_launch_ms": round(conv_launch_ms, 4), "flop_per_env_step": IMPALA_CONV_FLOP,
                    "envs_per_launch": L * E, "rollout_ms": round(rollout_ms, 3),
                    "mfma_busy_pmc": None if prof is None else prof.get("mfma_busy"),
                    "core_kernel": {"bound": "hbm", "achieved": round(core_gbs, 1), "peak": HBM_PEAK_GBS,
                                    "unit": "GB/s", "frac": round(core_gbs / HBM_PEAK_GBS, 4),
                                    "launch_ms": round(core_ms / T, 4), "bytes_per_lane_step": core_bytes,
                                    "hbm_bytes_per_launch_algorithmic": core_hbm,
                                    "form": ("pair on MFMA: theta x + s (E x) over fragment images, two pairs "
                                             "per workgroup (core_kernel_hpm2)" if fp16 else "pair (theta + s sigma-eps)"),
                                    "traffic": None if core_prof is None else core_prof.get("hbm_bytes_per_launch")},
                    "entropy_replay_ms": round(replay_ms, 3),
                    "profile": None if prof is None else "profiles/%s_summary.md" % prof.get("tag"),
                    "note": ("dense f16 MFMA peak" if fp16 else "f32 MFMA peak (= f32 vector peak)") +
                            "; conv time from HIP events between the step-loop launches (fdr_impala_profile); "
                            "traffic / mfma_busy_pmc: rocprofv3 PMC of the same command (profile)"}
        workload = ("BASELINE config %d per GPU: ImpalaPolicy(A=%d) P=%d, %d perturbations (%d directions x +/-) x "
                    "%d envs each, synthetic 3x64x64 frames, T=%d, %s, full FD step (rollout + entropy pass + "
                    "weights + gradient + DSGD%s)" % (5 if fp16 else 4, n_act, policy.num_params, L, L // 2, E, T,
                                                      "fp16 rollouts" if fp16 else "f32",
                                                      " + lane novelty vs a TVD strategy archive over %d zeta obs + "
                                                      "AdaptiveOmega step" % ZETA_SIZE if novelty else ""))
    else:
        flops = lane_step_flops(kind, n_in, n_act) * L * T
        achieved_tf = flops / (rollout_ms * 1e-3) / 1e12
        hbm = None
        if traffic:
            gbs = traffic / (rollout_ms * 1e-3) / 1e9
            hbm = {"traffic_bytes_per_launch": traffic, "achieved": round(gbs, 1), "unit": "GB/s",
                   "peak": HBM_PEAK_GBS, "frac": round(gbs / HBM_PEAK_GBS, 5)}
        roofline = {"bound": "valu", "achieved": round(achieved_tf, 3), "peak": FP32_PEAK_TFLOPS,
                    "unit": "TFLOP/s", "frac": round(achieved_tf / FP32_PEAK_TFLOPS, 4), "traffic": traffic,
                    "kernel": rollout_kernel_name(kind, n_in, n_act, L, dev),
                    "rollout_ms": round(rollout_ms, 4),
                    "flop_per_lane_step": lane_step_flops(kind, n_in, n_act),
                    "hbm": hbm,
                    "profile": None if prof is None else "profiles/%s_summary.md" % prof.get("tag"),
                    "note": "f32 VALU peak (v_pk_fma_f32; = the f32 MFMA peak on gfx950): theta' is VGPR/LDS-resident "
                            "for the whole episode, so the kernel is VALU-issue bound; its HBM traffic (PMC "
                            "FETCH_SIZE x2 + WRITE_SIZE of the same kernel, 'profile') is the noise-table gather once "
                            "per episode"}
        workload = ("BASELINE config 3: HalfCheetah-shaped synthetic env (obs 17, act 6), MujocoPolicy(17,6) P=%d, "
                    "%d antithetic perturbations per GPU (%d directions x +/-), T=%d fixed-length episodes, full FD "
                    "step (rollout + weights + gradient + DSGD)" % (policy.num_params, L, L // 2, T)
                    if args.config == "halfcheetah" else
                    "BASELINE config 2: CartPole-shaped synthetic env (obs 4, 2 actions), DiscretePolicy(4,2) P=%d, "
                    "%d antithetic perturbations (%d directions x +/-), T=%d, full FD step" % (
                        policy.num_params, L, L // 2, T) if args.config == "cartpole" else args.config)
    line = {
        "metric": METRIC,
        "value": round(value, 1),
        "unit": "env steps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup, "settle_steps": settle_steps,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "sec_per_fd_step": round(elapsed / args.steps, 6),
        # the timed loop's host time per step before its closing synchronize; the upload ring bounds the host's lead
        # (Worker._lanes_to_device), so it includes waiting: < ms_per_step means the GPU, not the host, paces the job
        "host_enqueue_ms_per_step": round(host_enqueue_ms, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f16" if (impala and fp16) else "f32",
        "data": "synthetic",
        "config": {"workload": workload, "perturbations_per_gpu": L, "envs_per_perturbation": E,
                   "global_perturbations": L * world, "episode_len": T, "n_params": policy.num_params,
                   "parallelism": "dp%d" % world},
        "roofline": roofline,
        "cpu_baseline": cpu,
        "variants": variants or None,
        "update_norm": upd,
    }
    if novelty:
        line["config"]["novelty"] = {"archive": len(handler.points), "zeta": ZETA_SIZE, "omega": omega.omega}
    if fdist.FORCE and world == 1 and dist.is_initialized():  # only when a group ran
        line["config"]["collectives"] = "forced on a one-rank process group (FDR_FORCE_COLLECTIVES=1)"
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


class _ZetaSource(object):
    """The attributes SequentialRunner._random_action_obs reads (env, device, rng)."""

    def __init__(self, env, dev):
        import numpy as np
        self.env, self.device, self.rng = env, dev, np.random.RandomState(124)


if __name__ == "__main__":
    main()
