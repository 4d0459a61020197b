"""Calibrate the on-box CPU baseline against the REFERENCE itself (build container only: needs /root/reference).

bench.py's cpu_baseline times the oracle's restatement of the reference's per-lane loop
(oracle/agent.py reference_collect_loop) because the reference cannot travel to the GPU box.  This script runs,
in one process on one thread (run_client.py:15), alternately:
  * the reference's own Worker.collect_returns -> Agent.collect_return (worker/worker.py:20-57,
    worker/agent.py:20-71) with its MujocoPolicy / DiscretePolicy on the build's synthetic envs, and
  * the oracle loop bench.py uses,
and the reference's SequentialRunner.train on the trap env (BASELINE config 1; run_sequential.py:113-179 with
SURVEY 8c's harness patches, via tests/golden/make_golden.py's import shim) against oracle/runner.run_trap, so the
oracle loop's per-core rate can be stated relative to the reference's on the same machine.  Writes its report to
stdout (committed as profiles/r06_cpu_calibration.txt).

    python tools/cpu_calibrate.py [--seconds 8]
"""
import argparse
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(REPO, "tests", "golden"))
import make_golden as mg  # noqa: E402  (gym / wandb stubs, the reference on sys.path, bytecode writing off)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def ref_worker_rate(kind, n_in, n_act, T, seconds):
    env = mg.SyntheticEnv(n_in, n_act, kind == "discrete", T, env_seed=0)
    pol = mg.make_policy(kind, n_in, n_act, 124)
    table = mg.SharedNoiseTable(2 ** 22, pol.num_params, random_seed=124)
    agent = mg.Agent(pol, env, random_seed=11)
    handler = mg.StrategyHandler(pol, mg.math_helpers.categorical_tvd)
    worker = mg.Worker(pol, agent, table, handler, sigma=0.02, eval_prob=0.0, random_seed=3)
    steps, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        steps += sum(r.timesteps for r in worker.collect_returns(1))
    return steps / (time.perf_counter() - t0)


def oracle_worker_rate(kind, n_in, n_act, T, seconds):
    from oracle import agent
    s, _, el = agent.reference_collect_loop(kind, n_in, n_act, T, seconds, 0)
    return s / el


def ref_trap_epochs(n_epochs):
    """The reference SequentialRunner.train on the trap env with SURVEY 8c's three harness patches only (as
    make_golden.g6_runner_trap, without its action-noise injection: the reference's own torch sampling)."""
    import contextlib
    import io
    mg._ENV_FACTORY["SimpleTrapEnv-v0"] = mg._trap_env
    rs_orig, up_orig = mg.run_sequential.RNGNoiseSource, mg.Worker.update
    mg.run_sequential.RNGNoiseSource = lambda n, random_seed=123: mg.SharedNoiseTable(2 ** 22, n, random_seed)

    def update(self, state):
        self.policy.set_trainable_flat(state.policy_params)
        self.epoch = state.epoch
        if state.obs_stats is not None:
            self.fixed_obs_stats.deserialize(state.obs_stats)
    mg.Worker.update = update
    try:
        runner = mg.run_sequential.SequentialRunner(env_id="SimpleTrapEnv-v0", batch_size=16, random_seed=124,
                                                    zeta_size=4, max_strategy_history_size=4)
        runner.learner.noise_std = 0.02
        t0 = time.perf_counter()
        with contextlib.redirect_stdout(io.StringIO()):
            runner.train(n_epochs)
        return runner.agent.cumulative_timesteps, time.perf_counter() - t0
    finally:
        mg.run_sequential.RNGNoiseSource, mg.Worker.update = rs_orig, up_orig


def oracle_trap_epochs(n_epochs):
    from oracle import runner
    t0 = time.perf_counter()
    out = runner.run_trap(n_epochs)
    return out["cum_steps"], time.perf_counter() - t0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=8.0)
    ap.add_argument("--trap-epochs", type=int, default=6)
    args = ap.parse_args()
    torch.set_num_threads(1)
    print("CPU calibration: reference vs oracle loop, 1 thread, same process, alternating (%s)"
          % time.strftime("%Y-%m-%d"))
    for name, kind, n_in, n_act, T in (("halfcheetah", "mujoco", 17, 6, 1000), ("cartpole", "discrete", 4, 2, 500)):
        ref, orc = [], []
        for _ in range(2):
            ref.append(ref_worker_rate(kind, n_in, n_act, T, args.seconds))
            orc.append(oracle_worker_rate(kind, n_in, n_act, T, args.seconds))
        print("%-12s reference Worker.collect_returns %8.0f env steps/s   oracle reference_collect_loop %8.0f"
              "   oracle / reference = %.2f" % (name, np.mean(ref), np.mean(orc), np.mean(orc) / np.mean(ref)))
    rs, rt = ref_trap_epochs(args.trap_epochs)
    os_, ot = oracle_trap_epochs(args.trap_epochs)
    print("trap (config 1) %d epochs x 16: reference SequentialRunner.train %.0f env steps/s (%.3f s/epoch)   "
          "oracle run_trap %.0f env steps/s (%.3f s/epoch)   oracle / reference = %.2f"
          % (args.trap_epochs, rs / rt, rt / args.trap_epochs, os_ / ot, ot / args.trap_epochs, (os_ / ot) / (rs / rt)))


if __name__ == "__main__":
    main()
