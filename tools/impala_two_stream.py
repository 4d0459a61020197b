"""Feasibility probe: config 5's rollout as two lane halves on two HIP streams (conv of one half beside the
HBM-bound core step of the other) against one launch sequence over all lanes.  Same lanes, same results
(lane_offset keys the counter streams); prints both times and the max |reward difference|.

    python tools/impala_two_stream.py [--lanes 1024 --envs 4 --T 100 --reps 3]"""
import argparse
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "dfd-starter_amd"))
from fdr import _lib, engine  # noqa: E402
from fdr._lib import lib, check  # noqa: E402


def launch(spec, lanes, n, seed, out, ws, stream, dev):
    d = spec.desc()
    check(lib.fdr_impala_rollout(engine._c(dev, None), ctypes.byref(d), ctypes.byref(lanes), n,
                                 ctypes.c_uint64(seed), 1, engine._p(out[0]), engine._p(out[1]), engine._p(out[2]),
                                 engine._p(out[3]), None, None, engine._p(ws), ws.numel(),
                                 ctypes.c_void_p(stream.cuda_stream)), "fdr_impala_rollout")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lanes", type=int, default=1024)
    ap.add_argument("--envs", type=int, default=4)
    ap.add_argument("--T", type=int, default=100)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--splits", type=int, default=2)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    A, L, E, T = 4, args.lanes, args.envs, args.T
    P = engine.impala_num_params(A)
    torch.manual_seed(0)
    theta = (torch.randn(P) * 0.02).to(dev)
    table = torch.randn(P + 100_000).to(dev)
    idx = torch.randint(0, 100_000, (L // 2,), dtype=torch.int64).repeat_interleave(2).to(dev)
    sign = torch.tensor([1, -1], dtype=torch.int8).repeat(L // 2).to(dev)
    spec = engine.ImpalaSpec(A, E, T, entropy=True, fp16=True, pairs=True)

    def outs(n):
        return (torch.empty(n * E, dtype=torch.float64, device=dev), torch.empty(n * E, dtype=torch.float64, device=dev),
                torch.empty(n * E, dtype=torch.int32, device=dev), torch.empty(n, dtype=torch.float64, device=dev))

    def wsz(n):
        return torch.empty(lib.fdr_impala_workspace_bytes(ctypes.byref(spec.desc()), n), dtype=torch.uint8, device=dev)

    S = args.splits
    h = L // S
    full_lanes = engine.lanes_desc(theta, 0, table, idx, sign, 0.02)
    part = [engine.lanes_desc(theta, 0, table, idx[i * h:(i + 1) * h], sign[i * h:(i + 1) * h], 0.02, lane_offset=i * h)
            for i in range(S)]
    o_full, ws_full = outs(L), wsz(L)
    o_part, ws_part = [outs(h) for _ in range(S)], [wsz(h) for _ in range(S)]
    streams = [torch.cuda.Stream(dev) for _ in range(S)]
    main_s = torch.cuda.current_stream(dev)

    def run_full():
        launch(spec, full_lanes, L, 5, o_full, ws_full, main_s, dev)

    def run_split():
        ev = torch.cuda.Event()
        ev.record(main_s)
        for i in range(S):
            streams[i].wait_event(ev)
            launch(spec, part[i], h, 5, o_part[i], ws_part[i], streams[i], dev)
        for i in range(S):
            e = torch.cuda.Event()
            e.record(streams[i])
            main_s.wait_event(e)

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(main_s)
        fn()
        b.record(main_s)
        torch.cuda.synchronize()
        return a.elapsed_time(b)

    for rep in range(args.reps):
        tf = timed(run_full)
        ts = timed(run_split)
        r_full = o_full[0].cpu()
        r_split = torch.cat([o[0].cpu() for o in o_part])
        print("rep %d: one sequence %.2f ms, %d streams %.2f ms (%.3fx); max |dret| %.3g, entropy %.3g" % (
            rep, tf, S, ts, tf / ts, (r_full - r_split).abs().max().item(),
            (o_full[1].cpu() - torch.cat([o[1].cpu() for o in o_part])).abs().max().item()), flush=True)


if __name__ == "__main__":
    main()
