"""Per-workgroup timeline of conv_kernel_h2 (diagnostics build with -DFDR_WG_TIMELINE: every workgroup's start /
end in s_memrealtime ticks (100 MHz) + HW_ID / XCC_ID).  Answers: how long one env's workgroup lives, how evenly the
16 envs per CU are dealt, and how much of the launch is dispatch gaps and tail.

    FDR_LIB=dfd-starter_amd/fdr/libfdr_tl.so python tools/impala_wg_timeline.py [--lanes 1024 --envs 4]"""
import argparse
import collections
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "dfd-starter_amd"))
from fdr import engine  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lanes", type=int, default=1024)
    ap.add_argument("--envs", type=int, default=4)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    A = 4
    P = engine.impala_num_params(A)
    torch.manual_seed(0)
    theta = (torch.randn(P) * 0.02).cuda()
    table = torch.randn(P + 4096).cuda()
    idx = torch.randint(0, 4096, (args.lanes,), dtype=torch.int64).cuda()
    sign = torch.ones(args.lanes, dtype=torch.int8).cuda()
    lanes = engine.lanes_desc(theta, 0, table, idx, sign, 0.02)
    nwg = args.lanes * args.envs
    dbg = torch.zeros(256 + 4 * nwg, dtype=torch.int64).cuda()
    ctx = engine.context()
    spec = engine.ImpalaSpec(A, args.envs, 2, entropy=False, fp16=True)
    engine.impala_rollout(spec, lanes, args.lanes, 1)  # warm
    for rep in range(args.reps):
        ctx.impala_debug_clock(dbg)
        engine.impala_rollout(spec, lanes, args.lanes, 1)
        torch.cuda.synchronize()
        ctx.impala_debug_clock(None)
        # the conv of step 0 and step 1 both write: the last launch's values remain (T = 2: the second conv launch)
        c = dbg.cpu().numpy()[256:].reshape(nwg, 4)
        t0, t1 = c[:, 0].astype(np.int64), c[:, 1].astype(np.int64)
        hw, xcc = c[:, 2].astype(np.int64), c[:, 3].astype(np.int64)
        ok = (t0 > 0) & (t1 > t0)
        dur = (t1 - t0)[ok] * 10.0  # ns
        span = (t1[ok].max() - t0[ok].min()) * 10.0
        cu = ((hw >> 8) & 0xF) | (((hw >> 13) & 0x7) << 4) | (((hw >> 12) & 1) << 7)  # cu_id | se_id | sh_id
        key = (xcc & 0xF) * 256 + cu
        per = collections.defaultdict(list)
        for i in np.nonzero(ok)[0]:
            per[int(key[i])].append((int(t0[i]), int(t1[i])))
        counts = np.array([len(v) for v in per.values()])
        busy_end = np.array([max(e for _, e in v) for v in per.values()])
        start = t0[ok].min()
        # per CU: time-average number of resident workgroups over [start, that CU's last end]
        occ = []
        for v in per.values():
            tot = sum(e - s for s, e in v)
            occ.append(tot / max(1, max(e for _, e in v) - start))
        print("rep %d: %d workgroups on %d CUs; launch span %.1f us; WG life mean %.1f us (min %.1f, p50 %.1f, p90 %.1f, "
              "max %.1f); WGs per CU %d..%d (mean %.2f); CU finish %.1f..%.1f us; mean resident WGs per CU %.2f" % (
                  rep, ok.sum(), len(per), span / 1e3, dur.mean() / 1e3, dur.min() / 1e3, np.median(dur) / 1e3,
                  np.percentile(dur, 90) / 1e3, dur.max() / 1e3, counts.min(), counts.max(), counts.mean(),
                  (busy_end.min() - start) * 1e-2, (busy_end.max() - start) * 1e-2, float(np.mean(occ))))
        # life by dispatch round (order of start on each CU)
        rounds = collections.defaultdict(list)
        for v in per.values():
            for r, (s, e) in enumerate(sorted(v)):
                rounds[r].append((e - s) * 1e-2)
        print("   life by start order on the CU (us): " + " ".join(
            "%d:%.1f" % (r, np.mean(rounds[r])) for r in sorted(rounds)))


if __name__ == "__main__":
    main()
