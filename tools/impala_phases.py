"""Phase breakdown of the Impala conv kernel (s_memtime clocks of workgroup 0, fdr_impala_debug_clock).

    python tools/impala_phases.py [--lanes 1024 --envs 4]
"""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "dfd-starter_amd"))
from fdr import engine  # noqa: E402
from fdr._lib import lib  # noqa: E402

NAMES = {0: "start", 1: "bn table + zero", 2: "frame"}
for st, pre, k0 in ((1, 2, 4), (2, 12, 14), (3, 22, 24)):
    NAMES[pre + 1] = "stage%d entry conv+pool+bn" % st
    for r in range(2):
        NAMES[k0 + 4 * r] = "stage%d res%d (launch)" % (st, r) if r == 0 else "stage%d res0 conv1 epilogue" % st
        NAMES[k0 + 4 * r + 1] = "stage%d res%d conv0" % (st, r)
        NAMES[k0 + 4 * r + 2] = "stage%d res%d epilogue0" % (st, r)
        NAMES[k0 + 4 * r + 3] = "stage%d res%d conv1" % (st, r)
NAMES[12] = "stage1 res1 conv1 epilogue"
NAMES[22] = "stage2 res1 conv1 epilogue"
NAMES[32] = "stage3 res1 conv1 epilogue (features)"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lanes", type=int, default=1024)
    ap.add_argument("--envs", type=int, default=4)
    ap.add_argument("--fp16", action="store_true")
    args = ap.parse_args()
    A = 6
    P = engine.impala_num_params(A)
    torch.manual_seed(0)
    theta = (torch.randn(P) * 0.02).cuda()
    table = torch.randn(P + 4096).cuda()
    idx = torch.randint(0, 4096, (args.lanes,), dtype=torch.int64).cuda()
    sign = torch.ones(args.lanes, dtype=torch.int8).cuda()
    lanes = engine.lanes_desc(theta, 0, table, idx, sign, 0.02)
    dbg = torch.zeros(64, dtype=torch.int64).cuda()
    engine.context().impala_debug_clock(dbg)
    spec = engine.ImpalaSpec(A, args.envs, 2, entropy=False, fp16=args.fp16)
    engine.impala_rollout(spec, lanes, args.lanes, 1)
    torch.cuda.synchronize()
    engine.context().impala_debug_clock(None)
    c = dbg.cpu().numpy().astype(np.int64)
    tot = c[32] - c[0]
    order = sorted(NAMES)
    print("conv workgroup 0: %d clocks total" % tot)
    for a, b in zip(order[:-1], order[1:]):
        print("%-28s %9d  %5.1f%%" % (NAMES[b], c[b] - c[a], 100.0 * (c[b] - c[a]) / tot))
    if not args.fp16:  # f32 kernel: entry conv / pool clocks summed over the bands
        for st, k0 in enumerate((40, 48, 56)):
            print("  stage%d entry: conv %7d  pool %7d" % (st + 1, c[k0], c[k0 + 1]))
    if args.fp16:  # entry-conv bands (fp16 kernel): conv + store, then pool, per band
        for st, (k0, start, end, nb) in enumerate(((40, 2, 3, 2), (48, 12, 13, 2), (56, 22, 23, 1))):
            prev = c[start]
            for b in range(nb):
                cv, pl = c[k0 + 2 * b], c[k0 + 2 * b + 1]
                print("  stage%d band%d: conv %7d  pool %7d" % (st + 1, b, cv - prev, pl - cv))
                prev = pl
            print("  stage%d bn+relu to padded: %7d" % (st + 1, c[end] - prev))


if __name__ == "__main__":
    main()
