"""Phase clocks of conv_kernel_h2 (fdr_impala_debug_clock: s_memtime of workgroup 0 at each barrier).

    make -C dfd-starter_amd/csrc STAMPS=1 OUT=../fdr/libfdr_stamps.so OBJDIR=../../build/obj_stamps
    FDR_LIB=$PWD/dfd-starter_amd/fdr/libfdr_stamps.so python tools/impala_phases_h2.py [--lanes 1024 --envs 4]

(The stamps are compiled only into that diagnostics build: in the product even runtime-gated stamps drained the
loads in flight at every phase boundary.)

Workgroup 0 shares its CU with a second workgroup for the whole launch (2 per CU), so a phase's clocks
include the issue slots the other workgroup takes."""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "dfd-starter_amd"))
from fdr import engine  # noqa: E402


def names(h3=False):
    n = {1: "bn table", 18: "stage1 bn -> padded", 36: "stage2 bn -> padded", 49: "stage3 bn -> padded"}
    if h3:  # in-register pool entries: one stamp per band (conv + pool + exchange + X store), one after the stage
        for st, base, nb in ((1, 2, 4), (2, 28, 2), (3, 45, 1)):
            for b in range(nb):
                n[base + b] = "stage%d band%d conv+pool" % (st, b)
            n[base + nb] = "stage%d entry end" % st
    else:
        for st, base, nb in ((1, 2, 8), (2, 28, 4), (3, 45, 2)):
            for b in range(nb):
                n[base + 2 * b] = "stage%d band%d conv" % (st, b)
                n[base + 2 * b + 1] = "stage%d band%d pool" % (st, b)
    for st, base in ((1, 19), (2, 37), (3, 50)):
        for r in range(2):
            for k, what in enumerate(("conv0", "epilogue0", "conv1", "epilogue1")):
                n[base + 4 * r + k] = "stage%d res%d %s" % (st, r, what)
    return n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lanes", type=int, default=1024)
    ap.add_argument("--envs", type=int, default=4)
    args = ap.parse_args()
    A = 4
    P = engine.impala_num_params(A)
    torch.manual_seed(0)
    theta = (torch.randn(P) * 0.02).cuda()
    table = torch.randn(P + 4096).cuda()
    idx = torch.randint(0, 4096, (args.lanes,), dtype=torch.int64).cuda()
    sign = torch.ones(args.lanes, dtype=torch.int8).cuda()
    lanes = engine.lanes_desc(theta, 0, table, idx, sign, 0.02)
    dbg = torch.zeros(128, dtype=torch.int64).cuda()
    ctx = engine.context()
    ctx.impala_debug_clock(dbg)
    spec = engine.ImpalaSpec(A, args.envs, 2, entropy=False, fp16=True)
    engine.impala_rollout(spec, lanes, args.lanes, 1)
    torch.cuda.synchronize()
    ctx.impala_debug_clock(None)
    c = dbg.cpu().numpy().astype(np.int64)
    n = names(h3=True)
    order = [0] + sorted(k for k in n if c[k] != 0)  # the 4-wave kernel has one stage-3 band
    tot = c[order[-1]] - c[0]
    print("conv_kernel_h2 workgroup 0: %d clocks total" % tot)
    groups = {}
    for a, b in zip(order[:-1], order[1:]):
        d = int(c[b] - c[a])
        print("%-28s %9d  %5.1f%%" % (n[b], d, 100.0 * d / tot))
        key = " ".join(w for w in n[b].split() if not w.startswith(("band", "res")) or True)
        kind = n[b].split()[-1]
        groups[kind] = groups.get(kind, 0) + d
    if c[64:].any():  # FDR_H3_FINE build: inside the entry bands (relative to the band's start)
        for b in range(4):
            t0 = c[1] if b == 0 else c[1 + b]
            print("stage1 band%d: conv issued %d, frame %d, pool %d, exchange+barrier+X %d" % (
                b, c[64 + 4 * b] - t0, c[65 + 4 * b] - c[64 + 4 * b], c[66 + 4 * b] - c[65 + 4 * b], c[2 + b] - c[66 + 4 * b]))
        for b in range(2):
            t0 = c[28 + b - 1] if b > 0 else max(c[k] for k in range(19, 27))
            print("stage2 band%d: conv %d, pool %d, exchange+barrier+X %d" % (
                b, c[80 + 4 * b] - t0, c[81 + 4 * b] - c[80 + 4 * b], c[28 + b] - c[81 + 4 * b]))
    print("by kind:", ", ".join("%s %d (%.1f%%)" % (k, v, 100.0 * v / tot) for k, v in sorted(groups.items(), key=lambda x: -x[1])))


if __name__ == "__main__":
    main()
