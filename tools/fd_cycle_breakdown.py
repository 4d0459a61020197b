"""Per-FD-step GPU time by phase from a rocprofv3 --kernel-trace CSV of bench.py --config impala_fp16: every cycle
between two rollouts' finish_kernel, with busy / idle time and the kernels grouped (conv, core step, entropy replay,
lane strategies, other).
    python tools/fd_cycle_breakdown.py gpurun_out/x/run_kernel_trace.csv"""
import collections
import csv
import sys


def phase(k):
    if "conv_kernel" in k:
        return "conv"
    if "core_kernel_hpm2<4, 0>" in k or "core_kernel_hpm2<2, 0>" in k or "core_kernel_hpm2<1, 0>" in k:
        return "core"
    if "hpm2<4, 1>" in k or "hpm2<2, 1>" in k or "xproj_pair_kernel<4" in k:
        return "replay"
    if "<1, 3>" in k or "fc_rows" in k or "lstm_xproj" in k or "xproj_pair_kernel<1" in k:
        return "strategies"
    return "other"


def main(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    fin = [i for i, r in enumerate(rows) if "finish_kernel" in r["Kernel_Name"]]
    for a, b in zip(fin, fin[1:]):
        t0, t1 = int(rows[a]["End_Timestamp"]), int(rows[b]["End_Timestamp"])
        agg = collections.defaultdict(float)
        busy = 0
        for i in range(a + 1, b + 1):
            d = int(rows[i]["End_Timestamp"]) - int(rows[i]["Start_Timestamp"])
            busy += d
            agg[phase(rows[i]["Kernel_Name"])] += d / 1e6
        print("cycle %5d -> %5d: span %8.2f ms  busy %8.2f  idle %6.2f  " % (a, b, (t1 - t0) / 1e6, busy / 1e6,
                                                                           (t1 - t0 - busy) / 1e6)
              + "  ".join("%s %.2f" % kv for kv in sorted(agg.items())))


if __name__ == "__main__":
    main(*sys.argv[1:])
