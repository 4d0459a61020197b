"""Per-step kernel durations and the idle gaps between them, from a rocprofv3 --kernel-trace CSV
(run_kernel_trace.csv): the median of each (kernel, gap-before) over the last N dispatches of the dominant cycle.
    python tools/trace_gaps.py gpurun_out/x/run_kernel_trace.csv [last_n]"""
import collections
import csv
import sys

import numpy as np


def main(path, last=200):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))[-int(last):]
    dur = collections.defaultdict(list)
    gap = collections.defaultdict(list)
    prev = None
    for r in rows:
        s, e, k = int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:60]
        dur[k].append((e - s) / 1e3)
        if prev is not None:
            gap[k].append((s - prev) / 1e3)
        prev = e
    for k in dur:
        print("%-60s n %4d  dur %9.2f us  gap before %7.2f us (median)" % (k, len(dur[k]), np.median(dur[k]),
                                                                         np.median(gap[k]) if gap[k] else 0))


if __name__ == "__main__":
    main(*sys.argv[1:])
