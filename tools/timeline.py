"""Print the GPU timeline (kernel trace) of the last K FD steps of a rocprofv3 --kernel-trace run:
    python tools/timeline.py gpurun_out/prof_x/run_kernel_trace.csv [marker-substring] [K]"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
marker = sys.argv[2] if len(sys.argv) > 2 else "rollout"
k = int(sys.argv[3]) if len(sys.argv) > 3 else 3
idx = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
first = idx[-k - 1] if len(idx) > k else 0
prev_end = None
for r in rows[first:]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = "" if prev_end is None else "%8.2f" % ((s - prev_end) / 1e3)
    print("%-60s dur %9.2f us  gap-before %s" % (r["Kernel_Name"][:60], (e - s) / 1e3, gap))
    prev_end = e
