"""LDS / VALU utilisation of one kernel from a rocprofv3 --pmc pass (the SQ_LDS_* counter set of a separate --pmc pass).
    python tools/pmc_lds.py <run_counter_collection.csv> [kernel-substring] [envs per launch]"""
import collections
import csv
import statistics
import sys

path = sys.argv[1]
ksub = sys.argv[2] if len(sys.argv) > 2 else "conv_kernel_h2"
envs = int(sys.argv[3]) if len(sys.argv) > 3 else 4096
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(path)):
    if ksub in r["Kernel_Name"]:
        acc[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
vals = collections.defaultdict(list)
for v in acc.values():
    for c, x in v.items():
        vals[c].append(x)
m = {c: statistics.mean(v) for c, v in vals.items()}
clk = m["GRBM_GUI_ACTIVE"] / 8  # per XCD
print("%d dispatches, %.0f clocks per launch" % (len(acc), clk))
if "SQ_LDS_IDX_ACTIVE" in m:
    print("LDS busy per CU %.3f; bank-conflict cycles %.3f of LDS cycles; LDS cycles per env %.0f (conflict %.0f); "
          "LDS wave-instructions per env %.0f" % (
              m["SQ_LDS_IDX_ACTIVE"] / 256 / clk, m["SQ_LDS_BANK_CONFLICT"] / m["SQ_LDS_IDX_ACTIVE"],
              m["SQ_LDS_IDX_ACTIVE"] / envs, m["SQ_LDS_BANK_CONFLICT"] / envs, m.get("SQ_INSTS_LDS", 0) / envs))
if "SQ_ACTIVE_INST_VALU" in m:  # SQ wave counters count quad-cycles
    print("VALU active per SIMD %.3f" % (4 * m["SQ_ACTIVE_INST_VALU"] / 1024 / clk))
