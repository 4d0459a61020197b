"""Summarise a tools/profile.sh output directory into profiles/<tag>_summary.md + the PMC json
bench.py reads (profiles/pmc_rollout_<config>.json).

    python tools/summarize_prof.py gpurun_out/prof_r01 r01 [config [kernel-substring [secondary [T]]]]

HBM bytes per launch = FETCH_SIZE*1024*2 + WRITE_SIZE*1024: MI355X_MICROARCH.md section HBM --
on gfx950 FETCH_SIZE reports half of a wide coalesced read; that x2 correction is applied to the
read side, and the raw counters are kept beside it (other access widths are uncalibrated).
"""
import collections
import csv
import json
import os
import sys


def per_kernel(path, counter=None):
    out = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if counter is None or r.get("Counter_Name") == counter:
            out[r["Kernel_Name"]].append(r)
    return out


def mfma_pass(d):
    """Per-kernel averages of the optional MFMA PMC pass (MFMA_PMC in tools/profile.sh)."""
    path = os.path.join(d, "pmc_mfma", "run_counter_collection.csv")
    if not os.path.exists(path):
        return {}
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(path)):
        acc[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in q.items()} for k, q in acc.items()}


def main(d, tag, config="halfcheetah", dominant="rollout_kernel", secondary=None, steps="1000"):
    steps = int(steps)  # env steps per launch of the dominant kernel (per-wave-step counts)
    stats = list(csv.DictReader(open(os.path.join(d, "trace", "run_kernel_stats.csv"))))
    fetch = per_kernel(os.path.join(d, "pmc_fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    write = per_kernel(os.path.join(d, "pmc_write", "run_counter_collection.csv"), "WRITE_SIZE")
    sq = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(os.path.join(d, "pmc_sq", "run_counter_collection.csv"))):
        sq[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    lines = ["# rocprofv3 summary -- %s (bench.py config %s, 1x MI355X)" % (tag, config), "",
             "Kernel stats (`rocprofv3 --kernel-trace --stats`):", "",
             "| kernel | calls | total ms | avg us | pct |", "|---|---|---|---|---|"]
    for s in stats:
        lines.append("| %s | %s | %.3f | %.2f | %.1f |" % (s["Name"][:70], s["Calls"], float(s["TotalDurationNs"]) / 1e6,
                                                          float(s["AverageNs"]) / 1e3, float(s["Percentage"])))
    lines += ["", "PMC (separate passes, averaged over dispatches):", "",
              "| kernel | FETCH_SIZE KB | WRITE_SIZE KB | HBM bytes/launch (fetch x2 + write) | SQ_INSTS_VALU | "
              "SQ_INSTS_LDS | SQ_WAVES | GRBM_GUI_ACTIVE |", "|---|---|---|---|---|---|---|---|"]
    rollout = None
    for k in fetch:
        f = sum(float(r["Counter_Value"]) for r in fetch[k]) / len(fetch[k])
        w = sum(float(r["Counter_Value"]) for r in write.get(k, [])) / max(1, len(write.get(k, [])))
        hbm = f * 1024 * 2 + w * 1024
        q = {c: sum(v) / len(v) for c, v in sq.get(k, {}).items()}
        lines.append("| %s | %.1f | %.1f | %.0f | %.0f | %.0f | %.0f | %.0f |" % (
            k[:70], f, w, hbm, q.get("SQ_INSTS_VALU", 0), q.get("SQ_INSTS_LDS", 0), q.get("SQ_WAVES", 0),
            q.get("GRBM_GUI_ACTIVE", 0)))
        if dominant in k:
            rollout = dict(kernel=k, fetch_size_kb=f, write_size_kb=w, hbm_bytes_per_launch=hbm, sq=q)
    if rollout:
        st = [s for s in stats if dominant in s["Name"]][0]
        avg_ns = float(st["AverageNs"])
        q = rollout["sq"]
        clk = q.get("GRBM_GUI_ACTIVE", 0) / 8 / (avg_ns * 1e-9) / 1e9 if avg_ns else 0
        rollout["avg_duration_us"] = avg_ns / 1e3
        rollout["effective_clock_ghz"] = clk
        # steady state: the last half of the dispatches (the clocks ramp over the first ~30 ms of load)
        tr = os.path.join(d, "trace", "run_kernel_trace.csv")
        if os.path.exists(tr):
            durs = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
                    for r in csv.DictReader(open(tr)) if r["Kernel_Name"] == st["Name"]]
            durs = [x for _, x in sorted(durs)]
            if durs:
                tail = durs[len(durs) // 2:]
                rollout["avg_duration_us_steady"] = sum(tail) / len(tail) / 1e3
                rollout["dispatches"] = len(durs)
        lines += ["", "Dominant kernel (%s): avg %.1f us, effective clock %.2f GHz (GRBM_GUI_ACTIVE/8/duration), "
                      "VALU instructions per wave-step %.1f, LDS per wave-step %.1f." % (
                          dominant, avg_ns / 1e3, clk, q.get("SQ_INSTS_VALU", 0) / max(1, q.get("SQ_WAVES", 1)) / steps,
                          q.get("SQ_INSTS_LDS", 0) / max(1, q.get("SQ_WAVES", 1)) / steps)]
        if "avg_duration_us_steady" in rollout:
            lines += ["", "Steady state (last %d of %d dispatches, after the clock ramp): avg %.1f us." % (
                rollout["dispatches"] - rollout["dispatches"] // 2, rollout["dispatches"],
                rollout["avg_duration_us_steady"])]
        mf = mfma_pass(d)
        if mf:
            lines += ["", "MFMA pass (SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE/8); MOPS x 512 = FLOP):", "",
                      "| kernel | MFMA busy | MFMA FLOP executed (F32 + F16 MOPS x 512) | clock GHz |", "|---|---|---|---|"]
            for k, q in mf.items():
                cyc = q.get("GRBM_GUI_ACTIVE", 0) / 8
                busy = q.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (1024 * cyc) if cyc else 0
                flop = 512 * (q.get("SQ_INSTS_VALU_MFMA_MOPS_F32", 0) + q.get("SQ_INSTS_VALU_MFMA_MOPS_F16", 0))
                st = [x for x in stats if x["Name"] == k]
                clk = cyc / (float(st[0]["AverageNs"]) * 1e-9) / 1e9 if st else 0
                lines.append("| %s | %.3f | %.3e | %.2f |" % (k[:70], busy, flop, clk))
                if dominant in k:
                    rollout["mfma_busy"] = round(busy, 4)
                    rollout["mfma_flop_per_launch"] = flop
        ex = os.path.join(d, "pmc_extra0", "run_counter_collection.csv")
        if os.path.exists(ex):  # issue / wait breakdown (tools/profile_round.sh ISSUE_PMC)
            acc = collections.defaultdict(list)
            for r in csv.DictReader(open(ex)):
                if r["Kernel_Name"] == rollout["kernel"]:
                    acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
            q = {c: sum(v) / len(v) for c, v in acc.items()}
            if q.get("SQ_WAVE_CYCLES") and q.get("GRBM_GUI_ACTIVE"):
                cyc = q["GRBM_GUI_ACTIVE"] / 8
                simds = 1024
                issue = dict(counters=q,
                             simd_valu_busy=q["SQ_ACTIVE_INST_VALU"] / (simds * cyc / 4),
                             cycles_per_valu_inst=(q["SQ_ACTIVE_INST_VALU"] * 4 / rollout["sq"]["SQ_INSTS_VALU"]
                                                   if rollout["sq"].get("SQ_INSTS_VALU") else None),
                             wave_frac_active=q["SQ_ACTIVE_INST_ANY"] / q["SQ_WAVE_CYCLES"],
                             wave_frac_wait_any=q["SQ_WAIT_ANY"] / q["SQ_WAVE_CYCLES"],
                             wave_frac_wait_inst=q["SQ_WAIT_INST_ANY"] / q["SQ_WAVE_CYCLES"],
                             wave_frac_wait_inst_lds=(q["SQ_WAIT_INST_LDS"] / q["SQ_WAVE_CYCLES"]
                                                      if "SQ_WAIT_INST_LDS" in q else None))
                rollout["issue"] = issue
                lines += ["", "Issue / wait PMC pass (quad-cycle SQ counters; SIMD VALU busy = SQ_ACTIVE_INST_VALU / "
                              "(1024 SIMDs x GRBM_GUI_ACTIVE/8 / 4)): VALU busy %.3f, %.2f cycles per VALU instruction; "
                              "wave cycles: %.1f %% issuing, %.1f %% waiting on counters, %.1f %% issue-stalled "
                              "(of which LDS issue %.1f %%)." % (
                                  issue["simd_valu_busy"], issue["cycles_per_valu_inst"] or 0,
                                  100 * issue["wave_frac_active"], 100 * issue["wave_frac_wait_any"],
                                  100 * issue["wave_frac_wait_inst"], 100 * (issue["wave_frac_wait_inst_lds"] or 0))]
        if secondary:
            for k in fetch:
                if secondary in k:
                    f = sum(float(r["Counter_Value"]) for r in fetch[k]) / len(fetch[k])
                    w = sum(float(r["Counter_Value"]) for r in write.get(k, [])) / max(1, len(write.get(k, [])))
                    st = [x for x in stats if x["Name"] == k]
                    rollout["core_kernel"] = dict(kernel=k, fetch_size_kb=f, write_size_kb=w,
                                                  hbm_bytes_per_launch=f * 1024 * 2 + w * 1024,
                                                  avg_duration_us=float(st[0]["AverageNs"]) / 1e3 if st else None)
                    lines += ["", "Secondary kernel %s: HBM bytes/launch %.0f (FETCH x2 + WRITE), avg %.1f us" % (
                        k[:70], f * 1024 * 2 + w * 1024, rollout["core_kernel"]["avg_duration_us"] or 0)]
                    break
        with open(os.path.join("profiles", "pmc_rollout_%s.json" % config), "w") as fh:
            json.dump(dict(rollout, source=d, tag=tag), fh, indent=1)
    with open(os.path.join("profiles", "%s_summary.md" % tag), "w") as fh:
        fh.write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main(*sys.argv[1:])
