#!/bin/bash
# Same-box A/B of library builds through bench.py: alternating runs of each lib (file stems under
# dfd-starter_amd/fdr/), one line per run with the step and rollout times.  Stops at the first failure.
#   LIBS="libfdr libfdr_variant" CONFIGS="cartpole" ROUNDS=3 BENCH_ARGS="--steps 50" bash tools/ab_bench.sh
set -u
mkdir -p gpurun_out
FAULT='HSA_STATUS_ERROR|illegal memory access|Memory access fault|hipErrorIllegalAddress'
for r in $(seq 1 ${ROUNDS:-3}); do
  for lib in ${LIBS:-libfdr}; do
    for c in ${CONFIGS:-halfcheetah}; do
      log=gpurun_out/abb_${lib}_${c}_$r.log
      FDR_LIB=$PWD/dfd-starter_amd/fdr/$lib.so timeout -k 10 300 python bench.py --config $c --no-cpu-baseline \
        --no-variant ${BENCH_ARGS:-} > $log 2>&1; rc=$?
      if [ $rc -ne 0 ] || grep -qE "$FAULT" $log; then echo "$lib $c FAIL rc=$rc"; tail -5 $log; exit 3; fi
      python - "$lib" "$c" "$log" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[3]) if l.startswith("{")][-1])
rf = d.get("roofline") or {}
print("%-22s %-12s value %.4g  ms/step %.4f  rollout_ms %s  frac %s" % (sys.argv[1], sys.argv[2], d["value"],
      d["ms_per_step"], rf.get("rollout_ms"), rf.get("frac")))
PY
    done
  done
done
