#!/bin/bash
# A/B of the rollout implementations (FDR_ROLLOUT=single|pair) on the GPU box, then the GPU parity
# tests on the default build.  Stops at the first fault / timeout.
set -u
mkdir -p gpurun_out
FAULT='HSA_STATUS_ERROR|illegal memory access|Memory access fault|hipErrorIllegalAddress'
# RUNS: space-separated <lib>:<impl> pairs (lib = file stem under dfd-starter_amd/fdr/)
for run in ${RUNS:-libfdr:single libfdr:pair libfdr:single libfdr:pair}; do
  lib=${run%%:*}; impl=${run##*:}
  for c in ${CONFIGS:-halfcheetah cartpole}; do
    log=gpurun_out/ab_${lib}_${impl}_${c}.log
    FDR_LIB=$PWD/dfd-starter_amd/fdr/$lib.so FDR_ROLLOUT=$impl timeout -k 10 120 \
      python tools/rollout_phases.py --config $c --iters 15 ${PHASE_ARGS:-} > $log 2>&1; rc=$?
    if [ $rc -ne 0 ] || grep -qE "$FAULT" $log; then
      echo "$lib $impl $c FAIL rc=$rc"; tail -5 $log; exit 3; fi
    echo "$lib $impl $c: $(grep evaluate $log)"
  done
done
if [ -z "${NO_PARITY:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/ab_parity.log 2>&1; rc=$?
  echo "parity rc=$rc"; tail -8 gpurun_out/ab_parity.log
fi
