#!/bin/bash
# A/B of rollout-kernel builds (GPU box): evaluate() time per build and config, then the GPU parity
# tests against the last build.  Usage: bash tools/ab_rollout.sh libfdr libfdr_v1 ...
set -u
mkdir -p gpurun_out
last=""
for v in "$@"; do
  for c in halfcheetah cartpole; do
    FDR_LIB=$PWD/dfd-starter_amd/fdr/$v.so timeout -k 10 120 python tools/rollout_phases.py --config $c --iters 15 \
      > gpurun_out/ab_${v}_${c}.log 2>&1 || { echo "$v $c FAIL rc=$?"; tail -5 gpurun_out/ab_${v}_${c}.log; exit 3; }
    echo "$v $c: $(grep evaluate gpurun_out/ab_${v}_${c}.log)"
  done
  last=$v
done
if [ -n "${PARITY:-}" ]; then
  FDR_LIB=$PWD/dfd-starter_amd/fdr/$last.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 \
    --timeout-method thread > gpurun_out/ab_parity.log 2>&1; rc=$?
  echo "parity ($last) rc=$rc"; tail -5 gpurun_out/ab_parity.log
fi
