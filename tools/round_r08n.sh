#!/bin/bash
# r08n: stage-1 band conv in a K order of horizontally adjacent tap pairs (one 16-byte B read per K-step, no operand
# assembly moves): parity + A/B against the previous build (libfdr_prev).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_impala.py tests/test_gpu_impala_novelty.py \
  > gpurun_out/r08n_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/r08n_tests.log; exit 3; }
tail -1 gpurun_out/r08n_tests.log
RUNS="libfdr_prev libfdr libfdr_prev libfdr libfdr_prev libfdr" CONFIGS="impala_fp16" T=60 bash tools/ab_impala.sh || exit 3
echo r08n done
