#!/bin/bash
# r08h: deeper fragment prefetch in the streamed convs (conv_h2 / conv_band_nat PD): parity + A/B
# libfdr_pd1: every PD = 1 (r08g build); libfdr_pdres: residual convs only; libfdr: residual + entry bands.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_impala.py tests/test_gpu_impala_novelty.py \
  > gpurun_out/r08h_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/r08h_tests.log; exit 3; }
tail -1 gpurun_out/r08h_tests.log
RUNS="libfdr_pd1 libfdr_pdres libfdr libfdr_pd1 libfdr_pdres libfdr" CONFIGS="impala_fp16" T=60 bash tools/ab_impala.sh || exit 3
timeout -k 10 120 python tools/impala_phases_h2.py --mode 2 > gpurun_out/r08h_phases.txt 2>&1 || exit 3
echo r08h done
