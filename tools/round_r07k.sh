#!/bin/bash
# r07k: in-register-pool stage entries (FDR_H3_ENTRY) -- bit identity vs conv_kernel_h, fp16 parity, phases, A/B vs the
# banded-S entries (libfdr_old = FDR_H3_ENTRY=0).
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_impala.py -k "h2" \
  > gpurun_out/r07k_tests.log 2>&1 || { echo "tests rc=$?"; tail -40 gpurun_out/r07k_tests.log; exit 3; }
tail -1 gpurun_out/r07k_tests.log
timeout -k 10 120 python -u tools/impala_phases_h2.py --mode 2 > gpurun_out/r07k_phases0.txt 2>&1 && FDR_LIB=$PWD/dfd-starter_amd/fdr/libfdr_fine.so timeout -k 10 120 python -u tools/impala_phases_h2.py --mode 2 > gpurun_out/r07k_phases.txt 2>&1 || { echo "phases rc=$?"; tail gpurun_out/r07k_phases.txt; exit 3; }
tail -3 gpurun_out/r07k_phases0.txt; cat gpurun_out/r07k_phases.txt
RUNS="libfdr libfdr_old libfdr libfdr_old" CONFIGS="impala_fp16" T=60 bash tools/ab_impala.sh || exit 3
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_impala.py \
  tests/test_gpu_impala_novelty.py -k "fp16 or strateg or forward" > gpurun_out/r07k_tests2.log 2>&1 \
  || { echo "tests2 rc=$?"; tail -30 gpurun_out/r07k_tests2.log; exit 3; }
tail -1 gpurun_out/r07k_tests2.log
