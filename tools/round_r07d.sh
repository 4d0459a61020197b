#!/bin/bash
# r07d: SrcC chaining -- the probe with a truly back-to-back K=32 -> K=16 pair, and the conv built with the
# chained remainder (libfdr_chain.so) against the fp16 reference golden / oracle tests.
set -u
mkdir -p gpurun_out
timeout -k 10 60 ./tools/probes/srcc_probe > gpurun_out/r07d_srcc.txt 2>&1 || { echo "probe rc=$?"; cat gpurun_out/r07d_srcc.txt; exit 3; }
cat gpurun_out/r07d_srcc.txt
FDR_LIB=$PWD/dfd-starter_amd/fdr/libfdr_chain.so timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread \
  tests/test_gpu_impala.py -k "fp16_forward or fp16_rollout_first or drift or whole_episode" > gpurun_out/r07d_chain_tests.log 2>&1
echo "chain tests rc=$?"
grep -E "PASSED|FAILED|Error|assert" gpurun_out/r07d_chain_tests.log | head -20
