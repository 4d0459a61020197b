#!/bin/bash
# r07e: SrcC wait-state sweep; A/B of conv_kernel_h2 stagger variants (conv ms per launch, HIP events), ABAB order.
set -u
mkdir -p gpurun_out
timeout -k 10 60 ./tools/probes/srcc_probe > gpurun_out/r07e_srcc.txt 2>&1 || { echo "probe rc=$?"; exit 3; }
cat gpurun_out/r07e_srcc.txt
for round in 1 2; do
  RUNS="libfdr libfdr_stag32000 libfdr_stag64000" CONFIGS="impala_fp16" T=60 bash tools/ab_impala.sh || exit 3
done
