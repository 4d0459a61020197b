#!/bin/bash
# Kernel-trace of config 5 (short episode) per fp16 conv mode; prints per-kernel medians of the rollout-size launches.
# Usage (GPU box): MODES="2 3" bash tools/prof_conv_modes.sh -> gpurun_out/prof_m<mode>/
set -u
export TMPDIR=/tmp
for m in ${MODES:-2 3}; do
  mkdir -p gpurun_out/prof_m$m
  FDR_CONV_H2=$m timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/prof_m$m -o run -- python3 bench.py \
    --config impala_fp16 --steps 1 --warmup 1 --episode-len ${T:-40} --no-cpu-baseline > gpurun_out/prof_m$m.log 2>&1 \
    || { echo "mode $m failed"; tail -5 gpurun_out/prof_m$m.log; exit 3; }
  python3 tools/rocpd_medians.py gpurun_out/prof_m$m/run_results.db conv_kernel_h2 conv_s3 core_kernel_hpm
done
