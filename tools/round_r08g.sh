#!/bin/bash
# r08g: the pair core's sigma-eps from the f16 sigma * table copy (core_table) and the chained K = 32 tap-8 remainder
# of conv_kernel_h2<512> (FDR_R32): parity, A/B (libfdr_cur: neither; libfdr_r32off: table only; libfdr: both).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2; do
  echo "-- images, R32 off"; FDR_CORE_TABLE=0 RUNS="libfdr_r32off" CONFIGS="impala_fp16" T=60 bash tools/ab_impala.sh || exit 3
  echo "-- table, R32 off"; RUNS="libfdr_r32off" CONFIGS="impala_fp16" T=60 bash tools/ab_impala.sh || exit 3
  echo "-- table, R32 on"; RUNS="libfdr" CONFIGS="impala_fp16" T=60 bash tools/ab_impala.sh || exit 3
done
timeout -k 10 400 python -u bench.py --config impala_fp16 --steps 2 --warmup 1 > gpurun_out/r08g_bench_impala_fp16.log 2>&1 || exit 3
tail -1 gpurun_out/r08g_bench_impala_fp16.log | cut -c1-300
echo r08g done
